// sdr_internal.h -- declarations shared by the translation units of libsdr_amd.so (not installed).
//
//   sdr_frontend.hip   u8 I/Q -> 101-tap FIR /D on I and Q -> discriminator   rffrontend.cpp:58-71
//   sdr_pll.hip        PLL / NCO recurrences, persistent PLL hand-offs        pll.cpp:4-61
//   sdr_kernels.hip    IF FIRs, resamplers, mixers, RDS bits, context and the C ABI
//
// Layout: channel-major [nch][len]. Every f32 stream that a later FIR/resampler reads with
// look-back is kept "extended": [2 parities][nch][HIST + len], the first HIST samples being the
// previous block's last HIST samples, so a kernel reads x[-HIST..len) with no branch; the
// producer of block b copies the history from the parity of block b-1.
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <vector>

#include "sdr_amd.h"

#define SDRK_HIDDEN __attribute__((visibility("hidden")))

namespace sdrk SDRK_HIDDEN {

constexpr int HIST = 160;        // history samples in front of every extended f32 stream (>= 150)
constexpr int BLK = 256;         // threads per workgroup for the streaming kernels
constexpr int FIR_TILE = 512;    // outputs per workgroup for the 101-tap FIRs
constexpr int DEC_STATE = 8;     // ints of RDS decoder state per channel

// MFMA front end (sdr_frontend.hip): digit planes of the fixed-point taps and tap fragments
constexpr int FT_ND = 4;
constexpr int FT_AFRAGS = 4 * FT_ND;
constexpr int FT_NB = 32;        // 16-output blocks per wave tile (16, 48, 64: slower, profiles/r05/mfma_tile_ab.txt)

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef int v4i __attribute__((ext_vector_type(4)));

// sets the thread's last-error text (sdr_last_error) and returns code
int fail(int code, const char* fmt, ...);

#define HIP_TRY(expr)                                                                       \
    do {                                                                                    \
        hipError_t e_ = (expr);                                                             \
        if (e_ != hipSuccess) return ::sdrk::fail(SDR_E_HIP, "%s: %s", #expr, hipGetErrorString(e_)); \
    } while (0)

#define LAUNCH_CHECK()                                                                              \
    do {                                                                                            \
        hipError_t e_ = hipGetLastError();                                                          \
        if (e_ != hipSuccess) return ::sdrk::fail(SDR_E_HIP, "launch failed at %s:%d: %s", __FILE__, __LINE__, \
                                                  hipGetErrorString(e_));                           \
    } while (0)

inline int cdiv(int a, int b) { return (a + b - 1) / b; }
inline size_t round_up(size_t a, size_t b) { return (a + b - 1) / b * b; }

// One PLL instance over nch channels (pll.cpp:4 arguments). A launch runs up to 2 of them
// (blockIdx.y), so the stereo (19 kHz) and RDS (114 kHz) PLLs of a block share one dispatch.
struct PllJob {
    const float* in;
    size_t in_stride;
    float* tbuf;
    size_t t_stride;
    float* out;
    size_t out_stride;
    sdr_pll_state* st;
    float freq, Fs, bw, ncoScale, phaseAdjust;
    // context mode: out[0] (pll.cpp:18) is the previous block's last carrier, read by the NCO from
    // that block's output row (prev_out[ch][n]); the PLL kernel then never touches lastCarrier, so
    // the NCO of block b can run on another stream while the PLL of block b+1 runs.
    const float* prev_out;
    // pll_math.h pll_rx of every input sample (written by the producer of `in`)
    const double* rx;
    size_t rx_stride;
    // -in (written by the producer; row stride neg_stride): with it the PLL runs on lane pairs
    // (sdr_pll.hip pll_run_split)
    const float* in_neg;
    size_t neg_stride;
};
struct PllJobs {
    PllJob j[2];
};
// the two parities of a persistent launch: p[0] is the parity of the launch's first block
struct PllJobs2 {
    PllJobs p[2];
};

// ---- sdr_frontend.hip
struct FrontendArgs {
    const uint8_t* iq;
    size_t iq_stride;
    const uint8_t* tail_in;
    uint8_t* tail_out;
    const float2* prev_in;
    float2* prev_out;
    float* fm;                 // this parity's fm_demod stream (data base)
    const float* fm_other;     // the other parity's (history source)
    size_t fm_stride;
    int nch, ntaps, block_iq, block_if, D;
    const float* h;            // plain taps (generic kernel)
    const float* hs;           // register-blocked tap table (k_frontend2)
    const void* afrag;         // MFMA tap fragments (fast mode)
    double yscale;             // MFMA fixed-point scale
    const uint32_t* pad80;     // 64 words of u8 128
    bool fast;
    hipEvent_t ev0, ev1;       // non-null: HIP events recorded with the launch (sdr_frontend_timing)
    unsigned long long* stamps;   // non-null (k_frontend2): [workgroup][start, end] on the 100 MHz clock
};
// the whole block (jn <= 0) or tiles [j0, j0 + jn) of every channel (exact front end only)
int frontend_launch(const FrontendArgs& a, hipStream_t s, int j0 = 0, int jn = 0);
int frontend_tiles(int block_if);   // exact front-end tiles per channel and block
int frontend_tab_r();               // outputs per lane of the exact front end (tap-table row length)
// workgroups of a whole-block launch that stamps itself (sdr_frontend_timing), 0: the kernel does not
int frontend_stamp_wgs(int block_if, int nch, int ntaps, int D, bool fast);

// ---- sdr_pll.hip
int launch_nco(const PllJobs& jobs, int njobs, int n, int nch, hipStream_t s);
int launch_plls(bool libm, const PllJobs& jobs, int njobs, int n, int nch, hipStream_t s, bool with_nco = true);
// the context-free fmpll primitive: reciprocals, PLL, NCO
// (tbuf, rxbuf, negbuf: scratch [nch][t_stride]; negbuf receives -in for the lane-pair PLL)
int launch_pll(bool libm, const float* in, size_t in_stride, int n, int nch, float freq, float Fs, float* tbuf,
               size_t t_stride, double* rxbuf, float* negbuf, float* out, size_t out_stride, sdr_pll_state* st,
               float ncoScale, float phaseAdjust, float bw, hipStream_t s);
// persistent PLLs: words = [pre_flag, err, (pad), (pad), done ring of PLL_DONE_RING per-sequence
// counters]; returns the number of waves in *waves. Block sequence s is done when its ring slot
// done[s % PLL_DONE_RING] reaches waves * (s / PLL_DONE_RING + 1): per-block counters, because
// waves drift apart by more than a block (a wave that redoes many chunks lags the others, which
// may already finish the next block) and one shared count would release a block early.
// What a CU mask holds at once (tools/microbench/cumask_probe.hip, profiles/r06/cumask/): bit b of a
// HIP CU mask is CU slot j = b / NXCC of XCC b % NXCC, and slot j sits in shader engine j % 4 of that
// XCC (4 SEs x 8 CUs per XCC on MI355X). Workgroups are dealt round-robin over the XCCs and, inside
// one, over its SEs whether or not the SE has room, so a launch is resident at once only while every
// SE's share fits its CUs: a 48-CU mask gives each XCC SEs of 2, 2, 1 and 1 CUs, and 96 workgroups at
// two per CU left 32 of them waiting (the 1536-channel timeout of round 5). Measured bound, never
// exceeded over 1, 2 and 4 workgroups per CU and masks of 8..192 CUs:
//   resident workgroups <= xcc_active x min over those XCCs of (SEs with CUs x min CUs per such SE) x per_cu
struct CuPlacement {
    int ncu = 0;            // CUs in the mask
    int xcc_active = 0;     // XCCs with a CU in the mask
    int min_units = 0;      // min over active XCCs of (active SEs x min CUs per active SE)
    long long resident(int per_cu) const { return (long long)xcc_active * min_units * per_cu; }
};
CuPlacement cu_placement(const uint32_t* mask, int nwords, int ncu_dev, int nxcc);
// the persistent PLL launch's shape for jobs.p[k].j[0 .. njobs) (njobs = 2: the stereo and RDS PLLs,
// 1: one of them): kernel, workgroups, waves, and how many of its workgroups the placement keeps
// resident at once (resident < groups: the launch would hang)
struct PllMultiPlan {
    const void* kern = nullptr;
    int WG = 1, tab_ok = 0, per_cu = 0;
    size_t lds = 0;
    dim3 g, b;
    uint32_t waves = 0;
    long long groups = 0, resident = 0;
};
int pll_multi_plan(const PllJobs2& jobs, int njobs, int n, int nch, const CuPlacement& pl, PllMultiPlan* plan);
int launch_pll_multi(const PllJobs2& jobs, int njobs, int n, int nch, int nblocks, uint32_t* words, uint32_t pre_first,
                     unsigned long long* t0, unsigned long long* t1, unsigned long long* tc, uint32_t* waves,
                     hipStream_t s, const CuPlacement& pl,   // refused unless every workgroup is resident at once
                     int sub_tile);                 // > 0: the first block's input may come in parts of this many samples
int launch_flag_store(uint32_t* flag, uint32_t v, hipStream_t s);
int launch_flag_wait(const uint32_t* ctr, uint32_t want, uint32_t* err, hipStream_t s);
int diag_pll_counts(unsigned long long* out, int reset);
int diag_pll_waves(unsigned long long* out, int nmax);
int diag_pll_hwid(unsigned long long* out, int nmax);
constexpr int PLL_WORDS_DONE = 4;      // index of the done ring in the words array
// words[PLL_WORD_SUB]: the parts of a launch's first block published so far, as launch_base *
// PLL_SUB_SCALE + FIR tiles (a value no earlier launch can have left behind: no reset needed)
constexpr int PLL_WORD_SUB = 2;
constexpr uint32_t PLL_SUB_SCALE = 8;
constexpr uint32_t PLL_DONE_RING = 16; // waves stay within a few blocks of each other
constexpr int PLL_WORDS = PLL_WORDS_DONE + (int)PLL_DONE_RING;

}  // namespace sdrk

// ============================================================================================
// Context (sdr_kernels.hip owns it; the other units see the layout)
// ============================================================================================
struct sdr_ctx {
    int device = 0, nch = 0, mode = 0, rds_on = 0, flags = 0;
    sdr_info info{};
    int ntaps = 101;
    // taps (device)
    float *rf_h = nullptr, *rf_hs = nullptr, *pilot_h = nullptr, *stereo_h = nullptr, *pilot_band_h = nullptr, *rds_h = nullptr, *rds_sq_h = nullptr,
          *rrc_h = nullptr;
    float *audio_pp = nullptr, *rdsbb_pp = nullptr;   // polyphase tables
    int *audio_cnt = nullptr, *rdsbb_cnt = nullptr;
    int audio_L = 0, rdsbb_L = 0;
    // extended streams [2][nch][HIST + len]; pointers below are the data bases of parity 0
    float *fm = nullptr, *sdc = nullptr, *rband = nullptr, *rdc = nullptr, *rfilt = nullptr;
    size_t fm_stride = 0, rf_stride = 0;               // per-channel strides (if, rds lengths)
    size_t fm_par = 0, rf_par = 0;                      // parity offsets in elements
    // plain per-block buffers
    float *pilot_neg = nullptr, *gpilot_neg = nullptr;  // -pilot, -gen_pilot (the lane-pair PLL's input)
    float *pilot = nullptr, *band = nullptr, *gpilot = nullptr, *carrier = nullptr, *ipll = nullptr,
          *rds_clean = nullptr, *t_st = nullptr, *t_rds = nullptr;
    int* rds_ptq = nullptr;                             // RDS resampler (q << 8 | phase) per output
    bool rdsbb_all101 = false;                          // every RDS polyphase row has 101 taps
    bool audio_u1_101 = false;                          // audio resampler U == 1 with 101 taps
    double *rx_st = nullptr, *rx_rds = nullptr;         // PLL input reciprocals (pll_math.h pll_rx),
                                                        // [2 parities][nch][plain_stride], from the FIRs
    size_t plain_stride = 0, pll_stride = 0, clean_stride = 0;
    size_t plain_par = 0, pll_par = 0;                  // pilot/band/gpilot and carrier/ipll are
                                                        // [2 parities][nch][...] so that the stages
                                                        // split at the PLL can overlap blocks
    // state
    uint8_t* tail = nullptr;                            // [2][nch][2*(ntaps-1)]
    float2* prev = nullptr;                             // [2][nch]
    sdr_pll_state *st_pll = nullptr, *rds_pll = nullptr;
    int32_t* dec = nullptr;                             // [nch][DEC_STATE]
    uint32_t* pad80 = nullptr;                          // 64 words of u8 128 (the zero sample)
    void* fe_afrag = nullptr;                           // MFMA front end: tap digit fragments
    double fe_yscale = 0.0;                             // 2^-(F+7): fixed-point taps, x = (u-128)/128
    int cus = 0;                                        // compute units of the device
    int parity = 1;                                     // parity of the current block
    long long block = -1;                               // index of the current block
    long long stereo_done = -1, rds_dsp_done = -1, rds_bits_done = -1, mono_done = -1;
    long long st_pre_done = -1, st_pll_done = -1, rds_pre_done = -1, rds_pll_done = -1;
    // persistent PLLs (sdr_plls_launch / _signal / _wait): device words (launch_pll_multi), per-block
    // timestamps of the last launch, and the host's sequence bookkeeping
    uint32_t* pers_words = nullptr;
    unsigned long long *pers_t0 = nullptr, *pers_t1 = nullptr;
    unsigned long long* pers_cyc = nullptr;             // [block][2]: sums over waves of cycles, 100 MHz ticks
    int pers_tcap = 0, pers_last_n = 0;
    int pers_prepared = 0;                              // sdr_plls_prepare's nblocks (0: none pending)
    uint32_t pers_prepared_launch = 0;                  // pers_launched when it was prepared
    uint32_t pers_launched = 0, pers_signaled = 0, pers_waves = 0;
    int pers_which = SDR_PLLS_BOTH;                     // the PLLs the last launch runs (sdr_plls_launch_sel)
    uint32_t pers_base = 0;                             // sequence number of the last launch's first block
    uint32_t pers_waited = 0;                           // sequence numbers below this have been waited for
    long long pers_first_block = -1;                    // the context block that sequence number belongs to
    hipStream_t pers_stream = nullptr;                  // stream of the last launch
    long long pers_block = -1;                          // block of the last signal
    uint32_t pers_block_seq = 0;                        // its sequence number
    hipEvent_t pers_ev = nullptr;                       // orders a prepare on another stream after the last launch
    // parity release (sdr_kernels.hip release_record / release_wait): rel_words[p][slot] counts the
    // blocks of parity p read by slot 0 sdr_mono (fm), 1 sdr_stereo_post (fm, band, t_st, carrier),
    // 2 sdr_rds_post's mixer (rband, t_rds, ipll), stored on the reader's stream (rel_stream) after
    // its kernels; the producers of the block two later wait for the count on their own streams
    static constexpr int REL_SLOTS = 3;
    uint32_t* rel_words = nullptr;                      // [2][REL_SLOTS] counters
    uint32_t rel_seq[2][REL_SLOTS] = {};
    hipStream_t rel_stream[2][REL_SLOTS] = {};
    uint32_t rel_waited[2][REL_SLOTS] = {};            // the count a wait on rel_waited_on already covers
    hipStream_t rel_waited_on[2][REL_SLOTS] = {};
    bool pers_failed = false;                           // sdr_plls_report saw a timeout of the current launch
    // streams whose post stages read the last launch's error word (sdr_plls_wait): the next launch's
    // prepare clears that word only after them (events recorded on each, waited for on its stream)
    static constexpr int PERS_READERS = 4;
    hipStream_t pers_readers[PERS_READERS] = {};
    int pers_nreaders = 0;
    hipEvent_t pers_reader_ev[PERS_READERS] = {};
    // the persistent launch's error word the post stages of the current block check (their outputs
    // are poisoned when a persistent wait timed out): only for blocks signalled through a launch
    const uint32_t* pers_err() const { return (pers_words && pers_block == block) ? pers_words + 1 : nullptr; }
    // release timeout (sdr_kernels.hip release_wait): fail_words[0] is set on the device by a parity
    // release wait that gave up (a reader had not released a buffer within ~5 s, and the producer
    // then overwrote it); every output stage poisons its block while it is set, and the same wait sets
    // the host-mapped *fail_host, which every later stage call checks (SDR_E_TIMEOUT). sdr_ctx_reset
    // clears both.
    uint32_t* fail_words = nullptr;
    uint32_t* fail_host = nullptr;                      // hipHostMalloc'd (coherent), host view
    uint32_t* fail_host_dev = nullptr;                  // its device address
    // sdr_frontend_timing: the dispatch stamps of the next fe_time_cap whole-block front-end launches
    std::vector<hipEvent_t> fe_ev;                      // [2 * cap]: start, end per launch (HIP events)
    unsigned long long* fe_stamps = nullptr;            // [cap][fe_stamp_wgs][2] (k_frontend2's own stamps)
    int fe_stamp_wgs = 0, fe_stamp_cap = 0;
    bool fe_use_stamps = false;                         // the exact front end (k_frontend2): stamps
    int fe_time_cap = 0, fe_time_n = 0;
    std::vector<void*> allocs;

    float* fm_cur() const { return fm + parity * fm_par; }
    float* fm_oth() const { return fm + (parity ^ 1) * fm_par; }
    float* ext(float* base, size_t par, int p) const { return base + p * par; }
    float* plain(float* base) const { return base + parity * plain_par; }
    float* pllbuf(float* base) const { return base + parity * pll_par; }
    double* rxbuf(double* base) const { return base + parity * plain_par; }
};
