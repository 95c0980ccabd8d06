/*
 * sdr_amd.h -- C ABI of the MI355X-native FM/RDS DSP hot path (libsdr_amd.so, gfx950).
 *
 * Drop-in boundary for TheZxc07/real-time-SDR's per-block DSP (reference paths are relative to
 * the reference repository root). Every entry point is extern "C", takes plain pointers and
 * sizes, returns an int status (SDR_OK = 0) and enqueues work on the caller's HIP stream
 * (`stream` = hipStream_t, NULL = default stream) without synchronising.
 *
 * Data layout (HBM): channel-major batches. A batch of nch independent I/Q streams is
 * `[nch][len]` with a per-channel stride (in elements); per-channel state lives in device memory
 * and is updated in place, exactly like the reference's by-reference state arguments.
 *
 * Numerics: the default ("exact") mode reproduces the reference's rounding points bit for bit:
 * f32 products and sums in tap order without FMA (filter.cpp:111-115), f64 demod denominator
 * and division (demod.cpp:17), f64 atan2/sin/cos rounded to f32 in the PLL (pll.cpp:39-52).
 */
#ifndef SDR_AMD_H
#define SDR_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SDR_OK 0
#define SDR_E_INVALID (-1)   /* bad argument / shape */
#define SDR_E_HIP (-2)       /* HIP runtime error (see sdr_last_error) */
#define SDR_E_NOMEM (-3)
#define SDR_E_NODEV (-4)     /* no gfx950 device */
#define SDR_E_TIMEOUT (-5)   /* a parity-release wait gave up (a reader held its block > 5 s): the context's
                              * outputs are poisoned from then on; every stage call fails until
                              * sdr_ctx_reset */

#define SDR_MAX_SYMS 256     /* symbols per block, >= n_rds/symbol_Fs + 1 for every mode */
#define SDR_MAX_BITS 256

/* Outputs of a block whose persistent PLL wait timed out (sdr_plls_launch), or of any block after a
 * parity-release wait timed out (SDR_E_TIMEOUT): the output stages write these instead of audio /
 * bits computed from phases that were never produced or from buffers the producer overwrote. */
#define SDR_PCM_POISON ((int16_t)-32768)  /* every L/R sample of the block */
#define SDR_NBITS_POISONED (-2)           /* nbits[ch] of sdr_rds_bits; rds_clean rows are NaN */

/* Context flags */
#define SDR_FLAG_FAST_FRONTEND 0x1  /* FMA front end: fm_demod within 1e-6 rel., not bit-exact */
#define SDR_FLAG_PLL_LIBM 0x2       /* PLL via per-step f64 libm calls (A/B reference) */
#define SDR_FLAG_KEEP_INTERMEDIATES 0x4  /* post stages store every intermediate row (carrier, stereo_dc,
                                          * ipll) for sdr_ctx_buffer; by default the NCO, mixers and
                                          * resamplers are fused and only the rows' history is stored */

/* pllblock_args, include/pll.h:10-17 (same field order and types) */
typedef struct sdr_pll_state {
    float feedbackI;
    float feedbackQ;
    float integrator;
    float phaseEst;
    double trigOffset;
    float lastCarrier;   /* the reference keeps it as pllOut[last]; out[0] of the next block */
} sdr_pll_state;

/* Static geometry of a context (mode table of project.cpp:67-108) */
typedef struct sdr_info {
    int nch, mode, rds_on;
    int rf_Fs, rf_decim, if_Fs, audio_upsample, audio_decim, symbol_Fs, rf_taps;
    int block_iq;   /* I/Q pairs per block (rffrontend.cpp:21)          mode 0: 73500 */
    int block_if;   /* fm_demod samples per block                        mode 0: 7350  */
    int n_audio;    /* audio frames per block (mono.cpp:28)             mode 0: 1470  */
    int n_rds;      /* RDS baseband samples per block (rds.cpp:130)      mode 0: 2836  */
    int history;    /* samples of history kept in front of each f32 stream */
} sdr_info;

typedef struct sdr_ctx sdr_ctx;

const char *sdr_last_error(void);
int sdr_version(void);

/* ------------------------------------------------------------------ tap design (host, once)
 * Same formulas, types and rounding as the reference; h must hold num_taps floats. */
int sdr_impulse_response_lpf(float Fs, float Fc, unsigned short num_taps, float *h);            /* filter.cpp:13-29 */
int sdr_impulse_response_lpf_gain(float Fs, float Fc, unsigned short num_taps, int u, float *h); /* filter.cpp:33-50 */
int sdr_impulse_response_bpf(float Fs, const float *Fb, unsigned short num_taps, float *h);     /* filter.cpp:55-71 */
int sdr_impulse_response_apf(float gain, unsigned short num_taps, float *h);                    /* filter.cpp:73-78 */
int sdr_impulse_response_rrc(float Fs, unsigned short num_taps, float *h);                      /* filter.cpp:80-102 */

/* ------------------------------------------------------------------ batched primitives
 * All pointers are device pointers. `state` arrays are [nch][nstate] (nstate >= ntaps-1 for
 * convolveFIR) and hold the previous block's last nstate inputs, zero-initialised by the caller
 * like the reference's std::vector<float>(rf_taps-1). */

/* convolveFIR(y, x, h, state, D): filter.cpp:106-121 (include/filter.h:20). y: [nch][nx/D]. */
int sdr_convolve_fir(float *y, size_t y_stride, const float *x, size_t x_stride, int nch, int nx,
                     const float *h, int ntaps, float *state, int nstate, int D, void *stream);
/* convolveFIR(y, x, h, state, U, D): filter.cpp:123-147 (include/filter.h:24). y: [nch][nx*U/D].
 * Phase restarts at 0 each block; only the last `nstate` (>= 100 for every mode) inputs of the
 * previous block are kept (the reference copies ntaps-1, reading before x). */
int sdr_convolve_fir_resample(float *y, size_t y_stride, const float *x, size_t x_stride, int nch, int nx,
                              const float *h, int ntaps, float *state, int nstate, int U, int D, void *stream);
/* fmDemodNoArctan(I, Q, prevI, prevQ, out): demod.cpp:3-24 (include/demod.h:5). prev: [nch][2]. */
int sdr_fm_demod(float *out, size_t out_stride, const float *I, const float *Q, size_t iq_stride, int nch,
                 int n, float *prev, void *stream);
/* fmpll(in, freq, Fs, out, state, ncoScale, phaseAdjust, bw): pll.cpp:4-61 (include/pll.h:20).
 * out: [nch][n+1]; out[ch][0] is set from state[ch].lastCarrier (the previous block's last
 * sample, pll.cpp:18), state[ch].lastCarrier <- out[ch][n]. */
int sdr_fmpll(float *out, size_t out_stride, const float *in, size_t in_stride, int nch, int n, float freq,
              float Fs, sdr_pll_state *state, float ncoScale, float phaseAdjust, float normBandwidth,
              void *stream);
/* cdr(sps, signal): rds_utilities.cpp:4-21 (include/rds_utilities.h:6). offset: [nch] int32. */
int sdr_cdr(int32_t *offset, const float *x, size_t x_stride, int nch, int n, int sps, void *stream);
/* manchester_decode(bits, symbols, block_count, half_symbol, start): rds_utilities.cpp:34-68
 * (include/rds_utilities.h:12). symbols [nch][sym_stride] 0/1 bytes with nsym[ch] valid;
 * state [nch][2] = {half_symbol, start} updated in place; bits [nch][bits_stride] 0/1 bytes,
 * nbits[ch] written. block_count as in the reference (0 selects the alignment search). */
int sdr_manchester_decode(uint8_t *bits, size_t bits_stride, int32_t *nbits, const uint8_t *symbols,
                          size_t sym_stride, const int32_t *nsym, int nch, int block_count, int32_t *state,
                          void *stream);
/* differential_decode(out, bits, last_bit, block_num): rds_utilities.cpp:70-88
 * (include/rds_utilities.h:14). last_bit [nch] int32 updated in place. */
int sdr_differential_decode(uint8_t *out, size_t out_stride, const uint8_t *bits, size_t bits_stride,
                            const int32_t *nbits, int nch, int block_num, int32_t *last_bit, void *stream);

/* ------------------------------------------------------------------ fused pipeline
 * A context owns the taps, every inter-stage buffer and all per-channel state of `nch`
 * channels of one mode on one device: RF_frontend + mono + stereo + rds of the reference
 * (rffrontend.cpp:9-77, mono.cpp:8-50, stereo.cpp:10-115, rds.cpp:11-193) as batched kernels. */
int sdr_ctx_create(sdr_ctx **out, int device, int nch, int mode, int rds_on, int flags);
int sdr_ctx_destroy(sdr_ctx *ctx);
/* all state back to the reference's initial values; clears a release timeout (SDR_E_TIMEOUT) and the
 * last persistent launch's hold on the current block. Call it once the streams that ran the context's
 * stages have drained. */
int sdr_ctx_reset(sdr_ctx *ctx, void *stream);
int sdr_ctx_info(const sdr_ctx *ctx, sdr_info *info);

/* RF_frontend loop body (rffrontend.cpp:58-71): iq [nch][2*block_iq] u8 interleaved I/Q ->
 * the context's fm_demod for this block. Advances the context to the next block. */
int sdr_frontend(sdr_ctx *ctx, const uint8_t *iq, size_t iq_stride, void *stream);
/* The parity-release wait the next sdr_frontend (or sdr_frontend_pre_parts) begins with, enqueued on
 * `stream` now (the producer's wait for its consumers' prepare(), threadsafequeue.h:29-31): that call,
 * on the same stream, then has nothing left to wait for, so a caller can time or order the front-end
 * kernel alone. Optional. */
int sdr_frontend_release_wait(sdr_ctx *ctx, void *stream);
/* Kernel timing of the front end (no reference counterpart; for benchmarks): the next `max_launches`
 * sdr_frontend kernels are timed -- the 101-tap exact and fast (MFMA) front ends by their own
 * workgroups' start and end stamps (s_memrealtime: the earliest start to the latest end, the kernel's
 * span as a rocprofv3 kernel trace sees it), the generic one by HIP events recorded with the launch
 * -- and sdr_frontend_times returns them in ms (synchronising the device). 0 disables; each call
 * re-arms from the first. sdr_frontend_pre_parts launches are not timed. */
int sdr_frontend_timing(sdr_ctx *ctx, int max_launches);
int sdr_frontend_times(sdr_ctx *ctx, double *ms, int max, int *n);
/* The same launches' earliest workgroup start and latest end as raw 100 MHz device ticks (the clock
 * of sdr_plls_timeline), stamping front ends only: where each block's front end sat in the pipeline. */
int sdr_frontend_stamps(sdr_ctx *ctx, unsigned long long *t_start, unsigned long long *t_end, int max, int *n);
/* mono loop body (mono.cpp:34-42) on the current block: audio [nch][n_audio] int16 */
int sdr_mono(sdr_ctx *ctx, int16_t *audio, size_t audio_stride, void *stream);
/* stereo loop body (stereo.cpp:74-107): lr [nch][2*n_audio] int16, L/R interleaved */
int sdr_stereo(sdr_ctx *ctx, int16_t *lr, size_t lr_stride, void *stream);
/* rds DSP (rds.cpp:105-133): rds_clean [nch][n_rds] f32 (may be NULL: kept internally) */
int sdr_rds_dsp(sdr_ctx *ctx, float *rds_clean, size_t rds_stride, void *stream);
/* The same two loop bodies split at their PLL, in this order per block (each part may run on its
 * own stream; the caller orders them with events): sdr_X = sdr_X_pre; sdr_X_pll; sdr_X_post.
 *   stereo_pre   pilot + band BPFs          stereo.cpp:74, :80
 *   stereo_pll   19 kHz PLL, x2 carrier      stereo.cpp:77
 *   stereo_post  mixer, delay, resamplers    stereo.cpp:83-107
 *   rds_pre      BPF, squaring, 114 kHz BPF  rds.cpp:105-116
 *   rds_pll      114 kHz PLL, x0.5           rds.cpp:119
 *   rds_post     delay, mixer, 247/640, RRC  rds.cpp:122-133
 * Intermediates crossing the split are kept per block parity, so the PLL of block b+1 may run
 * while block b's post part is still running. Parity release (threadsafequeue.h:29-31): the
 * readers of a block's parity buffers -- sdr_mono, sdr_stereo_post and sdr_rds_post's mixer --
 * record on their stream that they have read it, and sdr_frontend (likewise sdr_push_fm_demod,
 * the pre parts and sdr_frontend_pre_parts) waits on its own stream until the readers of block
 * b-2, which used the same parity, have done so: the caller needs no wait of its own for that
 * reuse. Outputs handed to the caller (lr, rds_clean, bits) are the caller's to order. The wait is
 * bounded (5 s): a reader that has not released its block by then makes it an error, never wrong
 * output -- the producer goes on, every output stage that runs afterwards writes SDR_PCM_POISON
 * audio (mono and stereo), NaN rds_clean rows and nbits = SDR_NBITS_POISONED, and every later call
 * on the context returns SDR_E_TIMEOUT until sdr_ctx_reset. */
int sdr_stereo_pre(sdr_ctx *ctx, void *stream);
int sdr_stereo_pll(sdr_ctx *ctx, void *stream);
int sdr_stereo_post(sdr_ctx *ctx, int16_t *lr, size_t lr_stride, void *stream);
int sdr_rds_pre(sdr_ctx *ctx, void *stream);
/* sdr_stereo_pre + sdr_rds_pre of the current block on ONE stream: the pilot, band and RDS band
 * BPFs read the staged fm_demod window once (stereo.cpp:74,80 and rds.cpp:105 share the input),
 * then the squared-RDS BPF. For callers that run both pre parts on the same stream. */
int sdr_pre(sdr_ctx *ctx, void *stream);
int sdr_rds_pll(sdr_ctx *ctx, void *stream);
int sdr_rds_post(sdr_ctx *ctx, float *rds_clean, size_t rds_stride, void *stream);
/* stereo_pll + rds_pll of the current block in one dispatch (2 x nch independent recurrences);
 * needs both _pre parts done. */
int sdr_plls(sdr_ctx *ctx, void *stream);
/* Persistent PLLs: the stereo + RDS PLLs of many consecutive blocks in ONE dispatch (no launch
 * gap between blocks). sdr_plls_launch(nblocks) on the PLL stream, before the sdr_frontend of the
 * first of those blocks; then per block, after both _pre parts, sdr_plls_signal on the stream that
 * ran them (instead of sdr_plls) and sdr_plls_wait on the stream of the _post parts. The kernel
 * waits for each block's signal (a device flag written in stream order), runs both PLLs, and
 * releases the waiting stream. The PLL stream must be one sdr_stream_create_cu_range made (it owns
 * its hardware queue; on a pool stream a signal could queue behind the waiting launch), and every
 * workgroup of the launch must be resident on that stream's CUs at once -- by the workgroups of its
 * kernel that fit one CU and by how the CU mask falls on the XCCs' shader engines (workgroups are
 * dealt to the engines evenly, so an engine with fewer CUs of the mask fills first; sdr_plls_fits):
 * otherwise the launch is refused with SDR_E_INVALID before anything is enqueued (use sdr_plls, or
 * another CU range). A wait longer than 5 s (a block
 * never signalled, or a post stream that waits for a block the PLL never finished) ends the launch
 * without computing: from then on the post stages of that launch's blocks write SDR_PCM_POISON
 * audio, NaN rds_clean rows and nbits = SDR_NBITS_POISONED (never audio from phases the PLL did
 * not produce), sdr_plls_report returns SDR_E_HIP, and after that report the post calls of those
 * blocks fail too; sdr_ctx_reset + a new launch recover. sdr_plls_report also returns each
 * block's PLL time of the last launch (ms, from the device clock: its last wave's end minus the
 * later of its signal and the previous block's end) and synchronises `stream`. While a launch still
 * waits for blocks, nothing may synchronise with the PLL stream implicitly: a CU-masked stream is a
 * blocking stream, so work on the legacy null stream would wait for it (until the 5 s bound). Each
 * block must be waited for (sdr_plls_wait) before the 16th block after it is signalled. Launching
 * again while blocks of the previous launch were never signalled first lets that launch time out
 * and drain. Not with SDR_FLAG_PLL_LIBM. */
int sdr_plls_launch(sdr_ctx *ctx, int nblocks, void *stream);
/* The same for one of the two PLLs (which = SDR_PLLS_STEREO or SDR_PLLS_RDS; SDR_PLLS_BOTH is
 * sdr_plls_launch): for a context that runs one chain only, as each consumer thread of the reference
 * does (project.cpp:134-136: stereo in the audio thread, RDS in the rds thread). sdr_plls_signal
 * then needs only that chain's _pre part, and only that chain's _post part follows the wait. */
#define SDR_PLLS_STEREO 1
#define SDR_PLLS_RDS 2
#define SDR_PLLS_BOTH 3
int sdr_plls_launch_sel(sdr_ctx *ctx, int nblocks, int which, void *stream);
/* Would sdr_plls_launch_sel(which) accept a stream made by sdr_stream_create_cu_range(first_cu, n_cu,
 * exclude = 0) for this context? Fills the launch's waves, its workgroups and how many of them that
 * CU range keeps resident at once; it fits when *groups <= *resident. No stream is made, nothing is
 * enqueued. */
int sdr_plls_fits(sdr_ctx *ctx, int which, int first_cu, int n_cu, int *waves, long long *groups,
                  long long *resident);
/* Optional, ahead of sdr_plls_launch(nblocks) (e.g. before a timed region): the launch's
 * bookkeeping -- allocation, the reset of its stamps and error word -- in `stream`'s order, so the
 * launch itself only enqueues the kernel. Ignored by a launch with another nblocks. */
int sdr_plls_prepare(sdr_ctx *ctx, int nblocks, void *stream);
int sdr_plls_signal(sdr_ctx *ctx, void *stream);
/* The pipeline fill: the FIRST block of a pending persistent launch as sdr_frontend + sdr_pre +
 * sdr_plls_signal in `nparts` sample ranges (at most one per 2048-sample pre-PLL FIR tile), each
 * range published as soon as its front end and pre-PLL FIRs are done, so the PLLs start on the
 * block's first range while the rest is produced (the reference's producer hands a block over whole,
 * threadsafequeue.h:24-44; the PLL consumes its input in order, pll.cpp:34-53, and waits before
 * every sample that is not published yet). Exact numerics, rds_on, 101 taps only. */
int sdr_frontend_pre_parts(sdr_ctx *ctx, const uint8_t *iq, size_t iq_stride, int nparts, void *stream);
int sdr_plls_wait(sdr_ctx *ctx, void *stream);
int sdr_plls_report(sdr_ctx *ctx, double *block_ms, int max_blocks, int *nblocks, void *stream);
/* The raw device stamps of the last persistent launch (100 MHz s_memrealtime ticks), per block:
 * t_start[j] = when its signal was seen, t_end[j] = its last wave's end; synchronises `stream`. */
int sdr_plls_timeline(sdr_ctx *ctx, unsigned long long *t_start, unsigned long long *t_end, int max_blocks,
                      int *nblocks, void *stream);
/* Per-step cost of the last persistent launch from the waves' own clocks: shader cycles per PLL step
 * and wave (s_memtime over each wave's compute of each block, averaged) and the shader clock over
 * the same intervals (against the 100 MHz s_memrealtime); synchronises `stream`. */
int sdr_plls_cycles(sdr_ctx *ctx, double *cycles_per_step, double *clock_mhz, void *stream);
/* The same per block j < max of the last persistent launch (cycles per step and wave, shader clock);
 * *n = the launch's block count. */
int sdr_plls_block_cycles(sdr_ctx *ctx, double *cycles_per_step, double *clock_mhz, int max, int *n,
                          void *stream);
/* rds symbol/bit recovery (rds.cpp:135-167): per channel, for blocks with block_count > 5 and
 * rds_on: offset = cdr(), symbols (0/1 bytes), bits (decoded 0/1 bytes). nbits[ch] = -1 on
 * blocks that do not decode. Any output pointer may be NULL. Strides in elements. */
int sdr_rds_bits(sdr_ctx *ctx, int32_t *offset, int32_t *nsym, uint8_t *symbols, size_t sym_stride,
                 int32_t *nbits, uint8_t *bits, size_t bits_stride, void *stream);
/* Consumer-side entry (wait_and_pop, threadsafequeue.h:46): make an fm_demod block produced
 * elsewhere (another context, another GPU, or host data copied to the device) the context's
 * current block; mono/stereo/rds then consume it. fm [nch][block_if] device memory. */
int sdr_push_fm_demod(sdr_ctx *ctx, const float *fm, size_t fm_stride, void *stream);
/* Copy out the context's current-block fm_demod [nch][block_if] (the reference's queue payload) */
int sdr_get_fm_demod(sdr_ctx *ctx, float *fm, size_t fm_stride, void *stream);
/* Debug / parity access to intermediates of the current block (device pointers into the
 * context, valid until the next sdr_frontend; "carrier", "stereo_dc" and "ipll" hold whole rows only
 * with SDR_FLAG_KEEP_INTERMEDIATES): name in {"fm","pilot","carrier","band","rds_band",
 * "gen_pilot","ipll","rds_dc","rds_filt","rds_clean","stereo_dc"}; *stride in elements. */
int sdr_ctx_buffer(sdr_ctx *ctx, const char *name, const float **ptr, size_t *stride, int *len);

/* Streams on disjoint CU sets (no reference counterpart: the reference's three threads,
 * project.cpp:134-136, share one CPU; this is their placement on the GPU). Creates a HIP stream
 * on `device` whose kernels run only on CU-mask bits [first_cu, first_cu + n_cu) (exclude = 0),
 * or on every CU except those (exclude = 1). Giving the serial PLL stream (sdr_plls) its own CUs
 * keeps the other stages' kernels off the SIMDs its lone waves issue from.
 * Release with sdr_stream_destroy. */
int sdr_stream_create_cu_range(void **stream, int device, int first_cu, int n_cu, int exclude);
int sdr_stream_destroy(void *stream);

/* Bandwidth calibration (no reference counterpart): device-to-device copy of `bytes` (a multiple
 * of 16, 16-byte aligned pointers) with a streaming kernel over every CU, so that a benchmark can
 * state the HBM rate a plain stream reaches next to the nominal peak. */
int sdr_hbm_copy(void *dst, const void *src, size_t bytes, void *stream);

#ifdef __cplusplus
}
#endif
#endif
