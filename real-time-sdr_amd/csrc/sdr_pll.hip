// sdr_pll.hip -- the PLL / NCO recurrence of the FM/RDS hot path on MI355X (gfx950):
//   fmpll, pll.cpp:4-61 (pllblock_args, include/pll.h:10-20), one lane per channel, with
//   pll_math.h's correctly-rounded fast paths and double-double fallbacks;
//   the persistent multi-block launch and its stream hand-offs.
#include "sdr_internal.h"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <type_traits>

#include "pll_math.h"

#pragma clang fp contract(off)

namespace sdrk {
namespace {
// ------------------------------------------------------------------------------------------
// PLL / NCO, pll.cpp:4-61. One lane per channel: the recurrence is serial in time.
//
// k_pll_libm: the literal restatement (f64 OCML atan2/sincos per step), kept as the A/B
// reference (flag SDR_FLAG_PLL_LIBM) and used for chunk redo.
// k_pll: the same recurrence with pll_math.h's correctly-rounded fast paths. Each 64-step chunk
// runs branch-free; if any step of a lane reported an ambiguous f32 rounding (~6.6e-6 per step)
// the lane restores its chunk snapshot and redoes the chunk with per-step f64-libm fallbacks.
// Both write out[0] = lastCarrier and out[i+1] = t_i (the f32 NCO phase); k_nco_out then turns
// t_i into cos(t_i*ncoScale + phaseAdjust) in parallel (pll.cpp:52) and updates lastCarrier.
// ------------------------------------------------------------------------------------------
struct PllRegs {
    float fbI, fbQ;              // in the reduced frame: RN(cos r), RN(sin r) (pll_math.h)
    f32x2 ip;                    // {integrator, phaseEst}: one packed multiply and add per step
    double toff;
    double c, s, mr;             // f64 cos r, sin r and -r of the previous step's t = q pi/2 + r
    uint32_t nq1, b;             // 1 - q (mod 2^32) for its quadrant q, and [r < 0]
};

// The carried rotation is rebuilt from the state's previous trigArg t = (float)(w*toff + phaseEst)
// (pll.cpp:47). The fast phase detector needs feedbackI/Q to be RN_f32(cos t), RN_f32(sin t) of
// that same t -- true for any state this PLL (or the reference) left behind and for the initial
// state (1, 0, toff 0, phase 0). Otherwise, or when t is out of the reduction's range, the
// feedback is kept as given with q = 0 and mr = NaN: the first fast step yields a NaN and the
// chunk is redone with libm fallbacks, which use the state's feedback exactly.
__device__ __forceinline__ PllRegs pll_load(const sdr_pll_state& st, double w) {
    PllRegs r;
    r.ip = f32x2{st.integrator, st.phaseEst};
    r.toff = st.trigOffset;
    const float t_prev = (float)(w * r.toff + (double)r.ip.y);
    const pllm::SinCosRN sc = pllm::sincos_rn(t_prev);
    float fI = (float)sc.cr, fQ = (float)sc.sr;
    pllm::rot_q(1u - sc.nq1, fI, fQ);
    const bool consistent = (__builtin_fabs((double)t_prev) < pllm::T_MAX) && sc.tie > pllm::TIE_MIN &&
                            fI == st.feedbackI && fQ == st.feedbackQ;
    if (consistent) {
        r.fbI = (float)sc.cr;
        r.fbQ = (float)sc.sr;
        r.c = sc.cr;
        r.s = sc.sr;
        r.mr = -sc.r;
        r.nq1 = sc.nq1;
        r.b = sc.b;
    } else {
        r.fbI = st.feedbackI;
        r.fbQ = st.feedbackQ;
        r.c = 1.0;
        r.s = 0.0;
        r.mr = __builtin_nan("");
        r.nq1 = 1u;
        r.b = 0u;
    }
    return r;
}

// Per-chunk proof obligations of the fast path (VGPR accumulators, one check per chunk):
//   * every phase-detector result is at least EPS_ABS_E2 from an f32 rounding boundary (split)
//     and |e| < pi - 2^-30 (so the wrap to [-pi, pi] is the reference's),
//   * every cos/sin is at least 64 f64 ulps from an f32 tie (tie),
//   * the chunk ends with |phaseEst| < 2^28, |integrator| < 2^20 (finite: a NaN or inf from an
//     invalid input -- pll_rx gives NaN for |x| < 2^-60 -- propagates into both),
//   * every |t| of the chunk is below 2^30 (T_MAX, the two-fma reduction's range): with the trigArg
//     table (TAB) the launch checked |w| (|toff| + n + 1) < 1.375 * 2^29, which leaves room for
//     |phaseEst| < 2^28 plus 16 steps of drift; without it the chunk's largest |t| is tracked.
struct PllProof {
    double emax = 0.0;
    float emaxf = 0.0f;     // lane-pair steps: max |RN32(ed)| (PLL_EMAX_F)
    uint32_t split = 0u;
    uint32_t tie = ~0u;
    float tmax = 0.0f;
};
// (the A/B variants of this step measured and dropped -- e bracket order, bracket by fma, pre-loop
// wait, packed loop filter, first table entries carried, one lane per chain, no trigArg table -- are
// kept as tools/patches/pll_variants.patch)
// |e| bound of the fast phase detector (the wrap to [-pi, pi] is the reference's below it)
constexpr double PLL_EMAX = pllm::PI - 0x1p-30;
// the largest f32 below PLL_EMAX: RN32 is monotone, so |RN32(ed)| < PLL_EMAX_F implies |ed| < PLL_EMAX_F
constexpr float PLL_EMAX_F = __builtin_bit_cast(float, 0x40490FDAu);
static_assert((double)PLL_EMAX_F < PLL_EMAX, "PLL_EMAX_F");
constexpr double PLL_TAB_WT_MAX = 0x1.6p29;   // |w * trigOffset| bound of the table path (above)

#ifndef SDR_PLL_COUNT
#define SDR_PLL_COUNT 0   // diagnosis build: count the fast chunks and the redone ones (sdr_diag_pll_counts)
#endif
#if SDR_PLL_COUNT
// [lane-chunks, lane-chunks that failed their proof, wave-chunks, wave-chunks redone]
// [4..7]: lane-chunks failing the e range, the e bracket, the cos/sin ties, the state range (a chunk
// can fail several); [8], [9]: failed lane-chunks of job 0 (stereo 19 kHz) and job 1 (RDS 114 kHz)
constexpr int PLL_NCOUNTS = 10;
__device__ unsigned long long g_pll_counts[PLL_NCOUNTS];
__device__ __forceinline__ void pll_count_reasons(bool emax_bad, bool split_bad, bool tie_bad, bool state_bad) {
    const unsigned long long exec = __builtin_amdgcn_read_exec();
    const unsigned long long m[4] = {__ballot(emax_bad) & exec, __ballot(split_bad) & exec, __ballot(tie_bad) & exec,
                                     __ballot(state_bad) & exec};
    const unsigned long long any = (m[0] | m[1] | m[2] | m[3]);
    if ((int)__lane_id() == __ffsll((long long)exec) - 1) {
        for (int k = 0; k < 4; k++) atomicAdd(&g_pll_counts[4 + k], (unsigned long long)__popcll(m[k]));
        atomicAdd(&g_pll_counts[8 + (blockIdx.y & 1)], (unsigned long long)__popcll(any));
    }
}
__device__ __forceinline__ void pll_count_chunk(bool ok) {
    const unsigned long long exec = __builtin_amdgcn_read_exec();
    const unsigned long long bad = __ballot(!ok) & exec;
    if ((int)__lane_id() == __ffsll((long long)exec) - 1) {
        atomicAdd(&g_pll_counts[0], (unsigned long long)__popcll(exec));
        atomicAdd(&g_pll_counts[1], (unsigned long long)__popcll(bad));
        atomicAdd(&g_pll_counts[2], 1ull);
        atomicAdd(&g_pll_counts[3], bad ? 1ull : 0ull);
    }
}
#endif

#ifndef SDR_PLL_WAVES
#define SDR_PLL_WAVES 0   // diagnosis build: per-wave totals of the last persistent launch (sdr_diag_pll_waves)
#endif
#if SDR_PLL_WAVES
// per wave of k_pll_multi: [0] shader cycles inside its blocks, [1] 100 MHz ticks from the start of
// each block's flag poll to after its acquire, [2] blocks computed, [3] job (0 stereo 19 kHz, 1 RDS
// 114 kHz) + 1, [4] ticks of [1] until the poll saw the flag, [5] polls that found it unset, [6]
// blocks whose first poll found it set, [7] ticks between the flag's publication (g_flag_t) and the
// poll's start, summed over the blocks where it was published first (negative: the wave waited)
constexpr int PLL_WAVE_SLOTS = 4096, PLL_WAVE_FIELDS = 8;
__device__ unsigned long long g_pll_waves[PLL_WAVE_SLOTS][PLL_WAVE_FIELDS];
// the 100 MHz time at which k_flag_store published each block flag value of the launch (indexed by
// value % 64; g_diag_flag: the launch's block flag word)
__device__ unsigned long long g_flag_t[64];
__device__ const uint32_t* g_diag_flag;
#endif

#ifndef SDR_PLL_HWID
#define SDR_PLL_HWID 0    // diagnosis build: where each k_pll wave ran and for how long (sdr_diag_pll_hwid)
#endif
#if SDR_PLL_HWID
// per wave of the last k_pll launches (slot = blockIdx.y * gridDim.x + blockIdx.x): [0] HW_ID
// (wave slot, SIMD, CU, shader array, SE), [1] XCC_ID, [2] shader cycles from entry to exit, [3], [4]
// 100 MHz time at entry and at exit
constexpr int PLL_HWID_SLOTS = 4096, PLL_HWID_FIELDS = 5;
__device__ unsigned long long g_pll_hwid[PLL_HWID_SLOTS][PLL_HWID_FIELDS];
#endif

// TAB: the trigArg offsets come from a table whose range the kernel checked once (pll_run)
template <bool TAB>
__device__ __forceinline__ bool pll_chunk_ok(const PllProof& pf, const PllRegs& r, double w, int chunk) {
    return (pf.emax < PLL_EMAX) & (pf.split == 0u) & (pf.tie > pllm::TIE_MIN) &
           (__builtin_fabs(r.ip.y) < 0x1p28f) & (__builtin_fabs(r.ip.x) < 0x1p20f) &
           (TAB || (pf.tmax < 0x1p30f));
}

// the f64 libm results of the reference step (pll.cpp:39, :49-50), out of line: only the rare
// fallbacks call them, and the unrolled redo chunks stay small. They return glibc's value RN64(f)
// from double-double evaluations (pll_math.h), not the device libm's, which differs from glibc by
// 1-2 ulps on 3-27% of inputs -- enough to flip an f32 rounding on the near-midpoint inputs that
// reach a fallback. |t| >= 2^30 (a stream past ~25 min for the 114 kHz PLL) reduces by
// Payne-Hanek in double-double (pll_math.h dd_reduce_f32_large); only inf/NaN keep the device libm.
__device__ __noinline__ float pll_atan2_ref(float eQ, float eI) {
    return (float)pllm::dd_atan2_f32(eQ, eI, atan2((double)eQ, (double)eI));
}
__device__ __noinline__ void pll_sincos_ref(float t, double* s, double* c) {
    if (__builtin_fabs(t) <= 3.4028234663852886e38f)
        pllm::dd_sincos_f32(t, s, c);
    else
        sincos((double)t, s, c);
}

// split accumulator of the phase detector's rounding test, per step: acc | (lo ^ hi) as ONE
// v_bitop3_b32 (truth table 0xF6 = s0 | (s1 ^ s2)). Written out because the compiler otherwise
// keeps all 16 (lo, hi) pairs of a chunk alive and compares them at its end.
__device__ __forceinline__ uint32_t or_xor(uint32_t acc, uint32_t lo, uint32_t hi) {
    uint32_t d;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0xf6" : "=v"(d) : "v"(acc), "v"(lo), "v"(hi));
    return d;
}

// tie accumulator: min(acc, tc, ts) as one v_min3_u32 (the compiler otherwise pairs the keys of
// consecutive steps into a v_min_u32 + v_min3_u32 tree)
__device__ __forceinline__ uint32_t min3_u32(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t d;
    asm("v_min3_u32 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c));
    return d;
}

// One step of pll.cpp:36-50. CHECKED: every result the fast path cannot prove is recomputed
// with the f64 libm exactly as the reference (used for chunk redo and short tails).
template <bool CHECKED, bool TAB>
__device__ __forceinline__ void pll_step(PllRegs& r, float x, double rx, float Kp, float Ki, double w, double wt,
                                         float& t_out, PllProof& pf) {
    // pll.cpp:36-37 in the reduced frame, as one packed multiply: x * (fbI, -fbQ)
    typedef float f2v __attribute__((ext_vector_type(2)));
    const f2v fb = {r.fbI, -r.fbQ};
    const f2v ee = x * fb;
    const float eI0 = ee.x, eQ0 = ee.y;
    // pll.cpp:39: atan2(eQ, eI) = base + Y/X (pll_math.h phase_detect2), rounding proven below
    const double base = pllm::base_angle_n(pllm::lo_word(rx), r.nq1, r.b, r.mr);
    const double Y = pllm::fma_((double)eI0, r.s, (double)eQ0 * r.c);
    const double ed = pllm::fma_(Y, rx, base);
    // hi (the value used) first: the loop filter's product can issue while lo, the range and the
    // split test fill its wait states
    const float hi = (float)(ed + pllm::EPS_ABS_E2);
    const float lo = (float)(ed - pllm::EPS_ABS_E2);
    float e = hi;                                             // = RN32(ed) whenever lo == hi
    if (CHECKED) {
        if (!((__builtin_fabs(ed) < PLL_EMAX) && lo == hi)) {
            float a = eI0, b = -eQ0;                          // eI - i eQ = i^q (eI0 - i eQ0)
            pllm::rot_q(1u - r.nq1, a, b);
            e = pll_atan2_ref(-b, a);                         // pll.cpp:39
        }
    } else {
        pf.emax = fmax(pf.emax, __builtin_fabs(ed));
        pf.split = or_xor(pf.split, __builtin_bit_cast(uint32_t, lo), __builtin_bit_cast(uint32_t, hi));
    }
    // pll.cpp:41-42: integ += Ki e; phaseEst = (phaseEst + Kp e) + integ, as scalar f32 (5 VALU,
    // no hazard wait states after packed-f32 results: +1.2 % against the packed form,
    // profiles/r02/ab_pll_lf.txt)
    {
        const float ki_e = Ki * e;
        const float integ = r.ip.x + ki_e;
        r.ip.y = (r.ip.y + Kp * e) + integ;
        r.ip.x = integ;
    }
    float t;
    if (TAB) {                                                // wt = w * trigOffset, tabulated
        t = (float)(wt + (double)r.ip.y);                     // pll.cpp:47
    } else {
        r.toff += 1.0;                                        // pll.cpp:46
        t = (float)(w * r.toff + (double)r.ip.y);             // pll.cpp:47
    }
    const pllm::SinCosRN sc = pllm::sincos_rn(t);
    r.c = sc.cr;
    r.s = sc.sr;
    r.mr = -sc.r;
    r.nq1 = sc.nq1;
    r.b = sc.b;
    r.fbI = (float)sc.cr;                                     // pll.cpp:49-50, reduced frame
    r.fbQ = (float)sc.sr;
    if (CHECKED) {
        const bool in_range = __builtin_fabs((double)t) < pllm::T_MAX;
        if (!(in_range && sc.tie > pllm::TIE_MIN)) {
            double sv, cv;
            pll_sincos_ref(t, &sv, &cv);
            pllm::rot_q(r.nq1 - 1u, cv, sv);                  // into the reduced frame, exactly
            r.fbI = (float)cv;
            r.fbQ = (float)sv;
            r.c = cv;
            r.s = sv;
            if (!in_range) r.mr = __builtin_nan("");
        }
    } else {
        pf.tie = min3_u32(pf.tie, sc.tc, sc.ts);
        if (!TAB) pf.tmax = fmaxf(pf.tmax, __builtin_fabsf(t));
    }
    t_out = t;
}

#ifndef SDR_PLL_CHUNK
#define SDR_PLL_CHUNK 16
#endif
constexpr int PLL_CHUNK = SDR_PLL_CHUNK;
#ifndef SDR_PLL_NBUF
#define SDR_PLL_NBUF 2
#endif
constexpr int PLL_NBUF = SDR_PLL_NBUF;   // register buffers of inputs (prefetch distance NBUF - 1 chunks)

// VEC: x / rx rows and the t buffer are 16-byte aligned with strides that are multiples of 4
// (x, t) and 2 (rx), so a chunk's inputs are prefetched with 16-byte loads one chunk ahead and
// the 16 phases are stored with 16-byte stores -- the unrolled chunk itself touches no memory.
// One lane per channel runs the n serial steps of one PllJob.
// TAB: every lane of the wave has the same trigOffset (a context's channels advance together), so
// w * trigOffset of every step comes from a table the wave builds in LDS up front (pll.cpp:46-47
// evaluated once per step index instead of once per channel and step).
template <bool VEC, bool TAB>
__device__ __forceinline__ void pll_run(const PllJob& jb, int n, int ch, const double* __restrict__ wtab) {
    const float* __restrict__ in = jb.in;
    const size_t in_stride = jb.in_stride, t_stride = jb.t_stride, out_stride = jb.out_stride;
    float* __restrict__ tbuf = jb.tbuf;
    float* __restrict__ out = jb.out;
    sdr_pll_state* __restrict__ st = jb.st;
    const float freq = jb.freq, Fs = jb.Fs, normBandwidth = jb.bw;
    const float Cp = 2.666;
    const float Ci = 3.555;
    const float Kp = normBandwidth * Cp;
    const float Ki = normBandwidth * normBandwidth * Ci;
    const double w = 2 * 3.14159265358979323846 * (freq / Fs);
    const sdr_pll_state s0 = st[ch];
    const float* x = in + (size_t)ch * in_stride;
    const double* rxp = jb.rx + (size_t)ch * jb.rx_stride;
    float* tb = tbuf + (size_t)ch * t_stride;
    if (!jb.prev_out) out[(size_t)ch * out_stride] = s0.lastCarrier;   // pll.cpp:18
    PllRegs r = pll_load(s0, w);
    // Chunks rotate through PLL_NBUF register buffers: chunk c computes from buffer c % NBUF, stores
    // its phases, then refills that buffer with chunk c + NBUF. A chunk's inputs are thus loaded
    // NBUF - 1 chunks ahead and, being issued after the previous chunk's stores, never make a
    // wait include those stores (vmcnt counts loads and stores in issue order). The main loop
    // covers a multiple of NBUF chunks; the rest (< NBUF chunks + n % CHUNK) runs checked steps.
    constexpr int C = PLL_CHUNK, NB = PLL_NBUF;
    const int nchunks = n / C;
    const int nmain = nchunks - nchunks % NB;
    float xb[NB][C];
    double rb[NB][C];
    auto load_chunk = [&](float* dx, double* dr, int i0) {
        if (VEC) {
#pragma unroll
            for (int k = 0; k < C / 4; k++) {
                const float4 v = reinterpret_cast<const float4*>(x + i0)[k];
                dx[4 * k] = v.x; dx[4 * k + 1] = v.y; dx[4 * k + 2] = v.z; dx[4 * k + 3] = v.w;
            }
#pragma unroll
            for (int k = 0; k < C / 2; k++) {
                const double2 v = reinterpret_cast<const double2*>(rxp + i0)[k];
                dr[2 * k] = v.x; dr[2 * k + 1] = v.y;
            }
        } else {
#pragma unroll
            for (int k = 0; k < C; k++) {
                dx[k] = x[i0 + k];
                dr[k] = rxp[i0 + k];
            }
        }
    };
    if (nmain > 0) {
#pragma unroll
        for (int u = 0; u < NB; u++) load_chunk(xb[u], rb[u], u * C);
    }
    for (int c0 = 0; c0 < nmain; c0 += NB) {
#pragma unroll
        for (int u = 0; u < NB; u++) {
            const int i0 = (c0 + u) * C;
            double wv[C];
            if (TAB) {
#pragma unroll
                for (int k = 0; k < C / 2; k++) {
                    const double2 v = reinterpret_cast<const double2*>(wtab + i0)[k];
                    wv[2 * k] = v.x; wv[2 * k + 1] = v.y;
                }
            }
            const PllRegs snap = r;
            PllProof pf;
            float tv[C];
#pragma unroll
            for (int j = 0; j < C; j++)
                pll_step<false, TAB>(r, xb[u][j], rb[u][j], Kp, Ki, w, TAB ? wv[j] : 0.0, tv[j], pf);
            const bool chunk_ok = pll_chunk_ok<TAB>(pf, r, w, C);
#if SDR_PLL_COUNT
            pll_count_chunk(chunk_ok);
#endif
            if (!chunk_ok) {
                r = snap;
#pragma unroll
                for (int j = 0; j < C; j++)
                    pll_step<true, TAB>(r, xb[u][j], rb[u][j], Kp, Ki, w, TAB ? wv[j] : 0.0, tv[j], pf);
            }
            if (VEC) {
#pragma unroll
                for (int k = 0; k < C / 4; k++)
                    reinterpret_cast<float4*>(tb + i0)[k] = make_float4(tv[4 * k], tv[4 * k + 1], tv[4 * k + 2], tv[4 * k + 3]);
            } else {
#pragma unroll
                for (int k = 0; k < C; k++) tb[i0 + k] = tv[k];
            }
            // refill (the last refills re-read the final chunk: harmless, keeps the loop branch-free)
            load_chunk(xb[u], rb[u], min(c0 + u + NB, nmain - 1) * C);
        }
    }
    {
        // the rest (< NB chunks + n % C steps), checked, from register buffers loaded one piece
        // ahead (one exposed memory latency for the whole rest instead of one per step)
        PllProof pf;
        const int i_rest = nmain * C;
        float xr[C];
        double rr[C], wr[C];
        auto load_rest = [&](int i0) {
#pragma unroll
            for (int k = 0; k < C; k++) {
                const int i = min(i0 + k, n - 1);
                xr[k] = x[i];
                rr[k] = rxp[i];
                wr[k] = TAB ? wtab[i] : 0.0;
            }
        };
        if (i_rest < n) load_rest(i_rest);
        for (int i0 = i_rest; i0 < n; i0 += C) {
            float xc[C];
            double rc[C], wc[C];
#pragma unroll
            for (int k = 0; k < C; k++) { xc[k] = xr[k]; rc[k] = rr[k]; wc[k] = wr[k]; }
            if (i0 + C < n) load_rest(i0 + C);
#pragma unroll
            for (int k = 0; k < C; k++)
                if (i0 + k < n) pll_step<true, TAB>(r, xc[k], rc[k], Kp, Ki, w, wc[k], tb[i0 + k], pf);
        }
    }
    if (TAB) r.toff = s0.trigOffset + (double)n;               // pll.cpp:46, n times (exact)
    // every field but lastCarrier (k_nco_out's); the feedback back in the frame of t
    pllm::rot_q(1u - r.nq1, r.fbI, r.fbQ);
    st[ch].feedbackI = r.fbI;
    st[ch].feedbackQ = r.fbQ;
    st[ch].integrator = r.ip.x;
    st[ch].phaseEst = r.ip.y;
    st[ch].trigOffset = r.toff;
}

// ------------------------------------------------------------------------------------------
// The PLL step on a LANE PAIR (SPLIT). One lane's step issues ~50 instructions, one per quad-cycle
// for a lone wave, and half of them are the two kernels of cos r and sin r and their roundings and
// tie keys. Here lanes 2k and 2k+1 both run channel k: the even lane (A) evaluates cos r, the odd
// lane (B) sin r -- the same instruction stream, f = u + z u P(z) with per-lane coefficients
// (A: u = 1, P = the cos kernel's; B: u = r, P = fdlibm's sin kernel) -- and the phase detector
// takes the partner's value across the pair with DPP:
//   g = RN32(xs * fb_partner)   A: xs = -x, RN32(-x fQ0) = eQ0    B: xs = x, RN32(x fI0) = eI0
//   q = g * f_own               A: eQ0 c                          B: eI0 s
//   Y = q + q_partner           eI0 s + eQ0 c on both lanes (the same two f64 products, one sum)
// (pll.cpp:36-39 in the reduced frame, pll_math.h phase_detect2; xs = -x comes from the producer:
// the sign of eQ0 cannot otherwise enter one lane only). e, the loop filter, t, the reduction and
// the proof accumulators are identical on both lanes; the e bracket is proven half on each lane
// (A: RN32(ed - eps) = e, B: RN32(ed + eps) = e) and each lane proves its own f32 rounding tie, so
// a chunk is accepted only when both lanes of the pair accept it. A redo runs the full checked
// step (pll_step<true>) on both lanes of the pair with the exchanged values.
// ------------------------------------------------------------------------------------------
struct SplitRegs {
    double f;        // A: cos r, B: sin r (f64)
    float fb;        // RN32(f): A: fI0, B: fQ0 (reduced frame)
    f32x2 ip;        // {integrator, phaseEst}
    double toff;
    double mr;       // -r
    uint32_t nq1, b; // 1 - q, [r < 0]
};

struct SplitLane {
    double c0, c1, c2, c3, c4, c5;   // P(z) = c0 + c1 z + ... + c5 z^5
    double k1, k0;                   // u = k1 r + k0
    double eps;                      // the end of the e bracket this lane proves
    bool a;                          // even lane: cos
};

__device__ __forceinline__ SplitLane split_lane() {
    SplitLane L;
    L.a = (threadIdx.x & 1) == 0;
    if (L.a) {   // cos r = 1 + z (-1/2 + C1 z + ... + C5 z^5) (pll_math.h, refitted)
        L.c0 = -0.5; L.c1 = pllm::C1; L.c2 = pllm::C2; L.c3 = pllm::C3; L.c4 = pllm::C4; L.c5 = pllm::C5;
        L.k1 = 0.0; L.k0 = 1.0; L.eps = -pllm::EPS_ABS_E2;
    } else {     // sin r = r + r z (S1 + S2 z + ... + S6 z^5) (fdlibm k_sin)
        L.c0 = pllm::S1; L.c1 = pllm::S2; L.c2 = pllm::S3; L.c3 = pllm::S4; L.c4 = pllm::S5; L.c5 = pllm::S6;
        L.k1 = 1.0; L.k0 = 0.0; L.eps = pllm::EPS_ABS_E2;
    }
    return L;
}

// value of the other lane of the pair (DPP quad_perm [1,0,3,2])
// (bound_ctrl set: both lanes of a pair are always active, and it lets the compiler fold the move
// into the consumer as a DPP source, v_mul_f32_dpp)
__device__ __forceinline__ float pair_swap(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0xB1, 0xF, 0xF, true));
}
__device__ __forceinline__ double pair_swap(double v) {
    const uint64_t u = __builtin_bit_cast(uint64_t, v);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)u, 0xB1, 0xF, 0xF, false);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)(u >> 32), 0xB1, 0xF, 0xF, false);
    return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}

__device__ __forceinline__ PllRegs split_to_full(const SplitRegs& s, bool a) {
    PllRegs r;
    const double fo = pair_swap(s.f);
    const float fbo = pair_swap(s.fb);
    r.c = a ? s.f : fo;
    r.s = a ? fo : s.f;
    r.fbI = a ? s.fb : fbo;
    r.fbQ = a ? fbo : s.fb;
    r.ip = s.ip;
    r.toff = s.toff;
    r.mr = s.mr;
    r.nq1 = s.nq1;
    r.b = s.b;
    return r;
}

__device__ __forceinline__ SplitRegs full_to_split(const PllRegs& r, bool a) {
    SplitRegs s;
    s.f = a ? r.c : r.s;
    s.fb = a ? r.fbI : r.fbQ;
    s.ip = r.ip;
    s.toff = r.toff;
    s.mr = r.mr;
    s.nq1 = r.nq1;
    s.b = r.b;
    return s;
}

template <bool TAB>
__device__ __forceinline__ void pll_step_split(SplitRegs& r, float xs, double rx, float Kp, float Ki, double w,
                                               double wt, float& t_out, PllProof& pf, const SplitLane& L) {
    // pll.cpp:36-39 across the pair (see above)
    const float g = xs * pair_swap(r.fb);
    const double q = (double)g * r.f;
    const double base = pllm::base_angle_n(pllm::lo_word(rx), r.nq1, r.b, r.mr);
    // (ed = base + rx qA + rx qB, own product first, is one dependent level shorter but needs both
    // bracket ends per lane: 2 instructions more, slower, profiles/r03/ab_pll_split.txt)
    const double Y = q + pair_swap(q);
    const double ed = pllm::fma_(Y, rx, base);
    const float e = (float)ed;                                     // = RN32(atan2) when proven
    pf.split = or_xor(pf.split, __builtin_bit_cast(uint32_t, (float)(ed + L.eps)), __builtin_bit_cast(uint32_t, e));
    pf.emaxf = fmaxf(pf.emaxf, __builtin_fabsf(e));               // f32: two steps per v_max3_f32
    {   // pll.cpp:41-42 (scalar f32, this unit is built without SLP: profiles/r03/ab_pll_split3.txt)
        const float ki_e = Ki * e, kp_e = Kp * e;
        const float integ = r.ip.x + ki_e;
        r.ip.y = (r.ip.y + kp_e) + integ;
        r.ip.x = integ;
    }
    float t;
    if (TAB) {
        t = (float)(wt + (double)r.ip.y);                         // pll.cpp:47
    } else {
        r.toff += 1.0;                                             // pll.cpp:46
        t = (float)(w * r.toff + (double)r.ip.y);
    }
    // reduction (pll_math.h sincos_rn) and this lane's kernel
    const double x = (double)t;
    const double kdp = pllm::fma_(x, -pllm::TWO_OVER_PI, pllm::MAGIC1);
    const double kdn = kdp - pllm::MAGIC1;
    const double rr = pllm::fma_(kdn, pllm::PIO2_LO, pllm::fma_(kdn, pllm::PIO2_HI, x));
    r.nq1 = (uint32_t)__builtin_bit_cast(uint64_t, kdp);
    r.b = (uint32_t)(__builtin_bit_cast(uint64_t, rr) >> 63);
    r.mr = -rr;
    const double z = rr * rr;
    const double u = pllm::fma_(rr, L.k1, L.k0);
    // Horner: one instruction fewer than Estrin (no z^2), two dependent levels more; faster than
    // Estrin and than a two-level form (profiles/r03/ab_pll_split3.txt)
    // (Estrin, two dependent levels shorter for two multiplies more, measured again in round 5:
    // 212 -> 224 cycles per step, with or without s_setprio; profiles/r05/ab_pll_est.txt)
    double P = pllm::fma_(z, L.c5, L.c4);
    P = pllm::fma_(z, P, L.c3);
    P = pllm::fma_(z, P, L.c2);
    P = pllm::fma_(z, P, L.c1);
    P = pllm::fma_(z, P, L.c0);
    r.f = pllm::fma_(z * u, P, u);
    r.fb = (float)r.f;                                             // pll.cpp:49-50, reduced frame
    pf.tie = min(pf.tie, pllm::tie_key64(r.f));                   // this lane's rounding (pll_math.h)
    if (!TAB) pf.tmax = fmaxf(pf.tmax, __builtin_fabsf(t));
    t_out = t;
}

constexpr unsigned long long PLL_WAIT_TICKS = 500000000ull;   // 5 s of s_memrealtime (persistent waits)

// Input gate of the persistent PLL's first block (the pipeline fill, sdr_frontend_pre_parts): the
// producer publishes the block's input in parts (sub = sub_base + FIR tiles published, each tile
// `tile` samples) before the whole-block flag; the waves start on the first part and wait before
// loading samples past what has been published. avail = samples published so far (wave-uniform,
// scalar): n for every other block, so the check per chunk never waits there.
struct InGate {
    const uint32_t* flag;
    const uint32_t* sub;
    uint32_t* err;
    uint32_t want, sub_base;
    int tile, n, avail;
    unsigned long long t0;
};

// samples [0, i_end) must be published: poll (relaxed) the whole-block flag and the part counter,
// acquire once; bounded like the launch's other waits (an expired wait records the error and lets
// the wave compute on: the post stages then poison the block)
__device__ __forceinline__ void gate_wait(InGate& g, int i_end) {
    if (i_end <= g.avail) return;
    while (true) {
        const uint32_t f = __hip_atomic_load(g.flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint32_t sb = __hip_atomic_load(g.sub, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        int av = (int32_t)(f - g.want) >= 0 ? g.n : (int)min((int32_t)(sb - g.sub_base), (int32_t)PLL_SUB_SCALE - 1) * g.tile;
        av = __builtin_amdgcn_readfirstlane(min(max(av, 0), g.n));
        if (av >= i_end) {
            g.avail = av;
            break;
        }
        __builtin_amdgcn_s_sleep(2);
        if (__builtin_amdgcn_s_memrealtime() - g.t0 > PLL_WAIT_TICKS) {
            if (threadIdx.x == 0) __hip_atomic_fetch_or(g.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            g.avail = g.n;
            break;
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
}

// pll_run on lane pairs: ch = channel of the pair, xneg = -x row of the producer (lane A's input).
// GATE: the input arrives in parts (*gate); a separate instantiation, so the blocks that need no
// gate run the loop without its checks
template <bool VEC, bool TAB, bool GATE = false>
__device__ __forceinline__ void pll_run_split(const PllJob& jb, int n, int ch, const double* __restrict__ wtab,
                                              InGate* gate = nullptr) {
    const SplitLane L = split_lane();
    const size_t in_stride = jb.in_stride, t_stride = jb.t_stride, out_stride = jb.out_stride;
    sdr_pll_state* __restrict__ st = jb.st;
    const float freq = jb.freq, Fs = jb.Fs, normBandwidth = jb.bw;
    const float Cp = 2.666;
    const float Ci = 3.555;
    const float Kp = normBandwidth * Cp;
    const float Ki = normBandwidth * normBandwidth * Ci;
    const double w = 2 * 3.14159265358979323846 * (freq / Fs);
    const sdr_pll_state s0 = st[ch];
    const float* xpos = jb.in + (size_t)ch * in_stride;
    const float* xs = L.a ? jb.in_neg + (size_t)ch * jb.neg_stride : xpos;   // lane A: -x
    const double* rxp = jb.rx + (size_t)ch * jb.rx_stride;
    float* tb = jb.tbuf + (size_t)ch * t_stride;
    if (!jb.prev_out && L.a) jb.out[(size_t)ch * out_stride] = s0.lastCarrier;   // pll.cpp:18
    SplitRegs r = full_to_split(pll_load(s0, w), L.a);
    constexpr int C = PLL_CHUNK, NB = PLL_NBUF;
    const int nchunks = n / C;
    const int nmain = nchunks - nchunks % NB;
    float xb[NB][C];
    double rb[NB][C];
    auto load_chunk = [&](float* dx, double* dr, int i0) {
        if (VEC) {
#pragma unroll
            for (int k = 0; k < C / 4; k++) {
                const float4 v = reinterpret_cast<const float4*>(xs + i0)[k];
                dx[4 * k] = v.x; dx[4 * k + 1] = v.y; dx[4 * k + 2] = v.z; dx[4 * k + 3] = v.w;
            }
#pragma unroll
            for (int k = 0; k < C / 2; k++) {
                const double2 v = reinterpret_cast<const double2*>(rxp + i0)[k];
                dr[2 * k] = v.x; dr[2 * k + 1] = v.y;
            }
        } else {
#pragma unroll
            for (int k = 0; k < C; k++) {
                dx[k] = xs[i0 + k];
                dr[k] = rxp[i0 + k];
            }
        }
    };
    if (nmain > 0) {
        if (GATE) gate_wait(*gate, NB * C);
#pragma unroll
        for (int u = 0; u < NB; u++) load_chunk(xb[u], rb[u], u * C);
    }
    for (int c0 = 0; c0 < nmain; c0 += NB) {
#pragma unroll
        for (int u = 0; u < NB; u++) {
            const int i0 = (c0 + u) * C;
            double wv[C];
            if (TAB) {
#pragma unroll
                for (int k = 0; k < C / 2; k++) {
                    const double2 v = reinterpret_cast<const double2*>(wtab + i0)[k];
                    wv[2 * k] = v.x; wv[2 * k + 1] = v.y;
                }
            }
            const SplitRegs snap = r;
            PllProof pf;
            float tv[C];
#pragma unroll
            for (int j = 0; j < C; j++)
                pll_step_split<TAB>(r, xb[u][j], rb[u][j], Kp, Ki, w, TAB ? wv[j] : 0.0, tv[j], pf, L);
            // this lane's proof: its half of the e bracket, the e range, its own rounding ties, and
            // the state range (a NaN from an invalid input fails it)
            const bool ok = (pf.emaxf < PLL_EMAX_F) & (pf.split == 0u) & (pf.tie > pllm::TIE_MIN) &
                            (__builtin_fabs(r.ip.y) < 0x1p28f) & (__builtin_fabs(r.ip.x) < 0x1p20f) &
                            (TAB || (pf.tmax < 0x1p30f));
#if SDR_PLL_COUNT
            pll_count_chunk(ok);
            pll_count_reasons(!(pf.emaxf < PLL_EMAX_F), pf.split != 0u, !(pf.tie > pllm::TIE_MIN),
                              !((__builtin_fabs(r.ip.y) < 0x1p28f) & (__builtin_fabs(r.ip.x) < 0x1p20f)));
#endif
            // the partner's verdict, read with every lane of the pair active (under `ok && ...` the
            // exchange would sit in a branch, and a lane reading a disabled partner keeps its own value)
            const int ok_partner = __builtin_amdgcn_mov_dpp((int)ok, 0xB1, 0xF, 0xF, false);
            const bool pair_ok = ok & (ok_partner != 0);
            if (!pair_ok) {
                PllRegs full = split_to_full(snap, L.a);
#pragma unroll
                for (int j = 0; j < C; j++)
                    pll_step<true, TAB>(full, L.a ? -xb[u][j] : xb[u][j], rb[u][j], Kp, Ki, w, TAB ? wv[j] : 0.0,
                                        tv[j], pf);
                r = full_to_split(full, L.a);
            }
            if (VEC) {
#pragma unroll
                for (int k = 0; k < C / 4; k++)
                    reinterpret_cast<float4*>(tb + i0)[k] = make_float4(tv[4 * k], tv[4 * k + 1], tv[4 * k + 2], tv[4 * k + 3]);
            } else {
#pragma unroll
                for (int k = 0; k < C; k++) tb[i0 + k] = tv[k];
            }
            if (GATE) gate_wait(*gate, (min(c0 + u + NB, nmain - 1) + 1) * C);
            load_chunk(xb[u], rb[u], min(c0 + u + NB, nmain - 1) * C);
        }
    }
    PllRegs full = split_to_full(r, L.a);
    {
        // the rest (< NB chunks + n % C steps): full checked steps on both lanes of the pair
        PllProof pf;
        const int i_rest = nmain * C;
        float xr[C];
        double rr[C], wr[C];
        auto load_rest = [&](int i0) {
#pragma unroll
            for (int k = 0; k < C; k++) {
                const int i = min(i0 + k, n - 1);
                xr[k] = xpos[i];
                rr[k] = rxp[i];
                wr[k] = TAB ? wtab[i] : 0.0;
            }
        };
        if (GATE) gate_wait(*gate, n);
        if (i_rest < n) load_rest(i_rest);
        for (int i0 = i_rest; i0 < n; i0 += C) {
            float xc[C];
            double rc[C], wc[C];
#pragma unroll
            for (int k = 0; k < C; k++) { xc[k] = xr[k]; rc[k] = rr[k]; wc[k] = wr[k]; }
            if (i0 + C < n) load_rest(i0 + C);
#pragma unroll
            for (int k = 0; k < C; k++)
                if (i0 + k < n) pll_step<true, TAB>(full, xc[k], rc[k], Kp, Ki, w, wc[k], tb[i0 + k], pf);
        }
    }
    if (TAB) full.toff = s0.trigOffset + (double)n;            // pll.cpp:46, n times (exact)
    if (L.a) {   // every field but lastCarrier (the NCO's); the feedback back in the frame of t
        pllm::rot_q(1u - full.nq1, full.fbI, full.fbQ);
        st[ch].feedbackI = full.fbI;
        st[ch].feedbackQ = full.fbQ;
        st[ch].integrator = full.ip.x;
        st[ch].phaseEst = full.ip.y;
        st[ch].trigOffset = full.toff;
    }
}

// ------------------------------------------------------------------------------------------
// COAL: the lane-pair loop for waves that share a CU (capacity launches, more than one PLL wave per
// CU). Per-lane row loads -- every lane reads 16 bytes of its own row, so each wave-instruction
// touches 64 cache lines -- saturate the CU's texture addresser once several waves issue them
// (209 -> 236 -> ~390 cycles per step at 1, 2, 4 waves per CU). Here a chunk's inputs
// reach LDS by LDS-DMA (global_load_lds_dwordx4) in line-shaped pieces -- 16 x-rows x 64 B or 8
// rx-rows x 128 B per instruction -- two chunks ahead into a ring of three LDS buffers, each lane then
// reads its own rows from LDS, and the 16 phases go out the same way in reverse (own row into LDS,
// line-shaped pieces out). The
// one-wave-per-CU path (the headline) keeps the register prefetch, which needs no LDS round trip.
// Layout of one buffer: pieces of 1 KiB at a 1040-byte pitch (a 16-byte rotation per piece keeps
// the own-row reads free of bank conflicts): 6 pieces per buffer (COAL_BUF), pieces 0-1 the x rows of
// channels q with q % 2 = k (lane A, which runs on -x, flips the sign bit as it reads), pieces 2-5 the
// rx rows q with q % 4 = k (piece 2 + k); a ring of COAL_RING = 3 buffers per wave, so a chunk's 6
// DMA pieces are in flight while the own-row reads wait for the older chunk's (vmcnt(6)). Every lane
// of the wave must run the loop (all 32 channels valid).
// ------------------------------------------------------------------------------------------
constexpr int COAL_PIECE = 1040;
constexpr int COAL_BUF = 6 * COAL_PIECE;              // pieces 0-1: x rows, 2-5: rx rows
// LDS buffers per wave: the DMA runs two chunks ahead (a ring of 2, one chunk ahead: 261-264 against
// 258-261 cycles per step, profiles/r05/coal/ring/)
constexpr int COAL_RING = 3;
constexpr int COAL_TROW = 80;                         // t staging: 32 rows of 64 B at an 80-byte pitch

template <bool TAB, bool GATE>
__device__ __forceinline__ void pll_run_split_coal(const PllJob& jb, int n, int ch, const double* __restrict__ wtab,
                                                   InGate* gate, uint8_t* __restrict__ lbuf,
                                                   uint8_t* __restrict__ ltst) {
    const SplitLane L = split_lane();
    const int lane = threadIdx.x & 63;
    const int chw0 = ch - (lane >> 1);                 // the wave's first channel
    const size_t t_stride = jb.t_stride, out_stride = jb.out_stride;
    sdr_pll_state* __restrict__ st = jb.st;
    const float freq = jb.freq, Fs = jb.Fs, normBandwidth = jb.bw;
    const float Cp = 2.666;
    const float Ci = 3.555;
    const float Kp = normBandwidth * Cp;
    const float Ki = normBandwidth * normBandwidth * Ci;
    const double w = 2 * 3.14159265358979323846 * (freq / Fs);
    const sdr_pll_state s0 = st[ch];
    const float* xpos = jb.in + (size_t)ch * jb.in_stride;
    const double* rxp = jb.rx + (size_t)ch * jb.rx_stride;
    float* tb = jb.tbuf + (size_t)ch * t_stride;
    if (!jb.prev_out && L.a) jb.out[(size_t)ch * out_stride] = s0.lastCarrier;   // pll.cpp:18
    SplitRegs r = full_to_split(pll_load(s0, w), L.a);
    constexpr int C = PLL_CHUNK;
    static_assert(C == 16, "COAL pieces: 16 samples per row and chunk");
    const int nchunks = n / C;
    const int nmain = nchunks - nchunks % 2;
    // this lane's pieces: x-row 4 (lane / 4) + k (even rows: -x of channel row / 2, odd: x), floats
    // 4 (lane % 4) ..; rx row 4 (lane / 8) + k, doubles 2 (lane % 8) ..
    // the x rows only (channel row 2 (lane / 4) + k in piece k; lane A flips the sign on the read):
    // 6 pieces per chunk instead of 8 with the -x rows, 262-267 -> 260-263 cycles per step
    // (profiles/r05/coal/xonly/)
    constexpr int NXP = 2;
    const float* xsrc[NXP];
#pragma unroll
    for (int k = 0; k < NXP; k++)
        xsrc[k] = jb.in + (size_t)(chw0 + 2 * (lane >> 2) + k) * jb.in_stride + 4 * (lane & 3);
    const double* rsrc[4];
#pragma unroll
    for (int k = 0; k < 4; k++)
        rsrc[k] = jb.rx + (size_t)(chw0 + 4 * (lane >> 3) + k) * jb.rx_stride + 2 * (lane & 7);
    auto issue = [&](int b, int i0) {                  // chunk at sample i0 -> buffer b (LDS-DMA)
        uint8_t* base = lbuf + b * COAL_BUF;
#pragma unroll
        for (int k = 0; k < NXP; k++)
            __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(xsrc[k] + i0), base + k * COAL_PIECE, 16, 0, 0);
#pragma unroll
        for (int k = 0; k < 4; k++)
            __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(rsrc[k] + i0), base + (2 + k) * COAL_PIECE,
                                             16, 0, 0);
    };
    float xb[C];
    double rb[C];
    // this lane's rows of buffer b once its DMA has landed: with a ring of 3 the next chunk's 6 pieces
    // (issued after it) may still be in flight; every chunk issues exactly 6 (the last ones re-read
    // chunk nmain - 1 into spent buffers), so the count is exact
    auto take = [&](int b) {
        asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
        const uint8_t* base = lbuf + b * COAL_BUF;
        const int q = lane >> 1;
        const uint8_t* xr = base + (q & 1) * COAL_PIECE + (q >> 1) * 64;
        const uint32_t flip = L.a ? 0x80000000u : 0u;      // lane A: -x (exact)
        const uint8_t* rr = base + (2 + (q & 3)) * COAL_PIECE + (q >> 2) * 128;
#pragma unroll
        for (int p = 0; p < 4; p++) {
            const uint4 v = *reinterpret_cast<const uint4*>(xr + 16 * p);
            xb[4 * p] = __builtin_bit_cast(float, v.x ^ flip);
            xb[4 * p + 1] = __builtin_bit_cast(float, v.y ^ flip);
            xb[4 * p + 2] = __builtin_bit_cast(float, v.z ^ flip);
            xb[4 * p + 3] = __builtin_bit_cast(float, v.w ^ flip);
        }
#pragma unroll
        for (int p = 0; p < 8; p++) {
            const double2 v = *reinterpret_cast<const double2*>(rr + 16 * p);
            rb[2 * p] = v.x; rb[2 * p + 1] = v.y;
        }
    };
    static_assert(!GATE, "COAL: not on the fill block (its input arrives in parts)");
    if (nmain > 0) {
        issue(0, 0);
        issue(1, min(1, nmain - 1) * C);
        issue(2, min(2, nmain - 1) * C);
        take(0);
    }
    int bc = 0;                                         // buffer of chunk c (c mod COAL_RING)
    for (int c0 = 0; c0 < nmain; c0 += 2) {
#pragma unroll
        for (int u = 0; u < 2; u++) {
            const int c = c0 + u, i0 = c * C;
            const int bn = bc + 1 == COAL_RING ? 0 : bc + 1;   // buffer of chunk c + 1
            double wv[C];
            if (TAB) {
#pragma unroll
                for (int k = 0; k < C / 2; k++) {
                    const double2 v = reinterpret_cast<const double2*>(wtab + i0)[k];
                    wv[2 * k] = v.x; wv[2 * k + 1] = v.y;
                }
            }
            const SplitRegs snap = r;
            PllProof pf;
            float tv[C];
#pragma unroll
            for (int j = 0; j < C; j++)
                pll_step_split<TAB>(r, xb[j], rb[j], Kp, Ki, w, TAB ? wv[j] : 0.0, tv[j], pf, L);
            const bool ok = (pf.emaxf < PLL_EMAX_F) & (pf.split == 0u) & (pf.tie > pllm::TIE_MIN) &
                            (__builtin_fabs(r.ip.y) < 0x1p28f) & (__builtin_fabs(r.ip.x) < 0x1p20f) &
                            (TAB || (pf.tmax < 0x1p30f));
            const int ok_partner = __builtin_amdgcn_mov_dpp((int)ok, 0xB1, 0xF, 0xF, false);
            const bool pair_ok = ok & (ok_partner != 0);
            if (!pair_ok) {
                PllRegs full = split_to_full(snap, L.a);
#pragma unroll
                for (int j = 0; j < C; j++)
                    pll_step<true, TAB>(full, L.a ? -xb[j] : xb[j], rb[j], Kp, Ki, w, TAB ? wv[j] : 0.0, tv[j], pf);
                r = full_to_split(full, L.a);
            }
            // the next chunk's rows (its DMA went out a chunk ago), then this chunk's phases out: the
            // even lanes' rows (both lanes of a pair hold the same phases) into LDS, line-shaped
            // pieces back: lane l stores 16 B of channel row 16 k + l / 4
            if (c + 1 < nmain) take(bn);
            if (L.a) {
#pragma unroll
                for (int p = 0; p < 4; p++)
                    *reinterpret_cast<float4*>(ltst + (lane >> 1) * COAL_TROW + 16 * p) =
                        make_float4(tv[4 * p], tv[4 * p + 1], tv[4 * p + 2], tv[4 * p + 3]);
            }
#pragma unroll
            for (int k = 0; k < 2; k++) {
                const int q = 16 * k + (lane >> 2);
                const float4 v = *reinterpret_cast<const float4*>(ltst + q * COAL_TROW + 16 * (lane & 3));
                *reinterpret_cast<float4*>(jb.tbuf + (size_t)(chw0 + q) * t_stride + i0 + 4 * (lane & 3)) = v;
            }
            issue(bc, min(c + 3, nmain - 1) * C);          // into chunk c's spent buffer
            bc = bn;
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // spare pieces land before the buffers are reused
    PllRegs full = split_to_full(r, L.a);
    {
        // the rest (< 2 chunks + n % C steps): full checked steps on both lanes of the pair
        PllProof pf;
        const int i_rest = nmain * C;
        if (GATE) gate_wait(*gate, n);
        for (int i = i_rest; i < n; i++)
            pll_step<true, TAB>(full, xpos[i], rxp[i], Kp, Ki, w, TAB ? wtab[i] : 0.0, tb[i], pf);
    }
    if (TAB) full.toff = s0.trigOffset + (double)n;            // pll.cpp:46, n times (exact)
    if (L.a) {   // every field but lastCarrier (the NCO's); the feedback back in the frame of t
        pllm::rot_q(1u - full.nq1, full.fbI, full.fbQ);
        st[ch].feedbackI = full.fbI;
        st[ch].feedbackQ = full.fbQ;
        st[ch].integrator = full.ip.x;
        st[ch].phaseEst = full.ip.y;
        st[ch].trigOffset = full.toff;
    }
}

// VEC: x / rx rows and the t buffer are 16-byte aligned with strides that are multiples of 4
// (x, t) and 2 (rx), so a chunk's inputs are prefetched with 16-byte loads and the 16 phases are
// stored with 16-byte stores -- the unrolled chunk itself touches no memory.
// Dynamic LDS: n doubles when the launch allows the trigArg table (launch_plls), else none.
// SPLIT: two lanes per channel (pll_run_split), else one.
template <bool VEC, bool SPLIT>
__global__ __launch_bounds__(64) void k_pll(const PllJobs jobs, int n, int nch, int tab_ok) {
    extern __shared__ double wtab[];
    const int lg = blockIdx.x * blockDim.x + threadIdx.x;
    const int ch = SPLIT ? lg >> 1 : lg;                    // lane 0 always holds a channel
    const bool active = ch < nch;
    const PllJob& jb = jobs.j[blockIdx.y];
    // the serial PLL bounds every block-step: let its waves win issue arbitration on shared SIMDs
    __builtin_amdgcn_s_setprio(3);
    const double toff0 = active ? jb.st[ch].trigOffset : 0.0;
    const double w = 2 * 3.14159265358979323846 * (jb.freq / jb.Fs);
    // one wave per workgroup: the table is valid when all channels of the wave share trigOffset
    // and every w * trigOffset of the launch stays below 2^29 (so |t| < 2^30 whenever
    // |phaseEst| < 2^28). All 64 lanes build it, then the lanes without a channel leave.
    const double toff_l0 = __shfl(toff0, 0);
    const bool tab = tab_ok && __all(!active || toff0 == toff_l0) &&
                     __builtin_fabs(w) * (__builtin_fabs(toff_l0) + (double)n + 1.0) < PLL_TAB_WT_MAX;
    if (tab) {
        for (int k = threadIdx.x; k < n; k += 64) wtab[k] = w * (toff_l0 + (double)(k + 1));   // pll.cpp:46-47
        __syncthreads();
    }
    if (!active) return;
#if SDR_PLL_HWID
    const unsigned long long hw_c0 = __builtin_amdgcn_s_memtime(), hw_r0 = __builtin_amdgcn_s_memrealtime();
#endif
    if (SPLIT) {
        if (tab) pll_run_split<VEC, true>(jb, n, ch, wtab);
        else pll_run_split<VEC, false>(jb, n, ch, nullptr);
    } else {
        if (tab) pll_run<VEC, true>(jb, n, ch, wtab);
        else pll_run<VEC, false>(jb, n, ch, nullptr);
    }
#if SDR_PLL_HWID
    const unsigned long long hw_c1 = __builtin_amdgcn_s_memtime(), hw_r1 = __builtin_amdgcn_s_memrealtime();
    uint32_t hw_id, xcc_id;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw_id));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc_id));
    const int slot = (int)(blockIdx.y * gridDim.x + blockIdx.x);
    if (threadIdx.x == 0 && slot < PLL_HWID_SLOTS) {
        g_pll_hwid[slot][0] = hw_id;
        g_pll_hwid[slot][1] = xcc_id;
        g_pll_hwid[slot][2] = hw_c1 - hw_c0;
        g_pll_hwid[slot][3] = hw_r0;
        g_pll_hwid[slot][4] = hw_r1;
    }
#endif
}

// ------------------------------------------------------------------------------------------
// Persistent PLLs (sdr_plls_launch / _signal / _wait): one dispatch runs the PLLs of `nblocks`
// consecutive blocks, so consecutive blocks are not separated by a dispatch (the ~19 us gap
// between back-to-back k_pll launches). Before block j the waves wait, with an
// agent-scope acquire, for the front-end stream's flag (k_flag_store, dispatched after the
// pre-PLL kernels of that block); after it each wave adds 1 to a done counter with an
// agent-scope release, which the post stream waits on (k_flag_wait). hipStreamWriteValue32 is
// not used for the flag: in a first version its write overtook the still-running pre-PLL kernel
// (the first block of a launch, whose waves are already waiting, read inputs before they were
// complete), while a kernel dispatch starts only after its predecessor has completed. Blocks alternate
// the context's two buffer parities. Every wait is bounded: after PLL_WAIT_TICKS of the 100 MHz
// clock the launch records an error and completes its remaining blocks without computing, so no
// wave and no waiting stream can hang.
// ------------------------------------------------------------------------------------------

// WG waves per workgroup (1, or 4 to pack one wave per SIMD): the group shares one trigArg table in
// LDS (all channels of a context advance together, so one table serves every wave whose lanes share
// the group's trigOffset), its wave 0 polls the block flag, and two barriers per block keep the
// group's waves on the same block (the table is rebuilt only after every wave finished reading it).
template <bool VEC, bool SPLIT, int WG, bool COAL = false>
__global__ __launch_bounds__(64 * WG) void k_pll_multi(const PllJobs2 jobs, int n, int nch, int tab_ok, int nblocks,
                                                       const uint32_t* pre_flag, uint32_t pre_first,
                                                       uint32_t* done_ring, uint32_t* err,
                                                       unsigned long long* t_start, unsigned long long* t_end,
                                                       unsigned long long* t_cyc, const uint32_t* sub_flag,
                                                       uint32_t sub_base, int sub_tile) {
    static_assert(!COAL || (VEC && SPLIT), "COAL: the lane-pair loop with 16-byte rows");
    extern __shared__ double wtab[];
    __shared__ double sh_toff;
    __shared__ int sh_dead;
    // COAL: per wave a ring of COAL_RING (3) DMA buffers of 6 pieces and the phase staging rows
    // (pll_run_split_coal)
    __shared__ __attribute__((aligned(16))) uint8_t coal_buf[COAL ? WG * COAL_RING * COAL_BUF : 16];
    __shared__ __attribute__((aligned(16))) uint8_t coal_tst[COAL ? WG * 32 * COAL_TROW : 16];
    uint8_t* const my_buf = coal_buf + (COAL ? (threadIdx.x >> 6) * COAL_RING * COAL_BUF : 0);
    uint8_t* const my_tst = coal_tst + (COAL ? (threadIdx.x >> 6) * 32 * COAL_TROW : 0);
    const int lg = blockIdx.x * blockDim.x + threadIdx.x;
    const int ch = SPLIT ? lg >> 1 : lg;
    const bool active = ch < nch;
    const bool lane0 = (threadIdx.x & 63) == 0;
    __builtin_amdgcn_s_setprio(3);
    bool dead = false;                                 // uniform across the workgroup
#if SDR_PLL_WAVES
    unsigned long long dw_cyc = 0, dw_wait = 0, dw_blocks = 0, dw_spin = 0, dw_polls = 0, dw_ready = 0, dw_early = 0;
    if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) g_diag_flag = pre_flag;
#endif
    for (int j = 0; j < nblocks; j++) {
        const PllJob& jb = jobs.p[j & 1].j[blockIdx.y];   // p[0]: the parity of the launch's first block
        const uint32_t want = pre_first + (uint32_t)j + 1u;
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        // the first block may start on its first published part (SPLIT: the lane-pair PLL gates its
        // loads, InGate)
        const bool parts = SPLIT && j == 0 && sub_flag != nullptr;
        if (!dead) {
            // poll with relaxed loads and acquire once: an acquire load at agent scope invalidates
            // the wave's caches (on a multi-XCD device its XCD's L2) on every poll, which slowed the
            // kernels running beside the waiting waves 2-3x
#if SDR_PLL_WAVES
            const unsigned long long p0 = dw_polls;
#endif
            if (threadIdx.x < 64) {
                while ((int32_t)(__hip_atomic_load(pre_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - want) < 0 &&
                       !(parts && (int32_t)(__hip_atomic_load(sub_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) -
                                            sub_base) >= 1)) {
                    __builtin_amdgcn_s_sleep(4);
#if SDR_PLL_WAVES
                    dw_polls++;
#endif
                    if (__builtin_amdgcn_s_memrealtime() - t0 > PLL_WAIT_TICKS) {
                        dead = true;
                        break;
                    }
                }
            }
#if SDR_PLL_WAVES
            dw_spin += __builtin_amdgcn_s_memrealtime() - t0;
            dw_ready += dw_polls == p0 ? 1u : 0u;
            {
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                const unsigned long long tf = __hip_atomic_load(&g_flag_t[want & 63], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (tf != 0 && tf < t0) dw_early += t0 - tf;
            }
#endif
            if (WG > 1) {
                if (threadIdx.x == 0) sh_dead = dead ? 1 : 0;
                __syncthreads();
                dead = sh_dead != 0;
            }
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            if (dead && threadIdx.x == 0) __hip_atomic_fetch_or(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        unsigned long long c0 = 0, r0 = 0;   // this wave's shader-clock and 100 MHz stamps of the block
        if (!dead) {
            c0 = __builtin_amdgcn_s_memtime();
            r0 = __builtin_amdgcn_s_memrealtime();
            if (lane0) __hip_atomic_fetch_min(t_start + j, r0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const double toff0 = active ? jb.st[ch].trigOffset : 0.0;
            const double w = 2 * 3.14159265358979323846 * (jb.freq / jb.Fs);
            double toff_g;
            if (WG == 1) {
                toff_g = __shfl(toff0, 0);
            } else {
                if (threadIdx.x == 0) sh_toff = toff0;
                __syncthreads();
                toff_g = sh_toff;
            }
            const bool group_tab =
                tab_ok && __builtin_fabs(w) * (__builtin_fabs(toff_g) + (double)n + 1.0) < PLL_TAB_WT_MAX;
            if (group_tab)
                for (int k = threadIdx.x; k < n; k += 64 * WG) wtab[k] = w * (toff_g + (double)(k + 1));   // pll.cpp:46-47
            __syncthreads();
            const bool tab = group_tab && __all(!active || toff0 == toff_g);
            if (active) {
                if (SPLIT) {
                    if (parts) {
                        InGate g{pre_flag, sub_flag, err, want, sub_base, sub_tile, n, 0, t0};
                        gate_wait(g, 1);      // the part(s) the wait above saw
                        if (tab) pll_run_split<VEC, true, true>(jb, n, ch, wtab, &g);
                        else pll_run_split<VEC, false, true>(jb, n, ch, nullptr, &g);
                    } else if constexpr (COAL) {
                        if (tab) pll_run_split_coal<true, false>(jb, n, ch, wtab, nullptr, my_buf, my_tst);
                        else pll_run_split_coal<false, false>(jb, n, ch, nullptr, nullptr, my_buf, my_tst);
                    } else {
                        if (tab) pll_run_split<VEC, true>(jb, n, ch, wtab);
                        else pll_run_split<VEC, false>(jb, n, ch, nullptr);
                    }
                } else {
                    if (tab) pll_run<VEC, true>(jb, n, ch, wtab);
                    else pll_run<VEC, false>(jb, n, ch, nullptr);
                }
            }
            __syncthreads();   // every lane's table reads and state/phase stores issued before the release
        }
        if (lane0) {
            if (!dead) {
                const unsigned long long c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
                __hip_atomic_fetch_max(t_end + j, r1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                // sums over waves: shader cycles and 100 MHz ticks spent on block j (sdr_plls_cycles)
                __hip_atomic_fetch_add(t_cyc + 2 * j, c1 - c0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_fetch_add(t_cyc + 2 * j + 1, r1 - r0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#if SDR_PLL_WAVES
                dw_cyc += c1 - c0;
                dw_wait += r0 - t0;
                dw_blocks++;
#endif
            }
            // block sequence pre_first + j done by this wave: its own slot of the ring
            __hip_atomic_fetch_add(done_ring + (pre_first + (uint32_t)j) % PLL_DONE_RING, 1u, __ATOMIC_RELEASE,
                                   __HIP_MEMORY_SCOPE_AGENT);
        }
    }
#if SDR_PLL_WAVES
    const int slot = ((int)(blockIdx.y * gridDim.x + blockIdx.x)) * WG + (int)(threadIdx.x >> 6);
    if (lane0 && slot < PLL_WAVE_SLOTS) {
        g_pll_waves[slot][0] = dw_cyc;
        g_pll_waves[slot][1] = dw_wait;
        g_pll_waves[slot][2] = dw_blocks;
        g_pll_waves[slot][3] = blockIdx.y + 1u;
        g_pll_waves[slot][4] = dw_spin;
        g_pll_waves[slot][5] = dw_polls;
        g_pll_waves[slot][6] = dw_ready;
        g_pll_waves[slot][7] = dw_early;
    }
#endif
}

// The two ends of the persistent PLLs' hand-offs, as one-wave kernels so that HIP's in-order
// kernel dispatch (each dispatch starts after the previous one in its stream has completed and
// released its writes) orders them: k_flag_store publishes "block ready" after the pre-PLL
// kernels of the front-end stream; k_flag_wait holds the post stream until the PLL waves have
// released a block (bounded, like the PLL's own waits).
__global__ void k_flag_store(uint32_t* flag, uint32_t v) {
#if SDR_PLL_WAVES
    if (threadIdx.x == 0 && flag == g_diag_flag) g_flag_t[v & 63] = __builtin_amdgcn_s_memrealtime();
#endif
    if (threadIdx.x == 0) __hip_atomic_store(flag, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
}
__global__ void k_flag_wait(const uint32_t* ctr, uint32_t want, uint32_t* err) {
    if (threadIdx.x != 0) return;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while ((int32_t)(__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - want) < 0) {
        __builtin_amdgcn_s_sleep(4);
        if (__builtin_amdgcn_s_memrealtime() - t0 > PLL_WAIT_TICKS) {
            __hip_atomic_fetch_or(err, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            break;
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");   // once, after the poll (see k_pll_multi)
}

// pll_rx and -x of a PLL input with no fused producer (the batched sdr_fmpll primitive)
__global__ __launch_bounds__(BLK) void k_pll_rx(double* __restrict__ rx, float* __restrict__ xneg, size_t rx_stride,
                                                const float* __restrict__ x, size_t x_stride, int n) {
    const int ch = blockIdx.y;
    const int i = blockIdx.x * BLK + threadIdx.x;
    if (i < n) {
        const float v = x[(size_t)ch * x_stride + i];
        rx[(size_t)ch * rx_stride + i] = pllm::pll_rx(v);
        xneg[(size_t)ch * rx_stride + i] = -v;
    }
}

__global__ __launch_bounds__(64) void k_pll_libm(const PllJobs jobs, int n, int nch) {
    const int ch = blockIdx.x * blockDim.x + threadIdx.x;
    if (ch >= nch) return;
    const PllJob& jb = jobs.j[blockIdx.y];
    const float* __restrict__ in = jb.in;
    const size_t in_stride = jb.in_stride, t_stride = jb.t_stride, out_stride = jb.out_stride;
    float* __restrict__ tbuf = jb.tbuf;
    float* __restrict__ out = jb.out;
    sdr_pll_state* __restrict__ st = jb.st;
    const float freq = jb.freq, Fs = jb.Fs, normBandwidth = jb.bw;
    const float Cp = 2.666;
    const float Ci = 3.555;
    const float Kp = normBandwidth * Cp;
    const float Ki = normBandwidth * normBandwidth * Ci;
    const double w = 2 * 3.14159265358979323846 * (freq / Fs);  // 2*PI*(freq/Fs), pll.cpp:47
    sdr_pll_state s = st[ch];
    const float* x = in + (size_t)ch * in_stride;
    if (!jb.prev_out) out[(size_t)ch * out_stride] = s.lastCarrier;
    float* o = tbuf + (size_t)ch * t_stride;
    float fbI = s.feedbackI, fbQ = s.feedbackQ, integ = s.integrator, ph = s.phaseEst;
    double toff = s.trigOffset;
    for (int i = 0; i < n; i++) {
        const float xi = x[i];
        const float eI = xi * fbI;
        const float eQ = xi * (-fbQ);
        const float e = (float)atan2((double)eQ, (double)eI);
        integ = integ + Ki * e;
        ph = ph + Kp * e + integ;
        toff += 1.0;
        const float t = (float)(w * toff + (double)ph);
        double sv, cv;
        sincos((double)t, &sv, &cv);
        fbI = (float)cv;
        fbQ = (float)sv;
        o[i] = t;
    }
    s.feedbackI = fbI;
    s.feedbackQ = fbQ;
    st[ch].feedbackI = fbI;
    st[ch].feedbackQ = fbQ;
    st[ch].integrator = integ;
    st[ch].phaseEst = ph;
    st[ch].trigOffset = toff;
}

// glibc's cos of pll.cpp:52 for the inputs the fast path cannot decide (see pll_atan2_ref)
__device__ __noinline__ float nco_cos_ref(float a) {
    double sv, cv;
    pll_sincos_ref(a, &sv, &cv);
    return (float)cv;
}

// out[ch][i+1]: t_i -> (float)cos((double)(t_i*ncoScale + phaseAdjust)) (pll.cpp:52), in parallel;
// lastCarrier <- out[ch][n] (pll.cpp:58)
__global__ __launch_bounds__(BLK) void k_nco_out(const PllJobs jobs, int n) {
    const int ch = blockIdx.y;
    const int i = blockIdx.x * BLK + threadIdx.x;
    if (i >= n) return;
    const PllJob& jb = jobs.j[blockIdx.z];
    const float* __restrict__ tbuf = jb.tbuf;
    const size_t t_stride = jb.t_stride, out_stride = jb.out_stride;
    float* __restrict__ out = jb.out;
    sdr_pll_state* __restrict__ st = jb.st;
    const float ncoScale = jb.ncoScale, phaseAdjust = jb.phaseAdjust;
    float* o = out + (size_t)ch * out_stride + 1;
    const float t = tbuf[(size_t)ch * t_stride + i];
    const float a = t * ncoScale + phaseAdjust;
    const pllm::SinCos sc = pllm::sincos_f32(a);
    float v = (float)sc.c;
    if (!sc.ok) v = nco_cos_ref(a);
    o[i] = v;
    if (i == n - 1) st[ch].lastCarrier = v;
    if (i == 0 && jb.prev_out) o[-1] = jb.prev_out[(size_t)ch * out_stride + n];
}
// PLL + NCO output: k_pll (fast, default) or k_pll_libm (SDR_FLAG_PLL_LIBM)
}  // namespace

// compile-time A/B switches for variant builds (tools/build_variant.sh), never read at run time:

int launch_nco(const PllJobs& jobs, int njobs, int n, int nch, hipStream_t s) {
    if (n > 0) {
        hipLaunchKernelGGL(k_nco_out, dim3(cdiv(n, BLK), nch, njobs), dim3(BLK), 0, s, jobs, n);
        LAUNCH_CHECK();
    }
    return SDR_OK;
}

int launch_plls(bool libm, const PllJobs& jobs, int njobs, int n, int nch, hipStream_t s, bool with_nco) {
    bool vec = true, split = true;
    for (int k = 0; k < njobs; k++) {
        const PllJob& j = jobs.j[k];
        vec = vec && (reinterpret_cast<uintptr_t>(j.in) % 16 == 0) && (j.in_stride % 4 == 0) &&
              (reinterpret_cast<uintptr_t>(j.tbuf) % 16 == 0) && (j.t_stride % 4 == 0) &&
              (reinterpret_cast<uintptr_t>(j.rx) % 16 == 0) && (j.rx_stride % 2 == 0) &&
              (!j.in_neg || (reinterpret_cast<uintptr_t>(j.in_neg) % 16 == 0 && j.neg_stride % 4 == 0));
        split = split && j.in_neg;   // lane pairs need the producer's -x row
    }
    const dim3 g(cdiv(split ? 2 * nch : nch, 64), njobs), b(64);
    // LDS table of w * trigOffset (k_pll): n doubles, 16-byte rows
    const size_t tab_bytes = round_up((size_t)std::max(n, 1), 2) * sizeof(double);
    const int tab_ok = tab_bytes <= 64 * 1024 ? 1 : 0;
    const size_t lds = tab_ok ? tab_bytes : 0;
    if (libm) {
        hipLaunchKernelGGL(k_pll_libm, g, b, 0, s, jobs, n, nch);
    } else if (vec) {
        if (split) hipLaunchKernelGGL((k_pll<true, true>), g, b, lds, s, jobs, n, nch, tab_ok);
        else hipLaunchKernelGGL((k_pll<true, false>), g, b, lds, s, jobs, n, nch, tab_ok);
    } else {
        if (split) hipLaunchKernelGGL((k_pll<false, true>), g, b, lds, s, jobs, n, nch, tab_ok);
        else hipLaunchKernelGGL((k_pll<false, false>), g, b, lds, s, jobs, n, nch, tab_ok);
    }
    LAUNCH_CHECK();
    return with_nco ? launch_nco(jobs, njobs, n, nch, s) : SDR_OK;
}

int launch_pll(bool libm, const float* in, size_t in_stride, int n, int nch, float freq, float Fs, float* tbuf,
               size_t t_stride, double* rxbuf, float* negbuf, float* out, size_t out_stride, sdr_pll_state* st,
               float ncoScale, float phaseAdjust, float bw, hipStream_t s) {
    if (n > 0) {
        hipLaunchKernelGGL(k_pll_rx, dim3(cdiv(n, BLK), nch), dim3(BLK), 0, s, rxbuf, negbuf, t_stride, in, in_stride,
                           n);
        LAUNCH_CHECK();
    }
    PllJobs jobs{};
    jobs.j[0] = PllJob{in, in_stride, tbuf, t_stride, out, out_stride, st, freq, Fs, bw, ncoScale, phaseAdjust, nullptr,
                       rxbuf, t_stride, negbuf, t_stride};
    return launch_plls(libm, jobs, 1, n, nch, s);
}

int pll_multi_plan(const PllJobs2& jobs, int njobs, int n, int nch, const CuPlacement& pl, PllMultiPlan* plan) {
    bool vec = true, split = true;
    for (int k = 0; k < 2; k++)
        for (int q = 0; q < njobs; q++) {
            const PllJob& j = jobs.p[k].j[q];
            vec = vec && (reinterpret_cast<uintptr_t>(j.in) % 16 == 0) && (j.in_stride % 4 == 0) &&
                  (reinterpret_cast<uintptr_t>(j.tbuf) % 16 == 0) && (j.t_stride % 4 == 0) &&
                  (reinterpret_cast<uintptr_t>(j.rx) % 16 == 0) && (j.rx_stride % 2 == 0) &&
                  (!j.in_neg || (reinterpret_cast<uintptr_t>(j.in_neg) % 16 == 0 && j.neg_stride % 4 == 0));
            split = split && j.in_neg;
        }
    PllMultiPlan& P = *plan;
    const size_t tab_bytes = round_up((size_t)std::max(n, 1), 2) * sizeof(double);
    P.tab_ok = tab_bytes <= 64 * 1024 ? 1 : 0;
    P.lds = P.tab_ok ? tab_bytes : 0;
    const int wave_cnt = cdiv(split ? 2 * nch : nch, 64) * njobs;
    // one wave per workgroup (its own CU time slice and table) while two tables per CU fit the
    // stream's CUs, else groups of 4 waves -- one per SIMD -- sharing one table per CU
    P.WG = wave_cnt > 2 * pl.ncu ? 4 : 1;
    P.g = dim3(cdiv(split ? 2 * nch : nch, 64 * P.WG), njobs);
    P.b = dim3(64 * P.WG);
    P.waves = P.g.x * P.g.y * P.WG;
    P.groups = (long long)P.g.x * P.g.y;
    auto kern_of = [&](auto v, auto sp, auto wg) -> const void* {
        return reinterpret_cast<const void*>(k_pll_multi<decltype(v)::value, decltype(sp)::value, decltype(wg)::value>);
    };
    using T = std::true_type;
    using F = std::false_type;
    using W1 = std::integral_constant<int, 1>;
    using W4 = std::integral_constant<int, 4>;
    const void* plain = P.WG == 4 ? (vec ? (split ? kern_of(T{}, T{}, W4{}) : kern_of(T{}, F{}, W4{}))
                                         : (split ? kern_of(F{}, T{}, W4{}) : kern_of(F{}, F{}, W4{})))
                                  : (vec ? (split ? kern_of(T{}, T{}, W1{}) : kern_of(T{}, F{}, W1{}))
                                         : (split ? kern_of(F{}, T{}, W1{}) : kern_of(F{}, F{}, W1{})));
    // every workgroup of a persistent launch must be resident at once (a wave that cannot start holds
    // up the done count of every block, and the producer of later blocks waits for that): the
    // workgroups of this kernel that fit one CU (its VGPRs, the LDS table) times what the placement of
    // the stream's CU mask keeps resident (sdr_internal.h CuPlacement)
    auto resident = [&](const void* kern, int* per_cu) {
        *per_cu = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(per_cu, kern, 64 * P.WG, P.lds) != hipSuccess || *per_cu <= 0)
            *per_cu = std::min(4 / P.WG, P.tab_ok ? (int)(160 * 1024 / tab_bytes) : 4 / P.WG);
        return pl.resident(*per_cu);
    };
    // packed groups (more than two waves per CU): the chunk inputs and phases through LDS in
    // line-shaped pieces (pll_run_split_coal; every lane of every wave must hold a channel): 357 -> 262
    // cycles per step at four waves per CU; at two it measured 231-235 -> 237, so one-wave groups keep
    // the register prefetch (profiles/r05/coal/). Its staging ring (3 x 6 KiB + 2.5 KiB per wave, 83 KiB per
    // group, beside the table) fits one group per CU: a launch that needs more falls back to the register-prefetch
    // groups, which fit two.
    P.kern = plain;
    if (vec && split && nch % 32 == 0 && P.WG == 4) {
        const void* coal = reinterpret_cast<const void*>(k_pll_multi<true, true, 4, true>);
        int pc = 0;
        const long long r = resident(coal, &pc);
        if (r >= P.groups) {
            P.kern = coal;
            P.per_cu = pc;
            P.resident = r;
            return SDR_OK;
        }
    }
    P.resident = resident(plain, &P.per_cu);
    return SDR_OK;
}

int launch_pll_multi(const PllJobs2& jobs, int njobs, int n, int nch, int nblocks, uint32_t* words, uint32_t pre_first,
                     unsigned long long* t0, unsigned long long* t1, unsigned long long* tc, uint32_t* waves,
                     hipStream_t s, const CuPlacement& pl, int sub_tile) {
    PllMultiPlan P;
    if (const int r = pll_multi_plan(jobs, njobs, n, nch, pl, &P)) return r;
    *waves = P.waves;
    if (P.groups > P.resident)
        return fail(SDR_E_INVALID, "plls_launch: %u waves do not fit the stream's %d CUs: %lld of %lld workgroups of "
                    "%d waves resident at once (%d per CU, %d XCCs x %d SE-balanced CU slots; use sdr_plls, a "
                    "stream over more CUs, or sdr_plls_fits to pick one)", P.waves, pl.ncu, P.resident, P.groups,
                    P.WG, P.per_cu, pl.xcc_active, pl.min_units);
    hipLaunchKernelGGL(reinterpret_cast<void (*)(PllJobs2, int, int, int, int, const uint32_t*, uint32_t, uint32_t*,
                                                 uint32_t*, unsigned long long*, unsigned long long*,
                                                 unsigned long long*, const uint32_t*, uint32_t, int)>(
                           const_cast<void*>(P.kern)),
                       P.g, P.b, P.lds, s, jobs, n, nch, P.tab_ok, nblocks, words, pre_first, words + PLL_WORDS_DONE,
                       words + 1, t0, t1, tc, sub_tile > 0 ? words + PLL_WORD_SUB : nullptr,
                       pre_first * PLL_SUB_SCALE, sub_tile);
    LAUNCH_CHECK();
    return SDR_OK;
}

int launch_flag_store(uint32_t* flag, uint32_t v, hipStream_t s) {
    hipLaunchKernelGGL(k_flag_store, dim3(1), dim3(64), 0, s, flag, v);
    LAUNCH_CHECK();
    return SDR_OK;
}

int launch_flag_wait(const uint32_t* ctr, uint32_t want, uint32_t* err, hipStream_t s) {
    hipLaunchKernelGGL(k_flag_wait, dim3(1), dim3(64), 0, s, ctr, want, err);
    LAUNCH_CHECK();
    return SDR_OK;
}

// Diagnosis builds only (-DSDR_PLL_COUNT=1): the PLL chunk counters [lane-chunks, failed lane-chunks,
// wave-chunks, redone wave-chunks, then per reason and per job (g_pll_counts)], 10 values,
// optionally reset; -1 in product builds.
int diag_pll_counts(unsigned long long* out, int reset) {
#if SDR_PLL_COUNT
    HIP_TRY(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_pll_counts), sizeof(unsigned long long) * PLL_NCOUNTS));
    if (reset) {
        const unsigned long long z[PLL_NCOUNTS] = {};
        HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_pll_counts), z, sizeof z));
    }
    return SDR_OK;
#else
    (void)out;
    (void)reset;
    return -1;
#endif
}

// Diagnosis builds only (-DSDR_PLL_WAVES=1): the per-wave totals of the last persistent launch
// (g_pll_waves), at most nmax waves of PLL_WAVE_FIELDS (8) values, cleared after the read; -1 in
// product builds.
int diag_pll_waves(unsigned long long* out, int nmax) {
#if SDR_PLL_WAVES
    const int nw = std::min(nmax, PLL_WAVE_SLOTS);
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_pll_waves), sizeof(unsigned long long) * PLL_WAVE_FIELDS * nw));
    static unsigned long long z[PLL_WAVE_SLOTS][PLL_WAVE_FIELDS];
    HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_pll_waves), z, sizeof z));
    return nw;
#else
    (void)out;
    (void)nmax;
    return -1;
#endif
}

// Diagnosis builds only (-DSDR_PLL_HWID=1): placement and duration of the last k_pll launch's waves
// (g_pll_hwid), at most nmax waves of PLL_HWID_FIELDS (5) values; -1 in product builds.
int diag_pll_hwid(unsigned long long* out, int nmax) {
#if SDR_PLL_HWID
    const int nw = std::min(nmax, PLL_HWID_SLOTS);
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_pll_hwid), sizeof(unsigned long long) * PLL_HWID_FIELDS * nw));
    return nw;
#else
    (void)out;
    (void)nmax;
    return -1;
#endif
}

}  // namespace sdrk
