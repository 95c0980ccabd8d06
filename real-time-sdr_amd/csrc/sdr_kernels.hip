// sdr_kernels.hip -- MI355X (gfx950) kernels, launchers and C ABI of the FM/RDS DSP hot path.
//
// Hot path of TheZxc07/real-time-SDR recast as batched kernels over many independent channels:
//   front end   u8 I/Q -> 101-tap FIR /10 on I and Q -> FM discriminator    rffrontend.cpp:58-71
//               (sdr_frontend.hip)
//   mono        101-tap resampler U/D -> int16                            mono.cpp:34-42
//   stereo      pilot BPF -> PLL(19k, x2) ; band BPF ; mixer ; delay ; 2 resamplers -> L/R
//                                                                          stereo.cpp:74-107
//   rds DSP     BPF -> square -> BPF -> PLL(114k, x0.5) ; delay ; mixer -> 247/640 resampler
//               -> RRC                                                     rds.cpp:105-133
//   rds bits    cdr -> slicer -> Manchester -> differential               rds.cpp:135-167
//   PLL / NCO   pll.cpp:4-61 (sdr_pll.hip)
//
// Numerics ("exact" mode, default): every kernel keeps the reference's rounding points --
// f32 product then f32 add in tap order (no contraction: `fp contract(off)` below), the
// discriminator's f64 denominator/division, the PLL's f64 atan2/sin/cos on f32 arguments.
// Layout: see sdr_internal.h.

#include "sdr_internal.h"

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <cstdarg>
#include <cstdlib>
#include <mutex>
#include <string>
#include <vector>

#include "sdr_amd.h"
#include "pll_math.h"
#include "nco.h"

#pragma clang fp contract(off)

#ifndef SDR_FILL_FE_PARTS
#define SDR_FILL_FE_PARTS 0      // sdr_frontend_pre_parts: one front-end launch per part (A/B only)
#endif

namespace sdrk {
namespace {
thread_local std::string g_err;
}  // namespace

int fail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

const char* last_error() { return g_err.c_str(); }
const char* last_error();
}  // namespace sdrk

using namespace sdrk;

namespace {

// static_cast<short>(float) as g++/x86-64 lowers it (mono.cpp:41, stereo.cpp:101-102):
// cvttss2si (INT_MIN when out of range or NaN), then the low 16 bits.
__device__ __forceinline__ int32_t cvt_i32_x86(float v) {
    return (v >= -2147483648.0f && v < 2147483648.0f) ? (int32_t)v : INT32_MIN;
}
__device__ __forceinline__ int16_t cvt_i16_x86(float v) {
    return (int16_t)(uint16_t)((uint32_t)cvt_i32_x86(v) & 0xFFFFu);
}

// The error words an output stage checks before it hands out a block (SDR_PCM_POISON audio, NaN
// rds_clean rows, nbits = SDR_NBITS_POISONED instead of outputs, include/sdr_amd.h):
//   pers  the persistent PLL launch that produced this block's phases (null for other blocks)
//   fail  the context's sticky release-timeout word: a producer overwrote a parity buffer whose
//         readers had not released it within the bounded wait (release_wait), so any reader that
//         runs after it may read the next block's data; set until sdr_ctx_reset.
struct Poison {
    const uint32_t* pers;
    const uint32_t* fail;
};
// read once per wave (scalar loads of kernel-argument addresses; the value is made wave-uniform)
__device__ __forceinline__ uint32_t poison_word(const Poison& p) {
    uint32_t v = 0;
    if (p.pers) v |= *p.pers;
    if (p.fail) v |= *p.fail;
    return __builtin_amdgcn_readfirstlane(v);
}
// The same words read again once the kernel's input loads have completed (issued after the staging
// barrier, consumed before the stores, so its latency hides behind the compute): a release wait that
// expires while a reader runs sets its word before the producer overwrites that reader's inputs, so
// a reader that loaded any overwritten sample sees the word here (agent-scope loads: from L2, the
// coherence point) and poisons instead of storing a mixed block.
__device__ __forceinline__ uint32_t poison_late(const Poison& p) {
    uint32_t v = 0;
    if (p.pers) v |= __hip_atomic_load(p.pers, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (p.fail) v |= __hip_atomic_load(p.fail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return v;
}

// ------------------------------------------------------------------------------------------
// Decimating FIR, filter.cpp:106-121: y[n] = sum_{k<ntaps} h[k] * x[nD-k], ascending k, f32
// mul then add. x[m] for m < 0 comes from `hist` (hist[m], m >= -nhist). NT = 1 or 2 tap sets
// sharing one staged window. SQUARE: the input is x*x (rds.cpp:111-113 fused into :116).
// ------------------------------------------------------------------------------------------
template <int NT, bool SQUARE>
__global__ __launch_bounds__(BLK) void k_fir(const float* __restrict__ x, size_t x_stride,
                                             const float* __restrict__ hist, size_t hist_stride,
                                             const float* __restrict__ h0, const float* __restrict__ h1, int ntaps,
                                             int D, int ny, int tile, float* __restrict__ y0,
                                             float* __restrict__ y1, size_t y_stride,
                                             double* __restrict__ rx0, size_t rx_stride) {
    extern __shared__ float4 smem4[];
    float* sh = reinterpret_cast<float*>(smem4);
    const int ntaps_pad = (ntaps + 3) & ~3;
    const int ch = blockIdx.y, tid = threadIdx.x;
    const int n0 = blockIdx.x * tile, n1 = min(n0 + tile, ny);
    const int m0 = n0 * D - (ntaps - 1), m1 = (n1 - 1) * D;
    const int W = m1 - m0 + 1;
    float* sx = sh + NT * ntaps_pad;
    const float* xc = x + (size_t)ch * x_stride;
    const float* hc = hist + (size_t)ch * hist_stride;
    for (int i = tid; i < ntaps; i += BLK) {
        sh[i] = h0[i];
        if (NT == 2) sh[ntaps_pad + i] = h1[i];
    }
    for (int i = tid; i < W; i += BLK) {
        const int m = m0 + i;
        float v = (m < 0) ? hc[m] : xc[m];
        if (SQUARE) v = v * v;
        sx[i] = v;
    }
    __syncthreads();
    for (int n = n0 + tid; n < n1; n += BLK) {
        const int base = n * D - m0;
        float a0 = 0.0f, a1 = 0.0f;
        for (int k = 0; k < ntaps; k++) {
            const float v = sx[base - k];
            a0 = a0 + sh[k] * v;
            if (NT == 2) a1 = a1 + sh[ntaps_pad + k] * v;
        }
        y0[(size_t)ch * y_stride + n] = a0;
        if (NT == 2) y1[(size_t)ch * y_stride + n] = a1;
        if (rx0) rx0[(size_t)ch * rx_stride + n] = pllm::pll_rx(a0);   // y0 feeds a PLL: its reciprocal
    }
}

// ------------------------------------------------------------------------------------------
// The IF-rate 101-tap FIRs without decimation (filter.cpp:106-121 with D = 1: pilot/band BPFs
// stereo.cpp:74,80, RDS BPF rds.cpp:105, squared-RDS BPF :116, RRC :133), register-blocked:
// each thread computes FRB_R consecutive outputs from a window of FRB_R + 100 samples read once
// from LDS (16-byte reads), and every output still sums h[k] * x[n-k] in ascending k as an f32
// product then an f32 add (no contraction). NT tap sets (1..3) share one staged window: the stereo
// pilot and band filters and the RDS band filter all read fm_demod (stereo.cpp:74,80, rds.cpp:105).
// Taps are wave-uniform scalar operands, fetched FRB_TC at a time: scalar loads return out of
// order, so every wait for one is lgkmcnt(0); the next chunk is therefore requested only after the
// current chunk's first products have waited for it, and its latency hides behind the rest of the
// chunk (FRB_TC x R x NT multiply-adds) instead of stalling every tap.
// ------------------------------------------------------------------------------------------
constexpr int FRB_T = 101;                 // taps (rf_taps, project.cpp:61)
constexpr int FRB_R = 8;                   // outputs per thread
constexpr int FRB_TILE = BLK * FRB_R;      // outputs per workgroup
constexpr int FRB_W = FRB_TILE + FRB_T - 1 + 3;   // staged samples (+3: whole 16-byte reads)

// Up to three tap sets over one input window. Output t goes to y[t] (stride y_stride[t]); y[0] may
// also get its PLL reciprocals (rx0) and its negation (y0neg, same stride: the lane-pair PLL's
// second input, sdr_pll.hip pll_run_split), and y[2] the history of an extended stream (hist2_src:
// the other parity's row, copied in front by the first tile of each channel).
struct FirRb {
    const float* h[3];
    const float* h01;          // {h[0][k], h[1][k]} interleaved, padded to 104 pairs (k_fir_rb<3, *, true>)
    float* y[3];
    size_t y_stride[3];
    float* y0neg;
    double* rx0;
    size_t rx_stride;
    const float* hist2_src;
    Poison err;                // {null, null}, or the block's error words: NaN outputs when one is set
    float* ydup;              // non-null: y[0] stored here too (stride ydup_stride)
    size_t ydup_stride;
    int x0;                    // first tile (blockIdx.x + x0): a part of the block (sdr_frontend_pre_parts)
};

// PK (NT == 3): tap sets 0 and 1 (the stereo pilot and band BPFs) run as packed pairs -- one
// v_pk_mul_f32 + one v_pk_add_f32 per sample and output for both, the same two roundings each as
// filter.cpp:115 -- and set 2 (the RDS BPF) scalar: 4 VALU per sample and output instead of 6.
template <int NT, bool SQUARE, bool PK = false>
__global__ __launch_bounds__(BLK) void k_fir_rb(const float* __restrict__ x, size_t x_stride,
                                                const float* __restrict__ hist, size_t hist_stride, int ny,
                                                const FirRb f) {
    static_assert(!PK || NT >= 2, "packed pairs: sets 0 and 1 of a 2- or 3-set pass");
    constexpr int T = FRB_T, R = FRB_R;
    __shared__ __attribute__((aligned(16))) float sx[(FRB_W + 3) & ~3];
    __shared__ uint32_t s_poison;                                 // one decision per workgroup
    const int ch = blockIdx.y, tid = threadIdx.x;
    const bool checks = f.err.pers || f.err.fail;
    if (checks && tid == 0) s_poison = poison_word(f.err);        // (its latency hides behind the staging)
    const int xt = (int)blockIdx.x + f.x0;                        // tile of the block
    const int n0 = xt * FRB_TILE;
    const int m0 = n0 - (T - 1);
    const int W = min(FRB_TILE, ny - n0) + T - 1;
    {
        // all loads of the tile in flight at once, then the LDS writes
        const float* xc = x + (size_t)ch * x_stride;
        const float* hc = hist + (size_t)ch * hist_stride;
        constexpr int NL = (FRB_TILE + FRB_T - 1 + BLK - 1) / BLK;
        float v[NL];
#pragma unroll
        for (int u = 0; u < NL; u++) {
            const int i = tid + u * BLK, m = m0 + i;
            v[u] = (i < W) ? (m < 0 ? hc : xc)[m] : 0.0f;
        }
#pragma unroll
        for (int u = 0; u < NL; u++) {
            const int i = tid + u * BLK;
            if (i < W) sx[i] = SQUARE ? v[u] * v[u] : v[u];       // rds.cpp:111-113
        }
    }
    if (NT == 3 && f.hist2_src && xt == 0 && tid < HIST)          // y[2]'s history (extended stream)
        f.y[2][(size_t)ch * f.y_stride[2] + tid - HIST] = f.hist2_src[(size_t)ch * f.y_stride[2] + ny - HIST + tid];
    __syncthreads();
    const int nb = n0 + tid * R;
    if (nb >= ny) return;
    const uint32_t late = checks ? poison_late(f.err) : 0u;     // after every input load of the tile
    // w[i] = x[nb - (T-1) + i]; output nb + j at tap k reads w[j + T-1 - k] (samples past the
    // staged window only feed outputs >= ny, which are not stored)
    float w[R + T - 1 + 3];
#pragma unroll
    for (int i = 0; i < (R + T - 1 + 3) / 4; i++) {
        const float4 v = reinterpret_cast<const float4*>(sx + tid * R)[i];
        w[4 * i] = v.x; w[4 * i + 1] = v.y; w[4 * i + 2] = v.z; w[4 * i + 3] = v.w;
    }
    float a[NT][R];
    constexpr int FRB_TC = 4;
    constexpr int FRB_NC = (FRB_T + FRB_TC - 1) / FRB_TC;   // chunks (tap buffers are padded past 101)
    typedef float f4v __attribute__((ext_vector_type(FRB_TC)));
    if constexpr (PK) {
        typedef float f8v __attribute__((ext_vector_type(2 * FRB_TC)));
        constexpr bool S2 = NT == 3;                     // a third, scalar set beside the pair
        f32x2 a01[R];
        float a2[R];
#pragma unroll
        for (int j = 0; j < R; j++) { a01[j] = f32x2{0.0f, 0.0f}; a2[j] = 0.0f; }
        f8v pb[2];                                       // {h0, h1} pairs of chunk c in pb[c & 1]
        f4v sb[2] = {};                                  // set 2's taps of chunk c
        auto load8 = [&](f8v& d, int c) {
            asm volatile("s_load_dwordx8 %0, %1, %2" : "=s"(d) : "s"(f.h01), "s"(c * FRB_TC * 8) : "memory");
        };
        auto load4 = [&](f4v& d, int c) {
            if constexpr (S2)
                asm volatile("s_load_dwordx4 %0, %1, %2" : "=s"(d) : "s"(f.h[NT - 1]), "s"(c * FRB_TC * 4) : "memory");
        };
        load8(pb[0], 0);
        load4(sb[0], 0);
        // the wait redefines the loaded registers, so no use of them is scheduled above it (a
        // product hoisted above a plain waitcnt read the taps before they landed)
        asm volatile("s_waitcnt lgkmcnt(0)" : "+s"(pb[0]), "+s"(sb[0]) :: "memory");
#pragma unroll
        for (int c = 0; c < FRB_NC; c++) {
#pragma unroll
            for (int kk = 0; kk < FRB_TC; kk++) {
                const int k = c * FRB_TC + kk;
                if (k < T) {
                    const double hp = __builtin_bit_cast(double, f32x2{pb[c & 1][2 * kk], pb[c & 1][2 * kk + 1]});
#pragma unroll
                    for (int j = 0; j < R; j++) {
                        const int i = j + T - 1 - k;
                        // plain vector code: the compiler broadcasts the sample by op_sel (no copy)
                        // and knows the packed result's latency (no inline-asm wait state, unlike an
                        // inline-asm v_pk_mul_f32)
                        const f32x2 pr = __builtin_bit_cast(f32x2, hp) * f32x2{w[i], w[i]};
                        a01[j] = a01[j] + pr;                                  // filter.cpp:115
                        if constexpr (S2) a2[j] = a2[j] + sb[c & 1][kk] * w[i];
                    }
                }
                if (kk == 0 && c + 1 < FRB_NC) {
                    __builtin_amdgcn_sched_barrier(0);
                    load8(pb[(c + 1) & 1], c + 1);
                    load4(sb[(c + 1) & 1], c + 1);
                    __builtin_amdgcn_sched_barrier(0);
                }
            }
            if (c + 1 < FRB_NC) {
                __builtin_amdgcn_sched_barrier(0);
                asm volatile("s_waitcnt lgkmcnt(0)" : "+s"(pb[(c + 1) & 1]), "+s"(sb[(c + 1) & 1]) :: "memory");
                __builtin_amdgcn_sched_barrier(0);
            }
        }
#pragma unroll
        for (int j = 0; j < R; j++) {
            a[0][j] = a01[j].x;
            a[1][j] = a01[j].y;
            if constexpr (S2) a[NT - 1][j] = a2[j];
        }
    } else {
#pragma unroll
    for (int t = 0; t < NT; t++)
#pragma unroll
        for (int j = 0; j < R; j++) a[t][j] = 0.0f;
    // taps: scalar loads issued by hand (the compiler would wait for every outstanding scalar load
    // at each tap's first use), one chunk of FRB_TC taps per tap set ahead
    f4v buf[2][NT];                                     // chunk c in buf[c & 1]
    // base address in an SGPR pair, byte offset in an SGPR (not one address pair per chunk)
    auto load = [&](f4v& d, const float* hp, int c) {
        asm volatile("s_load_dwordx4 %0, %1, %2" : "=s"(d) : "s"(hp), "s"(c * FRB_TC * 4) : "memory");
    };
#pragma unroll
    for (int t = 0; t < NT; t++) load(buf[0][t], f.h[t], 0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int t = 0; t < NT; t++) asm volatile("" : "+s"(buf[0][t]));   // no tap use above the wait
#pragma unroll
    for (int c = 0; c < FRB_NC; c++) {
#pragma unroll
        for (int kk = 0; kk < FRB_TC; kk++) {
            const int k = c * FRB_TC + kk;
            if (k < T) {
#pragma unroll
                for (int j = 0; j < R; j++) {
                    const float v = w[j + T - 1 - k];
#pragma unroll
                    for (int t = 0; t < NT; t++) a[t][j] = a[t][j] + buf[c & 1][t][kk] * v;   // filter.cpp:115
                    // the MACs stay scalar (this unit is built with -fno-slp-vectorize): packed f32 ops
                    // run at half rate (tools/microbench/valu_rate.hip), and pairing neighbouring
                    // outputs costs register realignment and occupancy
                }
            }
            if (kk == 0 && c + 1 < FRB_NC) {
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int t = 0; t < NT; t++) load(buf[(c + 1) & 1][t], f.h[t], c + 1);
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        if (c + 1 < FRB_NC) {
            __builtin_amdgcn_sched_barrier(0);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // chunk c + 1 landed
#pragma unroll
            for (int t = 0; t < NT; t++) asm volatile("" : "+s"(buf[(c + 1) & 1][t]));
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    }
    // every sum is complete here: otherwise the compiler sinks the second and third tap sets' products
    // past the first set's (divergent) stores and spills their taps from SGPRs
#pragma unroll
    for (int t = 0; t < NT; t++)
#pragma unroll
        for (int j = 0; j < R; j++) asm volatile("" : "+v"(a[t][j]));
    if (checks && (s_poison | __builtin_amdgcn_readfirstlane(late)) != 0u) {   // no valid input behind this block
#pragma unroll
        for (int t = 0; t < NT; t++)
#pragma unroll
            for (int j = 0; j < R; j++) a[t][j] = __builtin_nanf("");
    }
#pragma unroll
    for (int t = 0; t < NT; t++) {
        float* o = f.y[t] + (size_t)ch * f.y_stride[t] + nb;
        if (nb + R <= ny) {
#pragma unroll
            for (int j = 0; j < R; j += 4)
                reinterpret_cast<float4*>(o + j)[0] = make_float4(a[t][j], a[t][j + 1], a[t][j + 2], a[t][j + 3]);
        } else {
#pragma unroll
            for (int j = 0; j < R; j++)
                if (nb + j < ny) o[j] = a[t][j];
        }
    }
    if (f.ydup) {                                                 // a second copy of y[0]
        float* o = f.ydup + (size_t)ch * f.ydup_stride + nb;
        if (nb + R <= ny) {
#pragma unroll
            for (int j = 0; j < R; j += 4)
                reinterpret_cast<float4*>(o + j)[0] = make_float4(a[0][j], a[0][j + 1], a[0][j + 2], a[0][j + 3]);
        } else {
#pragma unroll
            for (int j = 0; j < R; j++)
                if (nb + j < ny) o[j] = a[0][j];
        }
    }
    if (f.y0neg) {                                                // y[0] feeds a PLL: -y[0]
        float* o = f.y0neg + (size_t)ch * f.y_stride[0] + nb;
        if (nb + R <= ny) {
#pragma unroll
            for (int j = 0; j < R; j += 4)
                reinterpret_cast<float4*>(o + j)[0] = make_float4(-a[0][j], -a[0][j + 1], -a[0][j + 2], -a[0][j + 3]);
        } else {
#pragma unroll
            for (int j = 0; j < R; j++)
                if (nb + j < ny) o[j] = -a[0][j];
        }
    }
    if (f.rx0) {                                                  // y[0] feeds a PLL: its reciprocal
        double* r = f.rx0 + (size_t)ch * f.rx_stride + nb;
        if (nb + R <= ny) {
#pragma unroll
            for (int j = 0; j < R; j += 2)
                reinterpret_cast<double2*>(r + j)[0] = make_double2(pllm::pll_rx(a[0][j]), pllm::pll_rx(a[0][j + 1]));
        } else {
#pragma unroll
            for (int j = 0; j < R; j++)
                if (nb + j < ny) r[j] = pllm::pll_rx(a[0][j]);
        }
    }
}

// ------------------------------------------------------------------------------------------
// Rational resampler, filter.cpp:123-147. Output n: phase = nD mod U, q = (nD - phase)/U,
// y[n] = sum_j hp[phase][j] * x[q - j] (j ascending == k ascending), hp = polyphase taps,
// cnt[phase] = number of taps of that phase. The phase restarts every block (the reference
// recomputes it from n, :131). OUT: 0 -> f32 y, 1 -> int16(16384*y) (mono.cpp:40-42),
// 2 -> stereo L/R int16 from two inputs a (mono) and b (stereo) (stereo.cpp:100-107).
// ------------------------------------------------------------------------------------------
template <int OUT, int NTAP = 0>   // NTAP > 0: U == 1 with NTAP taps (uniform taps, unrolled sums)
__global__ __launch_bounds__(BLK) void k_resample(const float* __restrict__ xa, const float* __restrict__ ha,
                                                  size_t xa_stride, size_t ha_stride,
                                                  const float* __restrict__ xb, const float* __restrict__ hb,
                                                  size_t xb_stride, size_t hb_stride,
                                                  const float* __restrict__ hp, const int* __restrict__ cnt,
                                                  int L, int U, int D, int ny, int tile, int hist_lo,
                                                  void* __restrict__ y, size_t y_stride) {
    extern __shared__ float4 smem4[];
    float* sa = reinterpret_cast<float*>(smem4);
    const int ch = blockIdx.y, tid = threadIdx.x;
    const int n0 = blockIdx.x * tile, n1 = min(n0 + tile, ny);
    const int qlo = (int)(((long long)n0 * D) / U) - L;   // smallest input index any output reads
    const int qhi = (int)(((long long)(n1 - 1) * D) / U);
    const int W = qhi - qlo + 1;
    const int Wp = (W + 3) & ~3;
    float* sb = sa + Wp;
    // staging: 4 loads per thread in flight per round
    auto stage = [&](float* dst, const float* xc, const float* hc) {
        for (int i0 = tid; i0 < W; i0 += 4 * BLK) {
            float v[4];
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const int i = i0 + u * BLK, m = qlo + i;
                v[u] = (i < W && m >= hist_lo) ? (m < 0 ? hc : xc)[m] : 0.0f;
            }
#pragma unroll
            for (int u = 0; u < 4; u++)
                if (i0 + u * BLK < W) dst[i0 + u * BLK] = v[u];
        }
    };
    stage(sa, xa + (size_t)ch * xa_stride, ha + (size_t)ch * ha_stride);
    if (OUT == 2) stage(sb, xb + (size_t)ch * xb_stride, hb + (size_t)ch * hb_stride);
    __syncthreads();
    for (int n = n0 + tid; n < n1; n += BLK) {
        const long long nd = (long long)n * D;
        const int ph = NTAP > 0 ? 0 : (int)(nd % U);
        const int q = NTAP > 0 ? (int)nd : (int)(nd / U);
        const float* hr = hp + (size_t)ph * L;
        const int base = q - qlo;
        float a = 0.0f, b = 0.0f;
        if (NTAP > 0) {                 // one polyphase row (U = 1): wave-uniform scalar taps
#pragma unroll 8
            for (int j = 0; j < NTAP; j++) {
                const float hj = hp[j];
                a = a + hj * sa[base - j];
                if (OUT == 2) b = b + hj * sb[base - j];
            }
        } else {
            const int c = cnt[ph];
            for (int j = 0; j < c; j++) {
                const float hj = hr[j];
                a = a + hj * sa[base - j];
                if (OUT == 2) b = b + hj * sb[base - j];
            }
        }
        if (OUT == 0) {
            static_cast<float*>(y)[(size_t)ch * y_stride + n] = a;
        } else if (OUT == 1) {
            static_cast<int16_t*>(y)[(size_t)ch * y_stride + n] = cvt_i16_x86(16384 * a);
        } else {
            int16_t* o = static_cast<int16_t*>(y) + (size_t)ch * y_stride + 2 * n;
            o[0] = cvt_i16_x86(16384 * (a + b));   // left  = 16384*(m + s)
            o[1] = cvt_i16_x86(16384 * (a - b));   // right = 16384*(m - s)
        }
    }
}

// ------------------------------------------------------------------------------------------
// The RDS 247/640 resampler (rds.cpp:130 -> filter.cpp:123-147) with lanes = channels: a
// workgroup takes 64 channels x RLC_TN outputs. Every output has its own polyphase row, shared by
// all 64 channels, so the rows of the tile are staged once in LDS and read as broadcasts, while
// each lane reads its own channel's samples from an odd-strided LDS tile (no bank conflicts).
// ptq[n] = (q << 8) | phase with phase = nD mod U, q = nD / U (host table; U < 256). Sums stay
// in ascending j (= ascending k of the reference) as f32 product then f32 add.
// ------------------------------------------------------------------------------------------
// outputs per workgroup, over 8 waves of 4 outputs: the x tile (64 channels x the tile's q span,
// 46 KB of LDS) bounds a CU to 2-3 workgroups, so 8 waves per workgroup instead of 4 give 16 waves per
// CU instead of 12 to hide the tap rows' scalar-load latency: 44.5 -> 37.7 us isolated. 16 outputs
// per workgroup (4 waves) or the tap rows by vector loads (lc_group_v, in order, 2 chunks ahead)
// were slower: 45.2, 59.5 us (profiles/r05/resample_lc_ab.txt).
constexpr int RLC_TN = 32;
constexpr int RLC_BLK = 64 * 8;   // threads per workgroup
constexpr int RLC_XL = 3;      // staged samples per lane and row: 64 * 3 >= the q span + look-back
constexpr int RLC_HL = 2;      // staged taps per lane and polyphase row: 64 * 2 >= L4

// four outputs of the 247/640 resampler whose q offsets from the first are (0, D1, D2, D3):
// acc[k] = sum_{j<101} hr[k*L4 + j] * x[q_k - j] in ascending j, x[q_0 - 100 + i] = xr[i]
template <int D1, int D2, int D3>
__device__ __forceinline__ void lc_group(const float* __restrict__ xr, const float* __restrict__ hr, int L4,
                                         float (&acc)[4]) {
    constexpr int NW = D3 + 101;
    constexpr int DK[4] = {0, D1, D2, D3};
    float w[NW];
#pragma unroll
    for (int i = 0; i < NW; i++) w[i] = xr[i];
#pragma unroll
    for (int k = 0; k < 4; k++) acc[k] = 0.0f;
    // taps of the 4 rows, 4 at a time (16-byte broadcasts), one chunk ahead; the barriers keep the
    // scheduler from hoisting every chunk's reads (4 x 104 registers) to the top
    float4 cur[4], nxt[4];
#pragma unroll
    for (int k = 0; k < 4; k++) cur[k] = *reinterpret_cast<const float4*>(hr + k * L4);
#pragma unroll
    for (int j0 = 0; j0 < 104; j0 += 4) {
        if (j0 + 4 < 104) {
#pragma unroll
            for (int k = 0; k < 4; k++) nxt[k] = *reinterpret_cast<const float4*>(hr + k * L4 + j0 + 4);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const float hv[4] = {cur[k].x, cur[k].y, cur[k].z, cur[k].w};
#pragma unroll
            for (int jj = 0; jj < 4; jj++) {
                const int j = j0 + jj;
                if (j < 101) acc[k] = acc[k] + hv[jj] * w[DK[k] + 100 - j];     // filter.cpp:139-141
            }
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int k = 0; k < 4; k++) cur[k] = nxt[k];
    }
}

// The same four outputs with the tap rows read by hand-issued scalar loads from the polyphase table
// (hr[k]: row of output k, wave-uniform) instead of LDS broadcasts: the rows are wave-uniform
// operands, so they need no LDS (the tile's x window alone fits three workgroups per CU instead of
// two) and no LDS bandwidth (the 16-byte broadcasts were most of the kernel's LDS traffic). Chunks
// of 4 taps of the 4 rows, one chunk ahead (scalar loads return out of order: every wait is
// lgkmcnt(0), as in k_fir_rb).
template <int D1, int D2, int D3>
__device__ __forceinline__ void lc_group_s(const float* __restrict__ xr, const float* h0, const float* h1,
                                           const float* h2, const float* h3, float (&acc)[4]) {
    constexpr int NW = D3 + 101;
    constexpr int DK[4] = {0, D1, D2, D3};
    constexpr int TC = 4, NC = 104 / TC;                   // rows padded past 101 (the table has slack)
    typedef float f4v __attribute__((ext_vector_type(TC)));
    float w[NW];
#pragma unroll
    for (int i = 0; i < NW; i++) w[i] = xr[i];
#pragma unroll
    for (int k = 0; k < 4; k++) acc[k] = 0.0f;
    const float* hr[4] = {h0, h1, h2, h3};
    f4v buf[2][4];
    auto load = [&](f4v& d, const float* hp, int c) {
        asm volatile("s_load_dwordx4 %0, %1, %2" : "=s"(d) : "s"(hp), "s"(c * TC * 4) : "memory");
    };
#pragma unroll
    for (int k = 0; k < 4; k++) load(buf[0][k], hr[k], 0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int k = 0; k < 4; k++) asm volatile("" : "+s"(buf[0][k]));   // no tap use above the wait
#pragma unroll
    for (int c = 0; c < NC; c++) {
#pragma unroll
        for (int kk = 0; kk < TC; kk++) {
            const int j = c * TC + kk;
            if (j < 101) {
#pragma unroll
                for (int k = 0; k < 4; k++) acc[k] = acc[k] + buf[c & 1][k][kk] * w[DK[k] + 100 - j];   // filter.cpp:139-141
            }
            if (kk == 0 && c + 1 < NC) {
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int k = 0; k < 4; k++) load(buf[(c + 1) & 1][k], hr[k], c + 1);
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        if (c + 1 < NC) {
            __builtin_amdgcn_sched_barrier(0);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // chunk c + 1 landed
#pragma unroll
            for (int k = 0; k < 4; k++) asm volatile("" : "+s"(buf[(c + 1) & 1][k]));
            __builtin_amdgcn_sched_barrier(0);
        }
    }
#pragma unroll
    for (int k = 0; k < 4; k++) asm volatile("" : "+v"(acc[k]));
}

template <int NTAP>   // > 0: every polyphase row has exactly NTAP taps (fully unrolled sums)
__global__ __launch_bounds__(RLC_BLK) void k_resample_lc(const float* __restrict__ x, size_t x_stride, int hist_lo,
                                                     const float* __restrict__ hp, const int* __restrict__ cnt,
                                                     int L, const int* __restrict__ ptq, int ny, int nch,
                                                     float* __restrict__ y, size_t y_stride) {
    extern __shared__ float4 smem4[];
    float* smem = reinterpret_cast<float*>(smem4);
    constexpr int PW = RLC_TN / (RLC_BLK / 64);              // outputs per wave
    const int c0 = blockIdx.y * 64, n0 = blockIdx.x * RLC_TN;
    const int nn = min(RLC_TN, ny - n0);
    // wave index as a scalar: the per-output table reads (ptq, cnt) are then scalar loads issued
    // together, not vector loads each waiting for every load before it
    const int wave = __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6), lane = threadIdx.x & 63;
    const int qlo = (ptq[n0] >> 8) - (L - 1);
    const int W = (ptq[n0 + nn - 1] >> 8) - qlo + 1;
    const int SW = W | 1;
    const int L4 = (L + 3) & ~3;
    // NTAP == 101: the tap rows come from the table by scalar loads (lc_group_s), not from LDS
    constexpr bool STAGE_TAPS = NTAP != 101;
    float* sx = smem;                                        // [64][SW]
    float* sh = smem + ((64 * SW + 3) & ~3);                 // [RLC_TN][L4] (STAGE_TAPS)
    // staging with every load of a wave in flight before its LDS writes: rows c = wave + 4u of the
    // x tile (lanes along the row, RLC_XL loads per row), then the polyphase rows of the outputs
    {
        constexpr int NR = 64 / (RLC_BLK / 64);
        float v[NR][RLC_XL];
#pragma unroll
        for (int u = 0; u < NR; u++) {
            const int ch = min(c0 + wave + u * (RLC_BLK / 64), nch - 1);
            const float* xc = x + (size_t)ch * x_stride;
#pragma unroll
            for (int k = 0; k < RLC_XL; k++) {
                const int i = lane + 64 * k, m = qlo + i;
                v[u][k] = (i < W && m >= hist_lo) ? xc[m] : 0.0f;
            }
        }
        // the polyphase rows' loads go out with the x tile's, before any LDS write waits for them
        // (one round of global-memory latency per workgroup instead of two)
        float hv[PW][RLC_HL];
        if (STAGE_TAPS) {
#pragma unroll
            for (int o8 = 0; o8 < PW; o8++) {
                const int o = min(wave * PW + o8, nn - 1);
                const int ph = ptq[n0 + o] & 255;
                const int cn = cnt[ph];
#pragma unroll
                for (int k = 0; k < RLC_HL; k++) {
                    const int j = lane + 64 * k;
                    hv[o8][k] = (j < cn) ? hp[(size_t)ph * L + j] : 0.0f;
                }
            }
        }
#pragma unroll
        for (int u = 0; u < NR; u++) {
            const int c = wave + u * (RLC_BLK / 64);
#pragma unroll
            for (int k = 0; k < RLC_XL; k++) {
                const int i = lane + 64 * k;
                if (i < W) sx[c * SW + i] = v[u][k];
            }
        }
        if (STAGE_TAPS) {
#pragma unroll
            for (int o8 = 0; o8 < PW; o8++) {
                const int o = wave * PW + o8;
#pragma unroll
                for (int k = 0; k < RLC_HL; k++) {
                    const int j = lane + 64 * k;
                    if (o < nn && j < L4) sh[o * L4 + j] = hv[o8][k];
                }
            }
        }
    }
    __syncthreads();
    const int ch = c0 + lane;
    float out[PW];
    if (NTAP == 101) {
        // groups of 4 consecutive outputs from one register window: their q offsets (q_k - q_0) follow
        // one of four patterns for the 247/640 ratio (the fraction of 640 n / 247 picks it), a
        // wave-uniform branch into statically indexed code; the window is read from LDS once per
        // group (109 samples for 4 outputs instead of 4 x 101) and each tap row as 16-byte broadcasts
        static_assert(PW % 4 == 0, "whole groups");
#pragma unroll
        for (int g = 0; g < PW / 4; g++) {
            const int o = wave * PW + 4 * g;
            bool done = false;
            if (o + 3 < nn) {
                const int q0 = ptq[n0 + o] >> 8;
                const int d1 = (ptq[n0 + o + 1] >> 8) - q0, d2 = (ptq[n0 + o + 2] >> 8) - q0,
                          d3 = (ptq[n0 + o + 3] >> 8) - q0;
                const float* xr = sx + lane * SW + (q0 - qlo) - 100;   // xr[i] = x[q0 - 100 + i]
                // the 4 outputs' polyphase rows in the table (wave-uniform addresses)
                const float* h0 = hp + (size_t)__builtin_amdgcn_readfirstlane((ptq[n0 + o] & 255) * L);
                const float* h1 = hp + (size_t)__builtin_amdgcn_readfirstlane((ptq[n0 + o + 1] & 255) * L);
                const float* h2 = hp + (size_t)__builtin_amdgcn_readfirstlane((ptq[n0 + o + 2] & 255) * L);
                const float* h3 = hp + (size_t)__builtin_amdgcn_readfirstlane((ptq[n0 + o + 3] & 255) * L);
                float acc4[4];
                done = true;
                if (d1 == 3 && d2 == 5 && d3 == 8) lc_group_s<3, 5, 8>(xr, h0, h1, h2, h3, acc4);
                else if (d1 == 2 && d2 == 5 && d3 == 7) lc_group_s<2, 5, 7>(xr, h0, h1, h2, h3, acc4);
                else if (d1 == 2 && d2 == 5 && d3 == 8) lc_group_s<2, 5, 8>(xr, h0, h1, h2, h3, acc4);
                else if (d1 == 3 && d2 == 6 && d3 == 8) lc_group_s<3, 6, 8>(xr, h0, h1, h2, h3, acc4);
                else done = false;
                if (done) {
#pragma unroll
                    for (int k = 0; k < 4; k++) out[4 * g + k] = acc4[k];
                }
            }
            if (!done) {
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    float acc = 0.0f;
                    if (o + k < nn) {
                        const int e = ptq[n0 + o + k];
                        const float* xr = sx + lane * SW + ((e >> 8) - qlo);
                        const float* hr = hp + (size_t)(e & 255) * L;   // (the table: taps are not staged)
                        for (int j = 0; j < 101; j++) acc = acc + hr[j] * xr[-j];
                    }
                    out[4 * g + k] = acc;
                }
            }
        }
    } else
#pragma unroll
    for (int o8 = 0; o8 < PW; o8++) {
        const int o = wave * PW + o8;
        float acc = 0.0f;
        if (o < nn) {
            const int e = ptq[n0 + o];
            const int cn = cnt[e & 255];
            const float* xr = sx + lane * SW + ((e >> 8) - qlo);  // x[q - j] = xr[-j]
            const float* hr = sh + o * L4;
            if (NTAP > 0) {
#pragma unroll
                for (int j = 0; j < NTAP; j++) acc = acc + hr[j] * xr[-j];
            } else {
            int j = 0;
            for (; j + 4 <= cn; j += 4) {
                const float4 h4 = *reinterpret_cast<const float4*>(hr + j);
                acc = acc + h4.x * xr[-j];
                acc = acc + h4.y * xr[-j - 1];
                acc = acc + h4.z * xr[-j - 2];
                acc = acc + h4.w * xr[-j - 3];
            }
            for (; j < cn; j++) acc = acc + hr[j] * xr[-j];
            }
        }
        out[o8] = acc;
    }
    if (ch < nch) {
        float* yo = y + (size_t)ch * y_stride + n0 + wave * PW;
        const int m = min(PW, nn - wave * PW);
#pragma unroll
        for (int o8 = 0; o8 < PW; o8++)
            if (o8 < m) yo[o8] = out[o8];
    }
}

int resample_lc_span(int L, int U, int D) {   // samples a tile reads: q span + look-back
    return (int)(((long long)(RLC_TN - 1) * D + U - 1) / U) + 1 + L;
}

size_t resample_lc_lds_bytes(int L, int U, int D, bool stage_taps) {
    const int W = resample_lc_span(L, U, D);
    return (size_t)((((64 * (W | 1)) + 3) & ~3) + (stage_taps ? RLC_TN * ((L + 3) & ~3) : 0)) * sizeof(float);
}

// ------------------------------------------------------------------------------------------
// Audio resamplers with U == 1 (mode 0: D = 5, mode 1: D = 9; filter.cpp:123-147 with one
// polyphase row of 101 taps), register-blocked: a thread computes AR consecutive outputs from a
// window of D*(AR-1) + 101 samples read once from LDS, the taps are scalar operands fetched in
// chunks of 4 by hand-issued scalar loads (as k_fir_rb), and every output sums h[j] * x[nD - j] in
// ascending j as an f32 product then an f32 add.
// ------------------------------------------------------------------------------------------
constexpr int AR = 4;                       // audio outputs per thread
constexpr int AT = 128;                     // threads per workgroup
constexpr int ATILE = AR * AT;              // audio outputs per workgroup

// acc[r] = sum_{j<101} h[j] * w[D*r + 100 - j] (ascending j), h wave-uniform
template <int D, int NW>
__device__ __forceinline__ void audio_mac(const float* __restrict__ h, const float (&w)[NW], float (&acc)[AR]) {
    constexpr int T = 101, TC = 4, NC = (T + TC - 1) / TC;   // tap buffers are padded past 101
    typedef float f4v __attribute__((ext_vector_type(TC)));
    f4v buf[2];
    auto load = [&](f4v& d, int c) {
        asm volatile("s_load_dwordx4 %0, %1, %2" : "=s"(d) : "s"(h), "s"(c * TC * 4) : "memory");
    };
#pragma unroll
    for (int r = 0; r < AR; r++) acc[r] = 0.0f;
    load(buf[0], 0);
    asm volatile("s_waitcnt lgkmcnt(0)" : "+s"(buf[0]) :: "memory");   // no tap use above the wait
#pragma unroll
    for (int c = 0; c < NC; c++) {
#pragma unroll
        for (int kk = 0; kk < TC; kk++) {
            const int j = c * TC + kk;
            if (j < T) {
#pragma unroll
                for (int r = 0; r < AR; r++) acc[r] = acc[r] + buf[c & 1][kk] * w[D * r + T - 1 - j];
            }
            if (kk == 0 && c + 1 < NC) {
                __builtin_amdgcn_sched_barrier(0);
                load(buf[(c + 1) & 1], c + 1);
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        if (c + 1 < NC) {
            __builtin_amdgcn_sched_barrier(0);
            asm volatile("s_waitcnt lgkmcnt(0)" : "+s"(buf[(c + 1) & 1]) :: "memory");
            __builtin_amdgcn_sched_barrier(0);
        }
    }
#pragma unroll
    for (int r = 0; r < AR; r++) asm volatile("" : "+v"(acc[r]));
}

// thread tid's window of a tile staged at s (16-byte aligned: D*AR*tid floats in)
template <int D, int NW>
__device__ __forceinline__ void audio_window(const float* __restrict__ s, int tid, float (&w)[NW]) {
    static_assert((D * AR) % 4 == 0 && NW % 4 == 0, "16-byte LDS reads");
    const float4* p = reinterpret_cast<const float4*>(s + D * AR * tid);
#pragma unroll
    for (int i = 0; i < NW / 4; i++) {
        const float4 v = p[i];
        w[4 * i] = v.x; w[4 * i + 1] = v.y; w[4 * i + 2] = v.z; w[4 * i + 3] = v.w;
    }
}

template <int D>
constexpr int audio_win() { return D * (ATILE - 1) + 101; }         // staged samples per tile
template <int D>
constexpr int audio_tw() { return (D * (AR - 1) + 101 + 3) / 4 * 4; }   // window of one thread

// mono (mono.cpp:34-42): audio = short(16384 * resample(fm_demod))
template <int D>
__global__ __launch_bounds__(AT) void k_mono_out(const float* __restrict__ fm, size_t fm_stride,
                                                 const float* __restrict__ h, int n, int ny,
                                                 int16_t* __restrict__ audio, size_t audio_stride,
                                                 const Poison err) {
    constexpr int WIN = audio_win<D>(), TW = audio_tw<D>();
    __shared__ __attribute__((aligned(16))) float sa[(WIN + 3) / 4 * 4 + 4];
    __shared__ uint32_t s_poison;                            // one decision per workgroup
    const int ch = blockIdx.y, tid = threadIdx.x;
    if (tid == 0) s_poison = poison_word(err);
    const int o0 = blockIdx.x * ATILE;
    const int m0 = D * o0 - 100;
    const float* x = fm + (size_t)ch * fm_stride;
    const int kend = min(WIN, n - m0);                       // staged slots past the block feed only outputs >= ny
    {
        constexpr int NL = (WIN + AT - 1) / AT;              // every load of the tile in flight at once
        float v[NL];
#pragma unroll
        for (int u = 0; u < NL; u++) {
            const int k = tid + u * AT;
            v[u] = k < kend ? x[m0 + k] : 0.0f;
        }
#pragma unroll
        for (int u = 0; u < NL; u++)
            if (tid + u * AT < WIN) sa[tid + u * AT] = v[u];
    }
    __syncthreads();
    const int ob = o0 + tid * AR;
    if (ob >= ny) return;
    int16_t* o = audio + (size_t)ch * audio_stride + ob;
    if (s_poison != 0u) {        // fm_demod may hold another block's samples (a release wait timed out)
#pragma unroll
        for (int r = 0; r < AR; r++)
            if (ob + r < ny) o[r] = SDR_PCM_POISON;
        return;
    }
    const uint32_t late = poison_late(err);                  // after every input load of the tile
    float w[TW], acc[AR];
    audio_window<D>(sa, tid, w);
    audio_mac<D>(h, w, acc);
    const bool bad = __builtin_amdgcn_readfirstlane(late) != 0u;
#pragma unroll
    for (int r = 0; r < AR; r++)
        if (ob + r < ny) o[r] = bad ? (int16_t)SDR_PCM_POISON : cvt_i16_x86(16384 * acc[r]);   // mono.cpp:41
}

// ------------------------------------------------------------------------------------------
// Stereo post stage in one pass (stereo.cpp:83-107, U == 1). The staging of an audio tile
// computes, for every IF sample of its window, the 38 kHz carrier from the PLL phase (pll.cpp:52;
// carrier[0] is the previous block's last), the mixer product stereo_dc = RN32(2.0 * band *
// carrier) in f64 (stereo.cpp:83-85), and the mono delay fm[i - 50] (the 101-tap APF of :88 is
// an exact 50-sample shift); each thread then runs both resamplers over its register windows and
// writes L = short(16384 (m + s)), R = short(16384 (m - s)) (:100-107). The carrier and stereo_dc
// rows never reach HBM: only stereo_dc's last HIST samples (the next block's resampler history)
// and carrier[n] (the next block's carrier[0], and pllblock_args.lastCarrier) are stored.
// ------------------------------------------------------------------------------------------
struct StereoOut {
    const float* fm;            // this parity's fm_demod, extended (fm[-HIST..n))
    const float* band;          // band BPF output of this parity
    const float* t;             // PLL phases of this parity
    size_t fm_stride, plain_stride;
    float* car;                 // carrier rows of this parity: [ch][n] written
    const float* car_prev;      // the previous parity's: [ch][n] read
    size_t car_stride;
    sdr_pll_state* st;
    float ncoScale, phaseAdjust;
    float* sdc;                 // stereo_dc rows of this parity: the tail [n - HIST, n) written
    const float* sdc_prev;      // the previous parity's tail: this block's history
    size_t sdc_stride;
    const float* h;             // the 101 audio taps
    int n, ny;
    int16_t* lr;
    size_t lr_stride;
    Poison err;                 // the block's error words (persistent PLL launch, release timeout)
};

template <int D>
__global__ __launch_bounds__(AT) void k_stereo_out(const StereoOut a) {
    constexpr int WIN = audio_win<D>(), TW = audio_tw<D>();
    __shared__ __attribute__((aligned(16))) float sa[(WIN + 3) / 4 * 4 + 4];
    __shared__ __attribute__((aligned(16))) float sb[(WIN + 3) / 4 * 4 + 4];
    __shared__ uint32_t s_poison;                                  // one decision per workgroup
    const int ch = blockIdx.y, tid = threadIdx.x;
    const int o0 = blockIdx.x * ATILE;
    if (tid == 0) s_poison = poison_word(a.err);                   // read beside the staging loads
    const int m0 = D * o0 - 100;
    const bool last_tile = o0 + ATILE >= a.ny;
    // the last tile also computes up to the block end: stereo_dc's tail is the next block's history
    const int m1 = last_tile ? a.n : min(m0 + WIN, a.n);
    const float* fm = a.fm + (size_t)ch * a.fm_stride;
    const float* band = a.band + (size_t)ch * a.plain_stride;
    const float* tt = a.t + (size_t)ch * a.plain_stride;
    const float* sprev = a.sdc_prev + (size_t)ch * a.sdc_stride;
    float* scur = a.sdc + (size_t)ch * a.sdc_stride;
    const float car0 = a.car_prev[(size_t)ch * a.car_stride + a.n];
    // every load of the tile in flight at once (m1 <= m0 + WIN: the window of the last tile reaches
    // the block end), then the carriers, mixer products and LDS writes
    constexpr int NL = (WIN + AT - 1) / AT;
    float vb[NL], vt[NL], vf[NL];
#pragma unroll
    for (int u = 0; u < NL; u++) {
        const int i = m0 + tid + u * AT;
        const bool in = i < m1;
        vf[u] = in ? fm[i - 50] : 0.0f;                            // stereo.cpp:88
        vb[u] = (in && i >= 0) ? band[i] : (in ? sprev[a.n + i] : 0.0f);   // i >= -100: history
        vt[u] = (in && i > 0) ? tt[i - 1] : 0.0f;
    }
#pragma unroll
    for (int u = 0; u < NL; u++) {
        const int i = m0 + tid + u * AT, k = i - m0;
        if (i >= m1) continue;
        float sd = vb[u];
        if (i >= 0) {
            const float car = (i == 0) ? car0 : nco_carrier(vt[u], a.ncoScale, a.phaseAdjust);
            sd = (float)(2.0 * (double)vb[u] * (double)car);         // stereo.cpp:83-85
            if (i >= a.n - HIST) scur[i] = sd;
        }
        sb[k] = sd;
        sa[k] = vf[u];
    }
    if (last_tile && tid == 0) {                                   // carrier[n] (pll.cpp:52, :58)
        const float cl = nco_carrier(tt[a.n - 1], a.ncoScale, a.phaseAdjust);
        a.car[(size_t)ch * a.car_stride + a.n] = cl;
        a.st[ch].lastCarrier = cl;
    }
    __syncthreads();
    const int ob = o0 + tid * AR;
    if (ob >= a.ny) return;
    uint32_t* o = reinterpret_cast<uint32_t*>(a.lr + (size_t)ch * a.lr_stride) + ob;
    if (s_poison != 0u) {
        // a persistent PLL wait timed out (this block's phases were never computed, or not yet) or a
        // release wait did (the inputs may hold another block): the consumer gets a marked block
        // instead of audio (include/sdr_amd.h SDR_PCM_POISON)
        const uint32_t pp = (uint32_t)(uint16_t)SDR_PCM_POISON * 0x10001u;
#pragma unroll
        for (int r = 0; r < AR; r++)
            if (ob + r < a.ny) o[r] = pp;
        return;
    }
    const uint32_t late = poison_late(a.err);                      // after every input load of the tile
    float w[TW], m[AR], sv[AR];
    audio_window<D>(sa, tid, w);
    audio_mac<D>(a.h, w, m);                                       // mono resampler (:94)
    audio_window<D>(sb, tid, w);
    audio_mac<D>(a.h, w, sv);                                      // stereo resampler (:97)
    const bool bad = __builtin_amdgcn_readfirstlane(late) != 0u;
#pragma unroll
    for (int r = 0; r < AR; r++) {
        if (ob + r < a.ny) {
            const uint16_t l = (uint16_t)cvt_i16_x86(16384 * (m[r] + sv[r]));   // stereo.cpp:100-102
            const uint16_t rr = (uint16_t)cvt_i16_x86(16384 * (m[r] - sv[r]));
            o[r] = bad ? (uint32_t)(uint16_t)SDR_PCM_POISON * 0x10001u : (uint32_t)l | ((uint32_t)rr << 16);
        }
    }
}

// the unfused post stages' poison (SDR_FLAG_KEEP_INTERMEDIATES, the generic resamplers): rows
// [nch][n] of int16 overwritten with SDR_PCM_POISON when one of the block's error words is set
__global__ __launch_bounds__(BLK) void k_poison_i16(const Poison err, int16_t* __restrict__ p, size_t stride,
                                                    int n) {
    if (poison_word(err) == 0u) return;
    const int i = blockIdx.x * BLK + threadIdx.x;
    if (i < n) p[(size_t)blockIdx.y * stride + i] = SDR_PCM_POISON;
}

// ------------------------------------------------------------------------------------------
// RDS carrier and mixer in one pass (rds.cpp:119-127): ipll[i] from the 114 kHz PLL's phase
// (pll.cpp:52, ncoScale 0.5; ipll[0] = the previous block's last) and rds_dc[i] = (2 * delay[i]) *
// ipll[i] in f32 with delay[i] = rds_band[i - 50] + 0 (the APF of :122 is an exact 50-sample
// shift that turns -0 into +0) into the extended rds_dc stream, history included. ipll itself is
// not stored: only its last sample (the next block's ipll[0], and pllblock_args.lastCarrier).
// MIX_R samples per thread; the thread whose range holds n computes ipll[n].
// ------------------------------------------------------------------------------------------
struct RdsMix {
    const float* rband;         // this parity's rds_band, extended
    const float* t;             // PLL phases of this parity
    size_t fm_stride, plain_stride;
    float* car;                 // ipll rows of this parity: [ch][n] written
    const float* car_prev;      // the previous parity's: [ch][n] read
    size_t car_stride;
    sdr_pll_state* st;
    float ncoScale, phaseAdjust;
    float* rdc;                 // this parity's rds_dc, extended (history copied by tile 0)
    const float* rdc_prev;
    float* rfilt;               // this parity's rds_filt, extended: its history is copied by tile 0 too
    const float* rfilt_prev;
    size_t rf_stride;
    int n, n_rds;
};

// MIX_R consecutive samples per thread: one 16-byte load of the phases, two 8-byte loads of the
// delayed band (i - 50 = 2 mod 4), one 16-byte store -- 4x the bytes in flight per wave of the
// one-sample form, which waited on memory 74 % of its time (profiles/r03/stage_counters_v7.json)
constexpr int MIX_R = 4;
__global__ __launch_bounds__(BLK) void k_rds_mix(const RdsMix a) {
    const int ch = blockIdx.y;
    const int i0 = ((int)blockIdx.x * BLK + (int)threadIdx.x) * MIX_R;
    const float* tt = a.t + (size_t)ch * a.plain_stride;
    const float* rb = a.rband + (size_t)ch * a.fm_stride;
    float* y = a.rdc + (size_t)ch * a.fm_stride;
    auto carrier = [&](int i, float tprev) {
        return (i == 0) ? a.car_prev[(size_t)ch * a.car_stride + a.n] : nco_carrier(tprev, a.ncoScale, a.phaseAdjust);
    };
    if (i0 + MIX_R <= a.n) {
        const float4 tv = *reinterpret_cast<const float4*>(tt + i0);
        const float tm = i0 > 0 ? tt[i0 - 1] : 0.0f;
        const float2 r01 = *reinterpret_cast<const float2*>(rb + i0 - 50);
        const float2 r23 = *reinterpret_cast<const float2*>(rb + i0 - 48);
        const float tp[MIX_R] = {tm, tv.x, tv.y, tv.z};
        const float dl[MIX_R] = {r01.x, r01.y, r23.x, r23.y};
        float o[MIX_R];
#pragma unroll
        for (int k = 0; k < MIX_R; k++) {
            const float d = dl[k] + 0.0f;                                  // rds.cpp:122
            o[k] = 2 * d * carrier(i0 + k, tp[k]);                         // rds.cpp:125-127
        }
        *reinterpret_cast<float4*>(y + i0) = make_float4(o[0], o[1], o[2], o[3]);
    } else {
        for (int k = 0; k < MIX_R; k++) {
            const int i = i0 + k;
            if (i < a.n) {
                const float d = rb[i - 50] + 0.0f;
                y[i] = 2 * d * carrier(i, i > 0 ? tt[i - 1] : 0.0f);
            } else if (i == a.n) {
                const float cl = nco_carrier(tt[a.n - 1], a.ncoScale, a.phaseAdjust);
                a.car[(size_t)ch * a.car_stride + a.n] = cl;
                a.st[ch].lastCarrier = cl;
            }
        }
    }
    if (blockIdx.x == 0 && threadIdx.x < HIST) {
        y[(int)threadIdx.x - HIST] = a.rdc_prev[(size_t)ch * a.fm_stride + a.n - HIST + threadIdx.x];
        a.rfilt[(size_t)ch * a.rf_stride + (int)threadIdx.x - HIST] =
            a.rfilt_prev[(size_t)ch * a.rf_stride + a.n_rds - HIST + threadIdx.x];
    }
}

// ------------------------------------------------------------------------------------------
// Mixers. stereo.cpp:83-85: stereo_dc = 2.0*band*carrier (f64 product, one rounding).
// rds.cpp:125-127: rds_dc = (2*delay)*ipll with delay[i] = rds_band[i-50] (the 101-tap APF of
// filter.cpp:73-78 is an exact 50-sample delay for finite inputs). Also copies the history.
// ------------------------------------------------------------------------------------------
template <bool RDS>
__global__ __launch_bounds__(BLK) void k_mix(const float* __restrict__ a, size_t a_stride,
                                             const float* __restrict__ c, size_t c_stride, int n,
                                             float* __restrict__ y, const float* __restrict__ y_other,
                                             size_t y_stride, int delay) {
    const int ch = blockIdx.y;
    const int i = blockIdx.x * BLK + threadIdx.x;
    const float* ac = a + (size_t)ch * a_stride;
    const float* cc = c + (size_t)ch * c_stride;
    float* yc = y + (size_t)ch * y_stride;
    if (i < n) {
        if (RDS) {
            const float d = ac[i - delay] + 0.0f;   // + 0.0f: the APF sum turns -0 into +0
            yc[i] = 2 * d * cc[i];
        } else {
            yc[i] = (float)(2.0 * (double)ac[i] * (double)cc[i]);
        }
    }
    if (blockIdx.x == 0 && threadIdx.x < HIST) {
        yc[(int)threadIdx.x - HIST] = y_other[(size_t)ch * y_stride + n - HIST + threadIdx.x];
    }
}

// The parity-release wait (release_wait): every word w[k] with bit k of mask reaches want[k] (counts
// stored by k_flag_store after the readers' kernels); polled relaxed, acquired once, bounded like the
// persistent PLL's waits. After ~5 s it gives up: it sets the context's sticky fail word (every output
// stage then poisons its block: a reader that runs after the producer's overwrite would read the
// next block's data) and its host-mapped mirror (the next stage call returns SDR_E_TIMEOUT) before it
// lets the stream go on, so no reader can start after the overwrite without seeing the word.
__global__ void k_rel_wait(const uint32_t* w, uint32_t want0, uint32_t want1, uint32_t want2, unsigned mask,
                           uint32_t* fail, uint32_t* fail_host) {
    if (threadIdx.x != 0) return;
    const uint32_t want[3] = {want0, want1, want2};
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    bool expired = false;
    for (int k = 0; k < 3 && !expired; k++) {
        if (!(mask & (1u << k))) continue;
        while ((int32_t)(__hip_atomic_load(w + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - want[k]) < 0) {
            __builtin_amdgcn_s_sleep(4);
            if (__builtin_amdgcn_s_memrealtime() - t0 > 500000000ull) {
                expired = true;
                break;
            }
        }
    }
    if (expired) {
        __hip_atomic_fetch_or(fail, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(fail_host, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");          // both visible before the kernel ends
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
}

// copy the previous parity's last HIST samples in front of this parity's stream
__global__ void k_hist_copy(float* __restrict__ y, const float* __restrict__ y_other, size_t stride, int n) {
    const int ch = blockIdx.x;
    for (int i = threadIdx.x; i < HIST; i += blockDim.x)
        y[(size_t)ch * stride + i - HIST] = y_other[(size_t)ch * stride + n - HIST + i];
}

// Rows [nch][n] f32 from src to dst, and with hist_other the HIST samples in front of each dst row
// from the end of hist_other's row (the extended-stream history, as k_hist_copy): one pass at HBM
// rate (16-byte vectors when both rows are 16-byte aligned), where hipMemcpy2DAsync's rectangle blit
// moved the 30 MB of a 1024-channel fm_demod block at ~2 TB/s (31.8 us, profiles/r06/queue/).
constexpr int CR_BLK = 256, CR_V = 4;    // threads per workgroup, float4s per thread
__global__ __launch_bounds__(CR_BLK) void k_copy_rows(float* __restrict__ dst, size_t dst_stride,
                                                       const float* __restrict__ src, size_t src_stride, int n,
                                                       const float* __restrict__ hist_other, int vec) {
    const int ch = blockIdx.y;
    float* d = dst + (size_t)ch * dst_stride;
    const float* a = src + (size_t)ch * src_stride;
    if (hist_other && blockIdx.x == 0)
        for (int i = threadIdx.x; i < HIST; i += CR_BLK) d[i - HIST] = hist_other[(size_t)ch * dst_stride + n - HIST + i];
    const int i0 = blockIdx.x * CR_BLK * CR_V * 4;   // first float of this workgroup
    if (vec) {
        typedef float f4 __attribute__((ext_vector_type(4)));
        f4* d4 = reinterpret_cast<f4*>(d + i0);
        const f4* a4 = reinterpret_cast<const f4*>(a + i0);
        f4 v[CR_V];
#pragma unroll
        for (int u = 0; u < CR_V; u++) {
            const int i = i0 + 4 * (threadIdx.x + u * CR_BLK);
            if (i + 3 < n) v[u] = __builtin_nontemporal_load(a4 + threadIdx.x + u * CR_BLK);
        }
#pragma unroll
        for (int u = 0; u < CR_V; u++) {
            const int i = i0 + 4 * (threadIdx.x + u * CR_BLK);
            if (i + 3 < n) d4[threadIdx.x + u * CR_BLK] = v[u];
            else for (int k = i; k < n && k < i + 4; k++) d[k] = a[k];
        }
    } else {
        for (int i = i0 + threadIdx.x; i < min(n, i0 + CR_BLK * CR_V * 4); i += CR_BLK) d[i] = a[i];
    }
}
int copy_rows(float* dst, size_t dst_stride, const float* src, size_t src_stride, int n, int nch,
              const float* hist_other, hipStream_t s) {
    const int vec = (reinterpret_cast<uintptr_t>(dst) % 16 == 0 && reinterpret_cast<uintptr_t>(src) % 16 == 0 &&
                     dst_stride % 4 == 0 && src_stride % 4 == 0) ? 1 : 0;
    hipLaunchKernelGGL(k_copy_rows, dim3(cdiv(n, CR_BLK * CR_V * 4), nch), dim3(CR_BLK), 0, s, dst, dst_stride, src,
                       src_stride, n, hist_other, vec);
    LAUNCH_CHECK();
    return SDR_OK;
}

// state <- last nstate of x (filter.cpp:119 / :145) for the primitive entry points
__global__ void k_state_update(float* __restrict__ state, int nstate, const float* __restrict__ x,
                               size_t x_stride, int nx) {
    const int ch = blockIdx.x;
    float* s = state + (size_t)ch * nstate;
    const float* xc = x + (size_t)ch * x_stride;
    if (nx >= nstate) {
        for (int i = threadIdx.x; i < nstate; i += blockDim.x) s[i] = xc[nx - nstate + i];
    } else {
        // shift (single workgroup per channel: read all, barrier, write)
        for (int base = 0; base < nstate; base += blockDim.x) {
            const int i = base + threadIdx.x;
            float v = 0.0f;
            if (i < nstate) v = (i + nx < nstate) ? s[i + nx] : xc[i + nx - nstate];
            __syncthreads();
            if (i < nstate) s[i] = v;
            __syncthreads();
        }
    }
}

// fmDemodNoArctan over separate I/Q arrays (demod.cpp:3-24); prev updated by k_demod_prev.
__global__ __launch_bounds__(BLK) void k_demod(float* __restrict__ out, size_t out_stride,
                                               const float* __restrict__ I, const float* __restrict__ Q,
                                               size_t iq_stride, int n, const float2* __restrict__ prev) {
    const int ch = blockIdx.y;
    const int i = blockIdx.x * BLK + threadIdx.x;
    if (i >= n) return;
    const float* Ic = I + (size_t)ch * iq_stride;
    const float* Qc = Q + (size_t)ch * iq_stride;
    const float ci = Ic[i], cq = Qc[i];
    const float2 pv = (i == 0) ? prev[ch] : make_float2(Ic[i - 1], Qc[i - 1]);
    float r;
    if ((ci == 0) & (cq == 0)) {
        r = 0.0f;
    } else {
        const float num = ci * (cq - pv.y) - cq * (ci - pv.x);
        const double den = (double)ci * (double)ci + (double)cq * (double)cq;
        r = (float)((double)num / den);
    }
    out[(size_t)ch * out_stride + i] = r;
}

__global__ void k_demod_prev(float2* __restrict__ prev, const float* __restrict__ I, const float* __restrict__ Q,
                             size_t iq_stride, int n, int nch) {
    const int ch = blockIdx.x * blockDim.x + threadIdx.x;
    if (ch < nch) prev[ch] = make_float2(I[(size_t)ch * iq_stride + n - 1], Q[(size_t)ch * iq_stride + n - 1]);
}

// cdr(), rds_utilities.cpp:4-21: argmax over offsets i < sps of sum_k |(int)x[k*sps+i]|,
// first maximum wins, 0 when every sum is 0. One wave per channel, one lane per offset; the argmax
// is a wave reduction of (sum, -offset) over the sums > 0 (the reference's strict > from maxv = 0).
__device__ __forceinline__ int cdr_wave(const float* x, int n, int sps) {
    const int lane = threadIdx.x;
    const int nk = n / sps;
    unsigned long long key = 0;                     // (sum << 32) | ~offset of this lane's best offset
    for (int i = lane; i < sps; i += 64) {
        uint32_t s = 0;
        for (int k = 0; k < nk; k++) {
            const int32_t v = cvt_i32_x86(x[k * sps + i]);
            s += (uint32_t)(v < 0 ? -(uint32_t)v : (uint32_t)v);
        }
        const int32_t si = (int32_t)s;
        const unsigned long long ki = si > 0 ? ((unsigned long long)(uint32_t)si << 32) | (uint32_t)~(uint32_t)i : 0ull;
        if (ki > key) key = ki;
    }
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) {
        const unsigned long long o = __shfl_xor(key, m, 64);
        if (o > key) key = o;
    }
    return key ? (int)~(uint32_t)(key & 0xFFFFFFFFull) : 0;
}

__global__ __launch_bounds__(64) void k_cdr(int32_t* __restrict__ offset, const float* __restrict__ x,
                                            size_t x_stride, int n, int sps) {
    const int ch = blockIdx.x;
    const int off = cdr_wave(x + (size_t)ch * x_stride, n, sps);
    if (threadIdx.x == 0) offset[ch] = off;
}

// RDS symbol and bit recovery for one block (rds.cpp:135-167): cdr, slicer (:157-161),
// manchester_decode (rds_utilities.cpp:34-68), differential_decode (:70-88).
// dec[ch*8 + {0..4}] = block_count, half_symbol, start, last_bit, sample_offset.
__global__ __launch_bounds__(64) void k_rds_bits(const float* __restrict__ x, size_t x_stride, int n, int sps,
                                                 int rds_on, int32_t* __restrict__ dec,
                                                 int32_t* __restrict__ offset_out, int32_t* __restrict__ nsym_out,
                                                 uint8_t* __restrict__ sym_out, size_t sym_stride,
                                                 int32_t* __restrict__ nbits_out, uint8_t* __restrict__ bits_out,
                                                 size_t bits_stride, const Poison err, int vec4) {
    // dynamic LDS: the channel's whole block (n floats), staged with every load in flight (the cdr
    // reads it 39-strided and the slicer sps-strided: from LDS, not global memory)
    extern __shared__ float4 xs4[];
    float* xs = reinterpret_cast<float*>(xs4);
    __shared__ uint8_t symbols[SDR_MAX_SYMS];
    const int ch = blockIdx.x;
    const int lane = threadIdx.x;
    int32_t* d = dec + (size_t)ch * DEC_STATE;
    const int block_count = d[0];
    const float* xc = x + (size_t)ch * x_stride;
    const bool decode = (block_count > 5) && rds_on;
    if (poison_word(err) != 0u) {   // a persistent PLL or release wait timed out: no bits from this block
        if (lane == 0) {
            if (offset_out) offset_out[ch] = -1;
            if (nsym_out) nsym_out[ch] = 0;
            if (nbits_out) nbits_out[ch] = SDR_NBITS_POISONED;
        }
        return;
    }
    if (!decode) {
        if (lane == 0) {
            if (offset_out) offset_out[ch] = d[4];
            if (nsym_out) nsym_out[ch] = 0;
            if (nbits_out) nbits_out[ch] = -1;
            d[0] = block_count + 1;
        }
        return;
    }
    {
        // the whole row in one round of loads where it fits: 16-byte loads when the row is aligned
        // (VEC4), then the LDS writes
        constexpr int U4 = 12;
        int i_tail = 0;
        if (vec4) {
            const int n4 = n >> 2;
            for (int q0 = lane; q0 < n4; q0 += 64 * U4) {
                // loads and LDS writes unconditional at a clamped index (lanes past the row rewrite its
                // last element with the same value): conditional ones went to scratch, or were sunk
                // next to their writes, one load in flight at a time
                float4 v[U4];
#pragma unroll
                for (int u = 0; u < U4; u++) v[u] = reinterpret_cast<const float4*>(xc)[min(q0 + 64 * u, n4 - 1)];
#pragma unroll
                for (int u = 0; u < U4; u++) reinterpret_cast<float4*>(xs)[min(q0 + 64 * u, n4 - 1)] = v[u];
            }
            i_tail = n4 * 4;
        }
        constexpr int U = 8;
        for (int i0 = i_tail + lane; i0 < n; i0 += 64 * U) {
            float v[U];
#pragma unroll
            for (int u = 0; u < U; u++) v[u] = (i0 + 64 * u < n) ? xc[i0 + 64 * u] : 0.0f;
#pragma unroll
            for (int u = 0; u < U; u++)
                if (i0 + 64 * u < n) xs[i0 + 64 * u] = v[u];
        }
        __syncthreads();
    }
    const int off = cdr_wave(xs, n, sps);
    int m = 0;
    if (off < n) m = (n - off + sps - 1) / sps;     // i with off + i*sps < n
    if (m > SDR_MAX_SYMS) m = SDR_MAX_SYMS;
    for (int i = lane; i < m; i += 64) symbols[i] = xs[off + i * sps] > 0;
    __syncthreads();
    // manchester_decode + differential_decode with every lane: bit k of the block is half_symbol
    // (k < nb0, a symbol pair split across blocks) or symbols[start + 2 (k - nb0)]; the outputs are
    // bits[k] ^ bits[k-1] (bits[-1] = the previous block's last bit), the state comes from the ends
    const int half_in = d[1], start_in = d[2], last_in = d[3];
    const int nb0 = start_in ? 1 : 0;
    int start = start_in;
    if (block_count == 0) {  // dead in the reference (decoding starts at block 6), kept for parity
        int score = 0;
        for (int i = 0; i < m - 1; i += 2) score += symbols[i] ^ symbols[i + 1];
        for (int j = 1; j < m - 1; j += 2) score -= symbols[j] ^ symbols[j + 1];
        start = score < 0;
    }
    const int npairs = m - 1 > start ? (m - start) / 2 : 0;       // i = start, start + 2, ... < m - 1
    const int nb = min(nb0 + npairs, SDR_MAX_BITS);
    auto bit_at = [&](int k) -> int { return k < nb0 ? half_in : symbols[start + 2 * (k - nb0)]; };
    uint8_t* bo = bits_out ? bits_out + (size_t)ch * bits_stride : nullptr;
    if (bo) {
        for (int k = lane; k < nb; k += 64) {
            const int prev = k == 0 ? (block_count == 0 ? 0 : last_in) : bit_at(k - 1);
            bo[k] = (uint8_t)(bit_at(k) ^ prev);
        }
    }
    if (sym_out) {
        uint8_t* so = sym_out + (size_t)ch * sym_stride;
        for (int i = lane; i < m; i += 64) so[i] = symbols[i];
    }
    if (lane == 0) {
        const bool odd = ((m - start) & 0x01) == 1;
        d[1] = odd ? symbols[m - 1] : half_in;
        d[2] = odd ? 1 : 0;
        d[3] = nb > 0 ? bit_at(nb - 1) : last_in;
        d[4] = off;
        d[0] = block_count + 1;
        if (offset_out) offset_out[ch] = off;
        if (nsym_out) nsym_out[ch] = m;
        if (nbits_out) nbits_out[ch] = nb;
    }
}

// manchester_decode (rds_utilities.cpp:34-68), one lane per channel
__global__ void k_manchester(uint8_t* __restrict__ bits, size_t bits_stride, int32_t* __restrict__ nbits,
                             const uint8_t* __restrict__ symbols, size_t sym_stride,
                             const int32_t* __restrict__ nsym, int nch, int block_count,
                             int32_t* __restrict__ state) {
    const int ch = blockIdx.x * blockDim.x + threadIdx.x;
    if (ch >= nch) return;
    const uint8_t* sy = symbols + (size_t)ch * sym_stride;
    uint8_t* bo = bits + (size_t)ch * bits_stride;
    const int m = nsym[ch];
    int half_symbol = state[2 * ch], start = state[2 * ch + 1];
    int nb = 0;
    if (start) bo[nb++] = (uint8_t)half_symbol;
    if (block_count == 0) {
        int score = 0;
        for (int i = 0; i < m - 1; i += 2) score += sy[i] ^ sy[i + 1];
        for (int j = 1; j < m - 1; j += 2) score -= sy[j] ^ sy[j + 1];
        start = score < 0;
    }
    for (int i = start; i < m - 1; i += 2) bo[nb++] = sy[i];
    if (((m - start) & 0x01) == 1) {
        half_symbol = sy[m - 1];
        start = 1;
    } else {
        start = 0;
    }
    state[2 * ch] = half_symbol;
    state[2 * ch + 1] = start;
    nbits[ch] = nb;
}

// differential_decode (rds_utilities.cpp:70-88), one lane per channel
__global__ void k_differential(uint8_t* __restrict__ out, size_t out_stride, const uint8_t* __restrict__ bits,
                               size_t bits_stride, const int32_t* __restrict__ nbits, int nch, int block_num,
                               int32_t* __restrict__ last_bit) {
    const int ch = blockIdx.x * blockDim.x + threadIdx.x;
    if (ch >= nch) return;
    const int nb = nbits[ch];
    if (nb <= 0) return;
    const uint8_t* b = bits + (size_t)ch * bits_stride;
    uint8_t* o = out + (size_t)ch * out_stride;
    o[0] = (block_num == 0) ? b[0] : (uint8_t)(b[0] ^ (uint8_t)last_bit[ch]);
    for (int i = 1; i < nb; i++) o[i] = b[i] ^ b[i - 1];
    last_bit[ch] = b[nb - 1];
}

// x[ch][col] = v for every channel row (the carried last NCO sample at initialisation)
__global__ void k_set_col(float* x, size_t stride, int col, int nch, float v) {
    const int ch = blockIdx.x * blockDim.x + threadIdx.x;
    if (ch < nch) x[(size_t)ch * stride + col] = v;
}

__global__ void k_fill_u8(uint8_t* p, uint8_t v, size_t n) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = v;
}

// Bandwidth calibration (sdr_hbm_copy): one 16-byte element per lane, one short-lived workgroup per
// 4 KiB -- the fastest plain copy measured on this device (tools/hbm_copy_bench.hip: 6.2 TB/s, where
// grid-stride loops with 1-8 loads in flight per lane reach 4.1-5.7) -- the HBM rate a plain stream
// reaches, the practical ceiling the front end's roofline fraction is read against.
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
__global__ __launch_bounds__(256) void k_hbm_copy(u32x4* __restrict__ dst, const u32x4* __restrict__ src, size_t n) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) dst[i] = src[i];
}


size_t fir_lds_bytes(int ntaps, int nt, int tile, int D) {
    const int ntaps_pad = (ntaps + 3) & ~3;
    const int W = (tile - 1) * D + ntaps;
    return (size_t)(nt * ntaps_pad + W + 4) * sizeof(float);
}

size_t resample_lds_bytes(int L, int U, int D, int tile, int ninputs) {
    const int W = (int)(((long long)tile * D) / U) + L + 2;
    return (size_t)ninputs * ((W + 3) & ~3) * sizeof(float) + 64;
}

// polyphase tap table: row p holds h[p], h[p+U], ... (cnt[p] entries), rows padded to L
struct Polyphase {
    std::vector<float> table;
    std::vector<int> cnt;
    int L = 0;
};

Polyphase make_polyphase(const std::vector<float>& h, int U) {
    Polyphase p;
    const int ntaps = (int)h.size();
    int maxc = 0;
    p.cnt.resize(U);
    for (int ph = 0; ph < U; ph++) {
        p.cnt[ph] = ph < ntaps ? (ntaps - ph + U - 1) / U : 0;
        maxc = std::max(maxc, p.cnt[ph]);
    }
    p.L = (maxc + 3) & ~3;
    p.table.assign((size_t)U * p.L, 0.0f);
    for (int ph = 0; ph < U; ph++)
        for (int j = 0; j < p.cnt[ph]; j++) p.table[(size_t)ph * p.L + j] = h[ph + (size_t)U * j];
    return p;
}

}  // namespace

namespace {

template <typename T>
int dalloc(sdr_ctx* c, T** p, size_t count) {
    void* v = nullptr;
    HIP_TRY(hipMalloc(&v, count * sizeof(T) + 256));
    HIP_TRY(hipMemset(v, 0, count * sizeof(T) + 256));
    c->allocs.push_back(v);
    *p = static_cast<T*>(v);
    return SDR_OK;
}

template <typename T>
int upload(sdr_ctx* c, T** p, const std::vector<T>& host) {
    int r = dalloc(c, p, host.size());
    if (r) return r;
    HIP_TRY(hipMemcpy(*p, host.data(), host.size() * sizeof(T), hipMemcpyHostToDevice));
    return SDR_OK;
}

int fill_info(sdr_info* in, int nch, int mode, int rds_on) {
    std::memset(in, 0, sizeof(*in));
    in->nch = nch;
    in->mode = mode;
    in->rds_on = rds_on;
    in->rf_taps = 101;
    in->rf_Fs = 2400000; in->rf_decim = 10; in->if_Fs = 240000; in->audio_upsample = 1;
    in->audio_decim = 5; in->symbol_Fs = 39;
    switch (mode) {  // project.cpp:67-108
        case 0: break;
        case 1: in->rf_Fs = 1440000; in->rf_decim = 4; in->audio_decim = 9; in->if_Fs = 360000; break;
        case 2: in->audio_decim = 800; in->audio_upsample = 147; in->symbol_Fs = 20; break;
        case 3: in->rf_Fs = 1152000; in->rf_decim = 3; in->audio_decim = 1280; in->if_Fs = 384000;
                in->audio_upsample = 147; in->symbol_Fs = 20; break;
        default: return fail(SDR_E_INVALID, "mode %d not in 0..3", mode);
    }
    const int U = in->audio_upsample, D = in->audio_decim;
    in->block_iq = (1470 * in->rf_decim * D) / U;
    in->block_if = (1470 * D) / U;
    in->n_audio = in->block_if * U / D;
    in->n_rds = in->block_if * 247 / 640;
    in->history = HIST;
    return SDR_OK;
}

int init_state(sdr_ctx* c, hipStream_t s) {
    const sdr_info& in = c->info;
    // every buffer back to zero (the reference's value-initialised vectors)
    HIP_TRY(hipMemsetAsync(c->fm - HIST, 0, 2 * c->fm_par * sizeof(float), s));
    HIP_TRY(hipMemsetAsync(c->sdc - HIST, 0, 2 * c->fm_par * sizeof(float), s));
    HIP_TRY(hipMemsetAsync(c->rband - HIST, 0, 2 * c->fm_par * sizeof(float), s));
    HIP_TRY(hipMemsetAsync(c->rdc - HIST, 0, 2 * c->fm_par * sizeof(float), s));
    HIP_TRY(hipMemsetAsync(c->rfilt - HIST, 0, 2 * c->rf_par * sizeof(float), s));
    const size_t tail_bytes = (size_t)2 * c->nch * 2 * (c->ntaps - 1);
    hipLaunchKernelGGL(k_fill_u8, dim3((unsigned)((tail_bytes + 255) / 256)), dim3(256), 0, s, c->tail,
                       (uint8_t)128, tail_bytes);  // u8 128 == 0.0f: zero FIR state
    LAUNCH_CHECK();
    HIP_TRY(hipMemsetAsync(c->prev, 0, (size_t)2 * c->nch * sizeof(float2), s));
    std::vector<sdr_pll_state> st(c->nch);
    for (auto& p : st) p = sdr_pll_state{1.0f, 0.0f, 0.0f, 0.0f, 0.0, 1.0f};  // stereo.cpp:51-57, :45
    HIP_TRY(hipMemcpyAsync(c->st_pll, st.data(), st.size() * sizeof(sdr_pll_state), hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(c->rds_pll, st.data(), st.size() * sizeof(sdr_pll_state), hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemsetAsync(c->dec, 0, (size_t)c->nch * DEC_STATE * sizeof(int32_t), s));
    // carrier[0] of the first block = lastCarrier = 1 (stereo.cpp:45): the NCO reads it from the
    // other parity's row end
    for (int p = 0; p < 2; p++) {
        hipLaunchKernelGGL(k_set_col, dim3(cdiv(c->nch, 64)), dim3(64), 0, s, c->carrier + p * c->pll_par, c->pll_stride,
                           in.block_if, c->nch, 1.0f);
        hipLaunchKernelGGL(k_set_col, dim3(cdiv(c->nch, 64)), dim3(64), 0, s, c->ipll + p * c->pll_par, c->pll_stride,
                           in.block_if, c->nch, 1.0f);
    }
    LAUNCH_CHECK();
    HIP_TRY(hipStreamSynchronize(s));
    c->parity = 1;
    c->block = -1;
    c->stereo_done = c->rds_dsp_done = c->rds_bits_done = c->mono_done = -1;
    c->st_pre_done = c->st_pll_done = c->rds_pre_done = c->rds_pll_done = -1;
    (void)in;
    return SDR_OK;
}

inline hipStream_t S(void* s) { return static_cast<hipStream_t>(s); }

}  // namespace

namespace {
PllJob stereo_job(sdr_ctx* c) {   // stereo.cpp:77: fmpll(pilot, 19e3, rf_Fs/rf_decim, ..., 2.0, 0, 0.01)
    const sdr_info& in = c->info;
    return PllJob{c->plain(c->pilot), c->plain_stride, c->plain(c->t_st), c->plain_stride, c->pllbuf(c->carrier),
                  c->pll_stride, c->st_pll, 19e3f, (float)(in.rf_Fs / in.rf_decim), 0.01f, 2.0f, 0.0f,
                  c->carrier + (c->parity ^ 1) * c->pll_par, c->rxbuf(c->rx_st), c->plain_stride,
                  c->plain(c->pilot_neg), c->plain_stride};
}
PllJob rds_job(sdr_ctx* c) {      // rds.cpp:119: fmpll(gen_pilot, 114e3, if_Fs, ..., 0.5, 0, 0.001)
    const sdr_info& in = c->info;
    return PllJob{c->plain(c->gpilot), c->plain_stride, c->plain(c->t_rds), c->plain_stride, c->pllbuf(c->ipll),
                  c->pll_stride, c->rds_pll, 114e3f, (float)in.if_Fs, 0.001f, 0.5f, 0.0f,
                  c->ipll + (c->parity ^ 1) * c->pll_par, c->rxbuf(c->rx_rds), c->plain_stride,
                  c->plain(c->gpilot_neg), c->plain_stride};
}

}  // namespace

namespace {
// Scratch of the context-free PLL primitive (input reciprocals [nch][ts] f64 + phases [nch][ts]
// f32): one buffer per (device, stream), reused in that stream's order and grown on demand, so
// sdr_fmpll enqueues without synchronising (the round-2 diagnosis of the pool-allocated variants
// that this replaced: DESIGN.md 7, profiles/r02/diag_fmpll_scratch.txt).
struct StreamScratch {
    hipStream_t s;
    int dev;
    void* p;
    size_t bytes;
};
std::mutex g_scratch_mu;
std::vector<StreamScratch> g_scratch;

// caller holds g_scratch_mu until its kernels using the buffer are enqueued, so that another
// host thread on the same stream cannot grow (free) the buffer in between
int stream_scratch(hipStream_t s, size_t bytes, void** out) {
    int dev = 0;
    HIP_TRY(hipGetDevice(&dev));
    for (auto& e : g_scratch) {
        if (e.s != s || e.dev != dev) continue;
        if (e.bytes < bytes) {   // grow: work already queued on s may still read the old buffer
            HIP_TRY(hipStreamSynchronize(s));
            HIP_TRY(hipFree(e.p));
            e.p = nullptr;
            HIP_TRY(hipMalloc(&e.p, bytes));
            e.bytes = bytes;
        }
        *out = e.p;
        return SDR_OK;
    }
    void* p = nullptr;
    HIP_TRY(hipMalloc(&p, bytes));
    g_scratch.push_back({s, dev, p, bytes});
    *out = p;
    return SDR_OK;
}

// forget (and free) the scratch of a stream about to be destroyed
int release_stream_scratch(hipStream_t s) {
    std::lock_guard<std::mutex> lk(g_scratch_mu);
    for (size_t i = 0; i < g_scratch.size(); i++) {
        if (g_scratch[i].s != s) continue;
        HIP_TRY(hipStreamSynchronize(s));
        HIP_TRY(hipFree(g_scratch[i].p));
        g_scratch.erase(g_scratch.begin() + (long)i);
        return SDR_OK;
    }
    return SDR_OK;
}

// Streams made by sdr_stream_create_cu_range, with their device, CU mask and placement. The
// persistent PLL launch accepts only these: each has its own hardware queue (a pool stream can share
// one with the stream that signals the blocks, which then never runs), and its mask's placement
// bounds how many of the launch's workgroups can be resident at once (sdr_internal.h CuPlacement).
struct MaskedStream {
    hipStream_t s;
    int device;
    CuPlacement place;
};
std::mutex g_masked_mu;
std::vector<MaskedStream> g_masked;

bool masked_stream(hipStream_t s, int* device, CuPlacement* place) {
    std::lock_guard<std::mutex> lk(g_masked_mu);
    for (const MaskedStream& m : g_masked)
        if (m.s == s && s != nullptr) {
            *device = m.device;
            if (place) *place = m.place;
            return true;
        }
    return false;
}

// the mask of CUs [first_cu, first_cu + n_cu) of a device (or of every other CU: exclude)
std::vector<uint32_t> cu_range_mask(int ncu, int first_cu, int n_cu, int exclude, int* nset) {
    std::vector<uint32_t> mask((ncu + 31) / 32, 0u);
    *nset = 0;
    for (int cu = 0; cu < ncu; ++cu) {
        const bool in = cu >= first_cu && cu < first_cu + n_cu;
        if (in != (exclude != 0)) {
            mask[cu / 32] |= 1u << (cu % 32);
            ++*nset;
        }
    }
    return mask;
}

int device_xccs(int device) {
    int nx = 0;
    if (hipDeviceGetAttribute(&nx, hipDeviceAttributeNumberOfXccs, device) != hipSuccess || nx <= 0) nx = 8;
    return nx;
}

}  // namespace

CuPlacement sdrk::cu_placement(const uint32_t* mask, int nwords, int ncu_dev, int nxcc) {
    constexpr int SE_PER_XCC = 4;   // MI355X: 32 shader engines over 8 XCCs
    CuPlacement pl;
    if (nxcc <= 0 || ncu_dev % nxcc) nxcc = 1;
    const int slots = ncu_dev / nxcc;
    int min_units = -1;
    for (int x = 0; x < nxcc; x++) {
        int per_se[SE_PER_XCC] = {};
        int nx = 0;
        for (int j = 0; j < slots; j++) {
            const int bit = j * nxcc + x;
            if (bit / 32 < nwords && (mask[bit / 32] >> (bit % 32) & 1u)) {
                per_se[j % SE_PER_XCC]++;
                nx++;
            }
        }
        pl.ncu += nx;
        if (!nx) continue;
        pl.xcc_active++;
        int active = 0, lo = slots;
        for (int k = 0; k < SE_PER_XCC; k++)
            if (per_se[k]) {
                active++;
                lo = std::min(lo, per_se[k]);
            }
        const int units = active * lo;
        min_units = min_units < 0 ? units : std::min(min_units, units);
    }
    pl.min_units = std::max(min_units, 0);
    return pl;
}

namespace {
}  // namespace

extern "C" {

const char* sdr_last_error(void) { return sdrk::last_error(); }
int sdr_version(void) { return 1; }

int sdr_stream_create_cu_range(void** stream, int device, int first_cu, int n_cu, int exclude) {
    if (!stream) return fail(SDR_E_INVALID, "sdr_stream_create_cu_range: stream is NULL");
    int cur = 0;
    HIP_TRY(hipGetDevice(&cur));
    struct Restore {   // the caller's current device is left as it was
        int d;
        ~Restore() { (void)hipSetDevice(d); }
    } restore{cur};
    HIP_TRY(hipSetDevice(device));
    hipDeviceProp_t prop;
    HIP_TRY(hipGetDeviceProperties(&prop, device));
    const int ncu = prop.multiProcessorCount;
    if (first_cu < 0 || n_cu <= 0 || first_cu + n_cu > ncu || (exclude && n_cu >= ncu))
        return fail(SDR_E_INVALID, "sdr_stream_create_cu_range: CUs [%d, %d) outside [0, %d)",
                    first_cu, first_cu + n_cu, ncu);
    int nset = 0;
    std::vector<uint32_t> mask = cu_range_mask(ncu, first_cu, n_cu, exclude, &nset);
    hipStream_t s = nullptr;
    HIP_TRY(hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()));
    {
        std::lock_guard<std::mutex> lk(g_masked_mu);
        g_masked.push_back(MaskedStream{s, device, cu_placement(mask.data(), (int)mask.size(), ncu, device_xccs(device))});
    }
    *stream = s;
    return SDR_OK;
}

int sdr_stream_destroy(void* stream) {
    if (!stream) return fail(SDR_E_INVALID, "sdr_stream_destroy: stream is NULL");
    const int rc = release_stream_scratch((hipStream_t)stream);
    if (rc != SDR_OK) return rc;
    {
        std::lock_guard<std::mutex> lk(g_masked_mu);
        for (size_t i = 0; i < g_masked.size(); i++)
            if (g_masked[i].s == (hipStream_t)stream) {
                g_masked.erase(g_masked.begin() + (long)i);
                break;
            }
    }
    HIP_TRY(hipStreamDestroy((hipStream_t)stream));
    return SDR_OK;
}

int sdr_hbm_copy(void* dst, const void* src, size_t bytes, void* stream) {
    if (!dst || !src || (bytes & 15) || (reinterpret_cast<uintptr_t>(dst) & 15) || (reinterpret_cast<uintptr_t>(src) & 15))
        return fail(SDR_E_INVALID, "sdr_hbm_copy: pointers and size must be 16-byte aligned");
    if (bytes == 0) return SDR_OK;
    const size_t n = bytes / 16;
    if ((n + 255) / 256 > 0x7FFFFFFFu) return fail(SDR_E_INVALID, "sdr_hbm_copy: %zu bytes is too large", bytes);
    const int grid = (int)((n + 255) / 256);
    hipLaunchKernelGGL(k_hbm_copy, dim3(grid), dim3(256), 0, S(stream), static_cast<u32x4*>(dst),
                       static_cast<const u32x4*>(src), n);
    HIP_TRY(hipGetLastError());
    return SDR_OK;
}

// Test support (not part of sdr_amd.h): hold `stream` for `ms` milliseconds (at most 10 s) with one
// sleeping wave, so that a test can keep a reader stream from releasing its block (the bounded
// release wait's timeout, tests/test_gpu_pipeline.py).
__global__ void k_hold(unsigned long long ticks) {
    if (threadIdx.x != 0) return;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(127);
}
extern "C" int sdr_diag_hold(void* stream, int ms) {
    if (ms < 0 || ms > 10000) return fail(SDR_E_INVALID, "sdr_diag_hold: %d ms outside [0, 10000]", ms);
    hipLaunchKernelGGL(k_hold, dim3(1), dim3(64), 0, S(stream), (unsigned long long)ms * 100000ull);
    HIP_TRY(hipGetLastError());
    return SDR_OK;
}

// Test support (not part of sdr_amd.h): res[i] = 1 - x[i] * v_rcp_f64(x[i]) (one fma, exact), the
// hardware reciprocal's relative error that the exact front end's discriminator proof assumes
// below 2^-22 (sdr_frontend.hip, SDR_FE_DISC; tests/test_gpu_primitives.py).
__global__ void k_rcp64_residual(const double* __restrict__ x, double* __restrict__ res, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) res[i] = __builtin_fma(-x[i], __builtin_amdgcn_rcp(x[i]), 1.0);
}
extern "C" int sdr_diag_rcp64_residual(const double* x, double* res, int n, void* stream) {
    if (!x || !res || n <= 0) return fail(SDR_E_INVALID, "sdr_diag_rcp64_residual: bad arguments");
    hipLaunchKernelGGL(k_rcp64_residual, dim3((n + 255) / 256), dim3(256), 0, S(stream), x, res, n);
    HIP_TRY(hipGetLastError());
    return SDR_OK;
}

// Diagnosis builds only (-DSDR_PLL_COUNT=1): the PLL chunk counters; -1 in product builds.
// Not part of sdr_amd.h.
extern "C" int sdr_diag_pll_counts(unsigned long long* out, int reset) { return diag_pll_counts(out, reset); }
// Diagnosis builds only (-DSDR_PLL_WAVES=1): per-wave totals of the last persistent launch; -1 otherwise.
extern "C" int sdr_diag_pll_waves(unsigned long long* out, int nmax) { return diag_pll_waves(out, nmax); }
// Diagnosis builds only (-DSDR_PLL_HWID=1): placement and duration of the last k_pll launch's waves.
extern "C" int sdr_diag_pll_hwid(unsigned long long* out, int nmax) { return diag_pll_hwid(out, nmax); }

int sdr_ctx_create(sdr_ctx** out, int device, int nch, int mode, int rds_on, int flags) {
    if (!out || nch <= 0) return fail(SDR_E_INVALID, "bad arguments");
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= device || device < 0)
        return fail(SDR_E_NODEV, "no HIP device %d", device);
    HIP_TRY(hipSetDevice(device));
    sdr_ctx* c = new sdr_ctx();
    c->device = device;
    c->nch = nch;
    c->mode = mode;
    c->rds_on = rds_on ? 1 : 0;
    c->flags = flags;
    {
        int cus = 0;
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device);
        c->cus = cus;
    }
    int r = fill_info(&c->info, nch, mode, c->rds_on);
    if (r) { delete c; return r; }
    const sdr_info& in = c->info;
    const int T = in.rf_taps, U = in.audio_upsample;
    c->ntaps = T;
    // ---- taps (host design, reference formulas) ----
    std::vector<float> rf(T), audio((size_t)T * U), pilot(T), stereo(T), rds(T), rds_sq(T), rdsbb((size_t)T * 247),
        rrc(T);
    const float fb_pilot[2] = {18.5e3f, 19.5e3f}, fb_stereo[2] = {22e3f, 54e3f};
    const float fb_rds[2] = {54e3f, 60e3f}, fb_rds_sq[2] = {113.5e3f, 114.5e3f};
    sdr_impulse_response_lpf((float)in.rf_Fs, 100000.0f, (unsigned short)T, rf.data());                  // rffrontend.cpp:24
    sdr_impulse_response_lpf_gain((float)(in.if_Fs * U), 16000.0f, (unsigned short)(T * U), U, audio.data()); // mono.cpp:22
    sdr_impulse_response_bpf((float)(in.rf_Fs / in.rf_decim), fb_pilot, (unsigned short)T, pilot.data());  // stereo.cpp:65
    sdr_impulse_response_bpf((float)(in.rf_Fs / in.rf_decim), fb_stereo, (unsigned short)T, stereo.data()); // stereo.cpp:67
    sdr_impulse_response_lpf_gain((float)(in.if_Fs * 247), 3e3f, (unsigned short)(T * 247), 247, rdsbb.data()); // rds.cpp:61
    sdr_impulse_response_bpf((float)in.if_Fs, fb_rds, (unsigned short)T, rds.data());                      // rds.cpp:62
    sdr_impulse_response_bpf((float)in.if_Fs, fb_rds_sq, (unsigned short)T, rds_sq.data());                // rds.cpp:63
    sdr_impulse_response_rrc((float)(2375 * in.symbol_Fs), (unsigned short)T, rrc.data());                 // rds.cpp:65
    Polyphase pa = make_polyphase(audio, U), pr = make_polyphase(rdsbb, 247);
    c->audio_L = pa.L;
    c->rdsbb_L = pr.L;
#define TRY(x) do { int r_ = (x); if (r_) { sdr_ctx_destroy(c); return r_; } } while (0)
    TRY(upload(c, &c->rf_h, rf));
    {
        // exact front-end tap table: row S (input sample S of a thread window, R outputs) holds
        // h[r*D + 100 - S] / 128 (exact power-of-two scaling) or 0 where that tap does not exist;
        // 32 zero floats past the last row (whole 128-byte tap batches are loaded)
        const int R = frontend_tab_r(), D = in.rf_decim, TWIN = (R - 1) * D + T;
        std::vector<float> tt((size_t)TWIN * R + 32, 0.0f);
        for (int S_ = 0; S_ < TWIN; S_++)
            for (int r = 0; r < R; r++) {
                const int k = r * D + (T - 1) - S_;
                if (k >= 0 && k < T) tt[(size_t)S_ * R + r] = rf[k] * 0.0078125f;
            }
        TRY(upload(c, &c->rf_hs, tt));
    }
    if (T == 101 && (in.rf_decim == 10 || in.rf_decim == 4 || in.rf_decim == 3)) {
        // MFMA front end: taps as fixed point h*2^F in FT_ND balanced base-256 digits, laid out as
        // the A fragments of v_mfma_i32_16x16x64_i8: fragment f = FT_ND*kstep + digit, lane l holds
        // A[row l&15][k = 64*kstep + 16*(l>>4) + jj], A[i][k] = digit(h[D*i + 100 - k])
        const int D = in.rf_decim;
        double hmax = 0.0;
        for (float v : rf) hmax = std::max(hmax, (double)std::fabs(v));
        const int F = 8 * FT_ND - 2 - (int)std::ceil(std::log2(hmax));   // |h * 2^F| < 2^(8*ND - 2)
        std::vector<int8_t> dig((size_t)T * FT_ND);
        for (int k = 0; k < T; k++) {
            long long q = std::llround((double)rf[k] * std::ldexp(1.0, F));
            for (int p = FT_ND - 1; p >= 0; p--) {               // least significant digit first
                int d = (int)(((q % 256) + 256) % 256);
                if (d >= 128) d -= 256;
                dig[(size_t)k * FT_ND + p] = (int8_t)d;
                q = (q - d) / 256;
            }
        }
        std::vector<int8_t> fr((size_t)FT_AFRAGS * 64 * 16, 0);
        for (int ks = 0; ks < 4; ks++)
            for (int p = 0; p < FT_ND; p++)
                for (int l = 0; l < 64; l++)
                    for (int jj = 0; jj < 16; jj++) {
                        const int i = l & 15, k = 64 * ks + 16 * (l >> 4) + jj, tap = D * i + 100 - k;
                        if (tap >= 0 && tap < T)
                            fr[(((size_t)(FT_ND * ks + p) * 64) + l) * 16 + jj] = dig[(size_t)tap * FT_ND + p];
                    }
        int8_t* dfr = nullptr;
        TRY(upload(c, &dfr, fr));
        c->fe_afrag = dfr;
        c->fe_yscale = std::ldexp(1.0, -(F + 7));
    }
    TRY(upload(c, &c->pilot_h, pilot));
    TRY(upload(c, &c->stereo_h, stereo));
    {
        // {pilot[k], band[k]} interleaved for the 3-filter pass's packed pairs, 104 pairs (chunks of 4)
        std::vector<float> h01(2 * 104, 0.0f);
        for (int k = 0; k < T && k < 104; k++) { h01[2 * k] = pilot[k]; h01[2 * k + 1] = stereo[k]; }
        TRY(upload(c, &c->pilot_band_h, h01));
    }
    TRY(upload(c, &c->rds_h, rds));
    TRY(upload(c, &c->rds_sq_h, rds_sq));
    TRY(upload(c, &c->rrc_h, rrc));
    TRY(upload(c, &c->audio_pp, pa.table));
    TRY(upload(c, &c->audio_cnt, pa.cnt));
    TRY(upload(c, &c->rdsbb_pp, pr.table));
    TRY(upload(c, &c->rdsbb_cnt, pr.cnt));
    c->rdsbb_all101 = std::all_of(pr.cnt.begin(), pr.cnt.end(), [](int k) { return k == 101; });
    c->audio_u1_101 = in.audio_upsample == 1 && pa.cnt.size() == 1 && pa.cnt[0] == 101;
    // ---- extended streams ----
    c->fm_stride = round_up((size_t)HIST + in.block_if, 64);
    c->rf_stride = round_up((size_t)HIST + in.n_rds, 64);
    c->fm_par = c->fm_stride * nch;
    c->rf_par = c->rf_stride * nch;
    float* base = nullptr;
    TRY(dalloc(c, &base, 2 * c->fm_par)); c->fm = base + HIST;
    TRY(dalloc(c, &base, 2 * c->fm_par)); c->sdc = base + HIST;
    TRY(dalloc(c, &base, 2 * c->fm_par)); c->rband = base + HIST;
    TRY(dalloc(c, &base, 2 * c->fm_par)); c->rdc = base + HIST;
    TRY(dalloc(c, &base, 2 * c->rf_par)); c->rfilt = base + HIST;
    c->plain_stride = round_up((size_t)in.block_if, 64);
    c->pll_stride = round_up((size_t)in.block_if + 1, 64);
    c->clean_stride = round_up((size_t)in.n_rds, 64);
    c->plain_par = c->plain_stride * nch;
    c->pll_par = c->pll_stride * nch;
    TRY(dalloc(c, &c->pilot, 2 * c->plain_par));
    TRY(dalloc(c, &c->band, 2 * c->plain_par));
    TRY(dalloc(c, &c->gpilot, 2 * c->plain_par));
    TRY(dalloc(c, &c->pilot_neg, 2 * c->plain_par));
    TRY(dalloc(c, &c->gpilot_neg, 2 * c->plain_par));
    TRY(dalloc(c, &c->t_st, 2 * c->plain_par));
    TRY(dalloc(c, &c->t_rds, 2 * c->plain_par));
    {
        std::vector<int> ptq(std::max(in.n_rds, 1));
        for (int k = 0; k < in.n_rds; k++) {                // rds.cpp:130: U = 247, D = 640
            const long long nd = (long long)k * 640;
            ptq[k] = (int)((nd / 247) << 8) | (int)(nd % 247);
        }
        TRY(upload(c, &c->rds_ptq, ptq));
    }
    TRY(dalloc(c, &c->rx_st, 2 * c->plain_par));
    TRY(dalloc(c, &c->rx_rds, 2 * c->plain_par));
    TRY(dalloc(c, &c->carrier, 2 * c->pll_par));
    TRY(dalloc(c, &c->ipll, 2 * c->pll_par));
    TRY(dalloc(c, &c->rds_clean, c->clean_stride * nch));
    TRY(dalloc(c, &c->tail, (size_t)2 * nch * 2 * (T - 1)));
    {
        std::vector<uint32_t> pad(64, 0x80808080u);
        TRY(upload(c, &c->pad80, pad));
    }
    TRY(dalloc(c, &c->prev, (size_t)2 * nch));
    TRY(dalloc(c, &c->st_pll, (size_t)nch));
    TRY(dalloc(c, &c->rds_pll, (size_t)nch));
    TRY(dalloc(c, &c->dec, (size_t)nch * DEC_STATE));
    TRY(dalloc(c, &c->rel_words, (size_t)2 * sdr_ctx::REL_SLOTS));
    TRY(dalloc(c, &c->fail_words, (size_t)2));
    {
        // the release timeout's host-visible mirror: one coherent host word the device sets only on
        // the failure path, so that every stage call can check it without a synchronisation
        void* hp = nullptr;
        if (hipHostMalloc(&hp, 64, hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess || !hp)
            TRY(fail(SDR_E_NOMEM, "hipHostMalloc of the context's fail word"));
        c->fail_host = static_cast<uint32_t*>(hp);
        *c->fail_host = 0u;
        void* dp = nullptr;
        if (hipHostGetDevicePointer(&dp, hp, 0) != hipSuccess || !dp)
            TRY(fail(SDR_E_HIP, "hipHostGetDevicePointer of the context's fail word"));
        c->fail_host_dev = static_cast<uint32_t*>(dp);
    }
    TRY(init_state(c, nullptr));
#undef TRY
    *out = c;
    return SDR_OK;
}

int sdr_ctx_destroy(sdr_ctx* c) {
    if (!c) return SDR_OK;
    (void)hipSetDevice(c->device);
    for (void* p : c->allocs) (void)hipFree(p);
    if (c->fail_host) (void)hipHostFree(c->fail_host);
    if (c->pers_ev) (void)hipEventDestroy(c->pers_ev);
    for (hipEvent_t e : c->fe_ev) (void)hipEventDestroy(e);
    if (c->fe_stamps) (void)hipFree(c->fe_stamps);
    for (hipEvent_t e : c->pers_reader_ev)
        if (e) (void)hipEventDestroy(e);
    delete c;
    return SDR_OK;
}

int sdr_ctx_reset(sdr_ctx* c, void* stream) {
    if (!c) return fail(SDR_E_INVALID, "null context");
    HIP_TRY(hipSetDevice(c->device));
    c->pers_failed = false;   // a timed-out launch's poisoned state is what the reset replaces
    // no block of the reset context belongs to the last launch any more (its error word stays set
    // until the next launch's prepare: a block with the old index must not read it)
    c->pers_block = -1;
    c->pers_nreaders = 0;     // (the caller has drained its streams: nothing left to order after)
    // the release words back in step with the host's counts (a reader that never ran would leave its
    // slot short, and every later wait on it would expire again), then the release timeout cleared:
    // callers reset once the streams that ran the context's stages have drained
    hipStream_t s = S(stream);
    HIP_TRY(hipMemcpyAsync(c->rel_words, c->rel_seq, sizeof(c->rel_seq), hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemsetAsync(c->fail_words, 0, 2 * sizeof(uint32_t), s));
    const int r = init_state(c, s);   // (synchronises s)
    __atomic_store_n(c->fail_host, 0u, __ATOMIC_SEQ_CST);
    return r;
}

int sdr_ctx_info(const sdr_ctx* c, sdr_info* info) {
    if (!c || !info) return fail(SDR_E_INVALID, "null argument");
    *info = c->info;
    return SDR_OK;
}

extern "C++" {
namespace {
// the front end's arguments for the block that switches the context to parity p
FrontendArgs frontend_args(const sdr_ctx* c, const uint8_t* iq, size_t iq_stride, int p) {
    const sdr_info& in = c->info;
    const int hp = c->ntaps - 1;
    FrontendArgs a{};
    a.iq = iq;
    a.iq_stride = iq_stride;
    a.tail_in = c->tail + (size_t)(p ^ 1) * c->nch * 2 * hp;
    a.tail_out = c->tail + (size_t)p * c->nch * 2 * hp;
    a.prev_in = c->prev + (size_t)(p ^ 1) * c->nch;
    a.prev_out = c->prev + (size_t)p * c->nch;
    a.fm = c->fm + p * c->fm_par;
    a.fm_other = c->fm + (p ^ 1) * c->fm_par;
    a.fm_stride = c->fm_stride;
    a.nch = c->nch;
    a.ntaps = c->ntaps;
    a.block_iq = in.block_iq;
    a.block_if = in.block_if;
    a.D = in.rf_decim;
    a.h = c->rf_h;
    a.hs = c->rf_hs;
    a.afrag = c->fe_afrag;
    a.yscale = c->fe_yscale;
    a.pad80 = c->pad80;
    a.fast = (c->flags & SDR_FLAG_FAST_FRONTEND) != 0 && c->fe_afrag != nullptr;
    return a;
}
// Parity release across streams (threadsafequeue.h:29-31: a producer reuses a buffer only after its
// consumers released it). The block of parity p is read by the mono stage, the stereo post stage and
// the RDS mixer; each stores the count of blocks of that parity it has read into a device word on its
// stream after its kernels that read them (k_flag_store, ordered after them), and the stages that
// overwrite parity p two blocks later wait on their stream for the count the host last enqueued
// (k_flag_wait) -- unless that reader ran on the same stream, whose order already holds. Slots:
// REL_MONO (fm), REL_STEREO (fm, band, t_st, carrier), REL_RDS (rband, t_rds, ipll). Device words,
// not HIP events: a cross-stream event wait between the CU-masked streams started the waiting
// stream 60-200 us after the event's work had completed (profiles/r04/release/), a kernel poll
// within a few us.
constexpr unsigned REL_MONO = 1u, REL_STEREO = 2u, REL_RDS = 4u;
int release_record(sdr_ctx* c, unsigned slot, hipStream_t s) {
    const int p = c->parity, k = slot == REL_MONO ? 0 : slot == REL_STEREO ? 1 : 2;
    c->rel_seq[p][k]++;
    c->rel_stream[p][k] = s;
    return launch_flag_store(c->rel_words + p * sdr_ctx::REL_SLOTS + k, c->rel_seq[p][k], s);
}
int release_wait(sdr_ctx* c, int p, unsigned slots, hipStream_t s) {
    unsigned mask = 0;
    for (int k = 0; k < sdr_ctx::REL_SLOTS; k++) {
        const uint32_t want = c->rel_seq[p][k];
        if (!(slots & (1u << k)) || want == 0 || c->rel_stream[p][k] == s ||
            (c->rel_waited_on[p][k] == s && c->rel_waited[p][k] == want))
            continue;
        mask |= 1u << k;
        c->rel_waited[p][k] = want;
        c->rel_waited_on[p][k] = s;
    }
    if (!mask) return SDR_OK;
    hipLaunchKernelGGL(k_rel_wait, dim3(1), dim3(64), 0, s, c->rel_words + p * sdr_ctx::REL_SLOTS, c->rel_seq[p][0],
                       c->rel_seq[p][1], c->rel_seq[p][2], mask, c->fail_words, c->fail_host_dev);
    LAUNCH_CHECK();
    return SDR_OK;
}
// a parity-release wait of this context gave up (k_rel_wait set the host-mapped fail word): every
// stage call fails until sdr_ctx_reset (the device poisons the outputs of the stages already queued)
int check_failed(const sdr_ctx* c, const char* what) {
    if (c->fail_host && __atomic_load_n(c->fail_host, __ATOMIC_ACQUIRE) != 0u)
        return fail(SDR_E_TIMEOUT, "%s: a parity-release wait timed out (a reader did not release its block within "
                                   "5 s, and the producer overwrote it): outputs since are poisoned; sdr_ctx_reset",
                    what);
    return SDR_OK;
}
// the error words of the current block's output stages (kernel side: Poison)
Poison block_poison(const sdr_ctx* c) { return Poison{c->pers_err(), c->fail_words}; }
// After a stage that read the persistent launch's error word was enqueued on `s`: record that
// stream's reader event now, so the next launch's prepare can order its reset of the word after
// every reader by waiting on the events alone -- no stream handle is used after the call that
// supplied it (the handle only names the event's slot; a stream destroyed since is never touched).
// More than PERS_READERS streams fall back to a device synchronisation in the prepare.
int pers_reader_mark(sdr_ctx* c, hipStream_t s) {
    if (!c->pers_err()) return SDR_OK;
    int slot = -1;
    for (int i = 0; i < c->pers_nreaders && i < sdr_ctx::PERS_READERS; i++)
        if (c->pers_readers[i] == s) slot = i;
    if (slot < 0) {
        if (c->pers_nreaders >= sdr_ctx::PERS_READERS) {
            c->pers_nreaders = sdr_ctx::PERS_READERS + 1;
            return SDR_OK;
        }
        slot = c->pers_nreaders++;
        c->pers_readers[slot] = s;
    }
    if (!c->pers_reader_ev[slot]) HIP_TRY(hipEventCreateWithFlags(&c->pers_reader_ev[slot], hipEventDisableTiming));
    HIP_TRY(hipEventRecord(c->pers_reader_ev[slot], s));
    return SDR_OK;
}
int check_iq(const sdr_ctx* c, const uint8_t* iq, size_t iq_stride) {
    const sdr_info& in = c->info;
    if (iq_stride < (size_t)2 * in.block_iq || (iq_stride & 1) || (reinterpret_cast<uintptr_t>(iq) & 1))
        return fail(SDR_E_INVALID, "iq_stride %zu < 2*block_iq %d or misaligned", iq_stride, 2 * in.block_iq);
    return SDR_OK;
}
}  // namespace
}  // extern "C++"

int sdr_frontend(sdr_ctx* c, const uint8_t* iq, size_t iq_stride, void* stream) {
    if (!c || !iq) return fail(SDR_E_INVALID, "null argument");
    if (const int rf_ = check_failed(c, "frontend")) return rf_;
    if (const int r = check_iq(c, iq, iq_stride)) return r;
    const int p = c->parity ^ 1;
    // fm of parity p, and the pre stages' buffers too (one wait kernel: sdr_pre on this stream then
    // has nothing left to wait for; waiting for the RDS mixer only before the pre stages measured the
    // same, profiles/r04/release/)
    if (const int rw = release_wait(c, p, REL_MONO | REL_STEREO | REL_RDS, S(stream))) return rw;
    FrontendArgs a = frontend_args(c, iq, iq_stride, p);
    const bool timed = c->fe_time_n < c->fe_time_cap;
    if (timed && c->fe_use_stamps) {   // sdr_frontend_timing: the kernel's own workgroup stamps
        a.stamps = c->fe_stamps + (size_t)c->fe_time_n * c->fe_stamp_wgs * 2;
    } else if (timed) {                // (other front ends) HIP events recorded with the launch
        a.ev0 = c->fe_ev[2 * c->fe_time_n];
        a.ev1 = c->fe_ev[2 * c->fe_time_n + 1];
    }
    const int r = frontend_launch(a, S(stream));
    if (r) return r;
    if (timed) c->fe_time_n++;
    c->parity = p;
    c->block++;
    return SDR_OK;
}

int sdr_frontend_timing(sdr_ctx* c, int max_launches) {
    if (!c || max_launches < 0) return fail(SDR_E_INVALID, "frontend_timing: bad arguments");
    HIP_TRY(hipSetDevice(c->device));
    const sdr_info& in = c->info;
    const int wgs = frontend_stamp_wgs(in.block_if, c->nch, c->ntaps, in.rf_decim, c->flags & SDR_FLAG_FAST_FRONTEND);
    c->fe_use_stamps = wgs > 0;
    if (c->fe_use_stamps) {
        if (c->fe_stamp_cap < max_launches || c->fe_stamp_wgs != wgs) {
            if (c->fe_stamps) {
                HIP_TRY(hipDeviceSynchronize());   // a pending timed launch may still write the old buffer
                HIP_TRY(hipFree(c->fe_stamps));
                c->fe_stamps = nullptr;
            }
            void* p = nullptr;
            HIP_TRY(hipMalloc(&p, (size_t)std::max(max_launches, 1) * wgs * 2 * sizeof(unsigned long long)));
            c->fe_stamps = static_cast<unsigned long long*>(p);
            c->fe_stamp_cap = max_launches;
            c->fe_stamp_wgs = wgs;
        }
    } else {
        while ((int)c->fe_ev.size() < 2 * max_launches) {
            hipEvent_t e = nullptr;
            HIP_TRY(hipEventCreate(&e));
            c->fe_ev.push_back(e);
        }
    }
    c->fe_time_cap = max_launches;
    c->fe_time_n = 0;
    return SDR_OK;
}

// the timed launches' earliest workgroup start and latest workgroup end (100 MHz ticks)
static int frontend_spans(sdr_ctx* c, int k, unsigned long long* t0, unsigned long long* t1) {
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipDeviceSynchronize());
    const size_t per = (size_t)c->fe_stamp_wgs * 2;
    std::vector<unsigned long long> h(per);
    for (int i = 0; i < k; i++) {
        HIP_TRY(hipMemcpy(h.data(), c->fe_stamps + (size_t)i * per, per * sizeof(unsigned long long),
                          hipMemcpyDeviceToHost));
        unsigned long long lo = ~0ull, hi = 0;
        for (size_t g = 0; g < per; g += 2) {
            lo = std::min(lo, h[g]);
            hi = std::max(hi, h[g + 1]);
        }
        t0[i] = lo;
        t1[i] = hi;
    }
    return SDR_OK;
}

int sdr_frontend_stamps(sdr_ctx* c, unsigned long long* t_start, unsigned long long* t_end, int max, int* n) {
    if (!c || !t_start || !t_end || max < 0) return fail(SDR_E_INVALID, "frontend_stamps: bad arguments");
    if (!c->fe_use_stamps) return fail(SDR_E_INVALID, "frontend_stamps: only the 101-tap front ends stamp themselves");
    const int k = std::min(c->fe_time_n, max);
    if (const int r = frontend_spans(c, k, t_start, t_end)) return r;
    if (n) *n = k;
    return SDR_OK;
}

int sdr_frontend_times(sdr_ctx* c, double* ms, int max, int* n) {
    if (!c || (!ms && max > 0)) return fail(SDR_E_INVALID, "frontend_times: bad arguments");
    const int k = std::min(c->fe_time_n, std::max(max, 0));
    if (c->fe_use_stamps) {
        // each launch: the earliest workgroup start to the latest workgroup end
        std::vector<unsigned long long> t0((size_t)std::max(k, 1)), t1((size_t)std::max(k, 1));
        if (const int r = frontend_spans(c, k, t0.data(), t1.data())) return r;
        for (int i = 0; i < k; i++) ms[i] = t1[i] >= t0[i] ? (double)(t1[i] - t0[i]) * 1e-5 : -1.0;
    } else {
        if (k > 0) HIP_TRY(hipEventSynchronize(c->fe_ev[2 * c->fe_time_n - 1]));
        for (int i = 0; i < k; i++) {
            float t = 0.0f;
            HIP_TRY(hipEventElapsedTime(&t, c->fe_ev[2 * i], c->fe_ev[2 * i + 1]));
            ms[i] = t;
        }
    }
    if (n) *n = k;
    return SDR_OK;
}

int sdr_frontend_release_wait(sdr_ctx* c, void* stream) {
    if (!c) return fail(SDR_E_INVALID, "null context");
    if (const int rf_ = check_failed(c, "frontend_release_wait")) return rf_;
    // the wait the next sdr_frontend (or sdr_frontend_pre_parts) enqueues first; it then finds the
    // counts already waited for on this stream and enqueues none
    return release_wait(c, c->parity ^ 1, REL_MONO | REL_STEREO | REL_RDS, S(stream));
}

int sdr_get_fm_demod(sdr_ctx* c, float* fm, size_t fm_stride, void* stream) {
    if (!c || !fm) return fail(SDR_E_INVALID, "null argument");
    if (const int rf_ = check_failed(c, "get_fm_demod")) return rf_;
    if (c->block < 0) return fail(SDR_E_INVALID, "no block processed yet");
    const sdr_info& in = c->info;
    return copy_rows(fm, fm_stride, c->fm_cur(), c->fm_stride, in.block_if, c->nch, nullptr, S(stream));
}

int sdr_mono(sdr_ctx* c, int16_t* audio, size_t audio_stride, void* stream) {
    if (!c || !audio) return fail(SDR_E_INVALID, "null argument");
    if (const int rf_ = check_failed(c, "mono")) return rf_;
    if (c->block < 0 || c->mono_done == c->block) return fail(SDR_E_INVALID, "mono: no new block");
    const sdr_info& in = c->info;
    const float* fm = c->fm_cur();
    if (c->audio_u1_101 && (in.audio_decim == 5 || in.audio_decim == 9)) {   // register-blocked, modes 0 and 1
        const dim3 g(cdiv(in.n_audio, ATILE), c->nch);
        if (in.audio_decim == 5)
            hipLaunchKernelGGL(k_mono_out<5>, g, dim3(AT), 0, S(stream), fm, c->fm_stride, c->audio_pp, in.block_if,
                               in.n_audio, audio, audio_stride, block_poison(c));
        else
            hipLaunchKernelGGL(k_mono_out<9>, g, dim3(AT), 0, S(stream), fm, c->fm_stride, c->audio_pp, in.block_if,
                               in.n_audio, audio, audio_stride, block_poison(c));
        LAUNCH_CHECK();
        c->mono_done = c->block;
        if (const int r = pers_reader_mark(c, S(stream))) return r;
        return release_record(c, REL_MONO, S(stream));
    }
    const int tile = 512;
    dim3 grid(cdiv(in.n_audio, tile), c->nch);
    const size_t lds = resample_lds_bytes(c->audio_L, in.audio_upsample, in.audio_decim, tile, 1);
    auto km = c->audio_u1_101 ? k_resample<1, 101> : k_resample<1, 0>;
    hipLaunchKernelGGL(km, grid, dim3(BLK), lds, S(stream), fm, fm, c->fm_stride, c->fm_stride,
                       nullptr, nullptr, (size_t)0, (size_t)0, c->audio_pp, c->audio_cnt, c->audio_L,
                       in.audio_upsample, in.audio_decim, in.n_audio, tile, -HIST, (void*)audio, audio_stride);
    LAUNCH_CHECK();
    hipLaunchKernelGGL(k_poison_i16, dim3(cdiv(in.n_audio, BLK), c->nch), dim3(BLK), 0, S(stream), block_poison(c),
                       audio, audio_stride, in.n_audio);
    LAUNCH_CHECK();
    c->mono_done = c->block;
    if (const int r = pers_reader_mark(c, S(stream))) return r;
    return release_record(c, REL_MONO, S(stream));
}

// The stereo and RDS loop bodies split at their PLL (pre: FIRs feeding the PLL; pll: the serial
// recurrence; post: everything after it), so a caller can run the PLL of block b on its own stream
// back to back with block b+1's while other streams do the rest. Intermediates that cross the
// split are kept per block parity. sdr_stereo / sdr_rds_dsp run the three parts on one stream.
extern "C++" {
namespace {
// launch k_fir_rb with NT tap sets (one block of every channel of length n)
// tiles [x0, x0 + xn) of the block (xn <= 0: all)
template <int NT, bool SQUARE>
int fir_rb(const sdr_ctx* c, const float* x, size_t x_stride, int n, FirRb f, hipStream_t s, int x0 = 0,
           int xn = 0) {
    if (xn <= 0) { x0 = 0; xn = cdiv(n, FRB_TILE); }
    f.x0 = x0;
    // the 2- and 3-set passes with their first two sets (pilot, band) as packed pairs
    if constexpr (NT >= 2 && !SQUARE) {
        if (f.h01) {
            hipLaunchKernelGGL((k_fir_rb<NT, false, true>), dim3(xn, c->nch), dim3(BLK), 0, s, x,
                               x_stride, x, x_stride, n, f);
            LAUNCH_CHECK();
            return SDR_OK;
        }
    }
    hipLaunchKernelGGL((k_fir_rb<NT, SQUARE>), dim3(xn, c->nch), dim3(BLK), 0, s, x, x_stride, x,
                       x_stride, n, f);
    LAUNCH_CHECK();
    return SDR_OK;
}
// pilot BPF (stereo.cpp:74) -> pilot + its PLL reciprocals, band BPF (:80) -> band
FirRb stereo_fir(sdr_ctx* c) {
    FirRb f{};
    f.h[0] = c->pilot_h;
    f.h[1] = c->stereo_h;
    f.y[0] = c->plain(c->pilot);
    f.y[1] = c->plain(c->band);
    f.y_stride[0] = f.y_stride[1] = c->plain_stride;
    f.rx0 = c->rxbuf(c->rx_st);
    f.rx_stride = c->plain_stride;
    f.y0neg = c->plain(c->pilot_neg);
    // (not as the packed pair of the 3-set pass: k_fir_rb<2, false, true> measured 133 against 120 us
    // for the scalar 2-set pass, profiles/r06/queue/)
    return f;
}
}  // namespace
}  // extern "C++"

int sdr_stereo_pre(sdr_ctx* c, void* stream) {
    if (!c) return fail(SDR_E_INVALID, "null context");
    if (const int rf_ = check_failed(c, "stereo_pre")) return rf_;
    if (c->block < 0 || c->st_pre_done == c->block) return fail(SDR_E_INVALID, "stereo_pre: no new block");
    if (c->ntaps != FRB_T) return fail(SDR_E_INVALID, "stereo_pre: %d taps", c->ntaps);
    // band of this parity read by the stereo post stage two blocks back
    if (const int rw = release_wait(c, c->parity, REL_STEREO, S(stream))) return rw;
    // pilot BPF (stereo.cpp:74) + band BPF (:80) from one staged window of fm_demod
    const int r = fir_rb<2, false>(c, c->fm_cur(), c->fm_stride, c->info.block_if, stereo_fir(c), S(stream));
    if (r) return r;
    c->st_pre_done = c->block;
    return SDR_OK;
}

int sdr_stereo_pll(sdr_ctx* c, void* stream) {
    if (!c) return fail(SDR_E_INVALID, "null context");
    if (const int rf_ = check_failed(c, "stereo_pll")) return rf_;
    if (c->st_pre_done != c->block || c->st_pll_done == c->block)
        return fail(SDR_E_INVALID, "stereo_pll: run sdr_stereo_pre on a new block first");
    PllJobs jobs{};
    jobs.j[0] = stereo_job(c);   // PLL 19 kHz -> 38 kHz carrier (stereo.cpp:77); NCO output: stereo_post
    const int r = launch_plls(c->flags & SDR_FLAG_PLL_LIBM, jobs, 1, c->info.block_if, c->nch, S(stream), false);
    if (r) return r;
    c->st_pll_done = c->block;
    return SDR_OK;
}

// a persistent launch the host already knows timed out (sdr_plls_report): its blocks' post stages
// fail (the device poisons their outputs anyway, for callers that have not asked yet)
static int check_pers_failed(const sdr_ctx* c, const char* what) {
    if (c->pers_failed && c->pers_err())
        return fail(SDR_E_HIP, "%s: the persistent PLL launch of this block timed out (outputs invalid): "
                               "sdr_ctx_reset, then a new sdr_plls_launch", what);
    return SDR_OK;
}

int sdr_stereo_post(sdr_ctx* c, int16_t* lr, size_t lr_stride, void* stream) {
    if (!c || !lr) return fail(SDR_E_INVALID, "null argument");
    if (const int rf_ = check_failed(c, "stereo_post")) return rf_;
    if (c->st_pll_done != c->block || c->stereo_done == c->block)
        return fail(SDR_E_INVALID, "stereo_post: run sdr_stereo_pll on a new block first");
    if (const int rf = check_pers_failed(c, "stereo_post")) return rf;
    const sdr_info& in = c->info;
    hipStream_t s = S(stream);
    const int n = in.block_if;
    const float* fm = c->fm_cur();
    if (!(c->flags & SDR_FLAG_KEEP_INTERMEDIATES) && c->audio_u1_101 &&
        (in.audio_decim == 5 || in.audio_decim == 9)) {
        // NCO, mixer, mono delay, both resamplers and L/R in one pass (k_stereo_out)
        const int p = c->parity;
        StereoOut a{};
        a.fm = fm;
        a.band = c->plain(c->band);
        a.t = c->plain(c->t_st);
        a.fm_stride = c->fm_stride;
        a.plain_stride = c->plain_stride;
        a.car = c->pllbuf(c->carrier);
        a.car_prev = c->carrier + (p ^ 1) * c->pll_par;
        a.car_stride = c->pll_stride;
        a.st = c->st_pll;
        a.ncoScale = 2.0f;                          // stereo.cpp:77: fmpll(..., 2.0, 0, 0.01)
        a.phaseAdjust = 0.0f;
        a.sdc = c->sdc + p * c->fm_par;
        a.sdc_prev = c->sdc + (p ^ 1) * c->fm_par;
        a.sdc_stride = c->fm_stride;
        a.h = c->audio_pp;
        a.n = n;
        a.ny = in.n_audio;
        a.lr = lr;
        a.lr_stride = lr_stride;
        a.err = block_poison(c);
        const dim3 g(cdiv(in.n_audio, ATILE), c->nch);
        if (in.audio_decim == 5)
            hipLaunchKernelGGL(k_stereo_out<5>, g, dim3(AT), 0, s, a);
        else
            hipLaunchKernelGGL(k_stereo_out<9>, g, dim3(AT), 0, s, a);
        LAUNCH_CHECK();
        c->stereo_done = c->block;
        if (const int r = pers_reader_mark(c, s)) return r;
        return release_record(c, REL_STEREO, s);
    }
    {
        // NCO output of this block's PLL phases (pll.cpp:52), carrier[0] = last of the previous block
        PllJobs jobs{};
        jobs.j[0] = stereo_job(c);
        const int r = launch_nco(jobs, 1, n, c->nch, s);
        if (r) return r;
    }
    // mixer (stereo.cpp:83-85) into the extended stereo_dc stream
    const int p = c->parity;
    float* sdc = c->sdc + p * c->fm_par;
    hipLaunchKernelGGL(k_mix<false>, dim3(cdiv(n, BLK), c->nch), dim3(BLK), 0, s, c->plain(c->band),
                       c->plain_stride, c->pllbuf(c->carrier), c->pll_stride, n, sdc, c->sdc + (p ^ 1) * c->fm_par,
                       c->fm_stride, 0);
    LAUNCH_CHECK();
    // mono delay (:88, exact 50-sample shift of fm_demod) + both resamplers + L/R (:94-107)
    const int tile = 512;
    dim3 gr(cdiv(in.n_audio, tile), c->nch);
    const size_t lds = resample_lds_bytes(c->audio_L, in.audio_upsample, in.audio_decim, tile, 2);
    auto ks = c->audio_u1_101 ? k_resample<2, 101> : k_resample<2, 0>;
    hipLaunchKernelGGL(ks, gr, dim3(BLK), lds, s, fm - 50, fm - 50, c->fm_stride, c->fm_stride, sdc, sdc,
                       c->fm_stride, c->fm_stride, c->audio_pp, c->audio_cnt, c->audio_L, in.audio_upsample,
                       in.audio_decim, in.n_audio, tile, -(HIST - 50), (void*)lr, lr_stride);
    LAUNCH_CHECK();
    hipLaunchKernelGGL(k_poison_i16, dim3(cdiv(2 * in.n_audio, BLK), c->nch), dim3(BLK), 0, s, block_poison(c), lr,
                       lr_stride, 2 * in.n_audio);
    LAUNCH_CHECK();
    c->stereo_done = c->block;
    if (const int r = pers_reader_mark(c, s)) return r;
    return release_record(c, REL_STEREO, s);
}

int sdr_stereo(sdr_ctx* c, int16_t* lr, size_t lr_stride, void* stream) {
    if (!c || !lr) return fail(SDR_E_INVALID, "null argument");
    if (c->block < 0 || c->stereo_done == c->block) return fail(SDR_E_INVALID, "stereo: no new block");
    int r = sdr_stereo_pre(c, stream);
    if (!r) r = sdr_stereo_pll(c, stream);
    if (!r) r = sdr_stereo_post(c, lr, lr_stride, stream);
    return r;
}

extern "C++" {
namespace {
// squaring (rds.cpp:111-113) + 114 kHz BPF (:116) of the extended rds_band stream -> gen_pilot + its
// PLL reciprocals
int rds_sq_fir(sdr_ctx* c, hipStream_t s, int x0 = 0, int xn = 0) {
    FirRb f{};
    f.h[0] = c->rds_sq_h;
    f.y[0] = c->plain(c->gpilot);
    f.y_stride[0] = c->plain_stride;
    f.rx0 = c->rxbuf(c->rx_rds);
    f.rx_stride = c->plain_stride;
    f.y0neg = c->plain(c->gpilot_neg);
    return fir_rb<1, true>(c, c->rband + c->parity * c->fm_par, c->fm_stride, c->info.block_if, f, s, x0, xn);
}
}  // namespace
}  // extern "C++"

int sdr_rds_pre(sdr_ctx* c, void* stream) {
    if (!c) return fail(SDR_E_INVALID, "null context");
    if (const int rf_ = check_failed(c, "rds_pre")) return rf_;
    if (c->block < 0 || c->rds_pre_done == c->block) return fail(SDR_E_INVALID, "rds_pre: no new block");
    if (c->ntaps != FRB_T) return fail(SDR_E_INVALID, "rds_pre: %d taps", c->ntaps);
    hipStream_t s = S(stream);
    const int n = c->info.block_if, p = c->parity;
    float* rband = c->rband + p * c->fm_par;
    if (const int rw = release_wait(c, p, REL_RDS, s)) return rw;   // rband read by the RDS mixer
    // RDS band BPF (rds.cpp:105) into the extended rds_band stream
    hipLaunchKernelGGL(k_hist_copy, dim3(c->nch), dim3(HIST), 0, s, rband, c->rband + (p ^ 1) * c->fm_par,
                       c->fm_stride, n);
    LAUNCH_CHECK();
    FirRb f{};
    f.h[0] = c->rds_h;
    f.y[0] = rband;
    f.y_stride[0] = c->fm_stride;
    int r = fir_rb<1, false>(c, c->fm_cur(), c->fm_stride, n, f, s);
    if (!r) r = rds_sq_fir(c, s);
    if (r) return r;
    c->rds_pre_done = c->block;
    return SDR_OK;
}

extern "C++" {
namespace {
// pilot, band and RDS band BPFs (stereo.cpp:74,80, rds.cpp:105) from one staged fm_demod window --
// the third output into the extended rds_band stream, history included -- then the squared 114 kHz
// BPF; FIR tiles [x0, x0 + xn) of the block (xn <= 0: all)
int pre_launch(sdr_ctx* c, hipStream_t s, int x0 = 0, int xn = 0) {
    const int n = c->info.block_if, p = c->parity;
    FirRb f = stereo_fir(c);
    f.h[2] = c->rds_h;
    f.h01 = c->pilot_band_h;
    f.y[2] = c->rband + p * c->fm_par;
    f.y_stride[2] = c->fm_stride;
    f.hist2_src = c->rband + (p ^ 1) * c->fm_par;
    const int r = fir_rb<3, false>(c, c->fm_cur(), c->fm_stride, n, f, s, x0, xn);
    return r ? r : rds_sq_fir(c, s, x0, xn);
}
}  // namespace
}  // extern "C++"

int sdr_pre(sdr_ctx* c, void* stream) {
    if (!c) return fail(SDR_E_INVALID, "null context");
    if (const int rf_ = check_failed(c, "pre")) return rf_;
    if (c->block < 0 || c->st_pre_done == c->block || c->rds_pre_done == c->block)
        return fail(SDR_E_INVALID, "pre: no new block");
    if (!c->rds_on) return sdr_stereo_pre(c, stream);
    if (c->ntaps != FRB_T) return fail(SDR_E_INVALID, "pre: %d taps", c->ntaps);
    if (const int rw = release_wait(c, c->parity, REL_STEREO | REL_RDS, S(stream))) return rw;
    const int r = pre_launch(c, S(stream));
    if (r) return r;
    c->st_pre_done = c->rds_pre_done = c->block;
    return SDR_OK;
}

int sdr_rds_pll(sdr_ctx* c, void* stream) {
    if (!c) return fail(SDR_E_INVALID, "null context");
    if (const int rf_ = check_failed(c, "rds_pll")) return rf_;
    if (c->rds_pre_done != c->block || c->rds_pll_done == c->block)
        return fail(SDR_E_INVALID, "rds_pll: run sdr_rds_pre on a new block first");
    PllJobs jobs{};
    jobs.j[0] = rds_job(c);      // PLL 114 kHz -> 57 kHz (rds.cpp:119); NCO output: rds_post
    const int r = launch_plls(c->flags & SDR_FLAG_PLL_LIBM, jobs, 1, c->info.block_if, c->nch, S(stream), false);
    if (r) return r;
    c->rds_pll_done = c->block;
    return SDR_OK;
}

int sdr_plls(sdr_ctx* c, void* stream) {
    if (!c) return fail(SDR_E_INVALID, "null context");
    if (const int rf_ = check_failed(c, "plls")) return rf_;
    if (c->st_pre_done != c->block || c->st_pll_done == c->block || c->rds_pre_done != c->block ||
        c->rds_pll_done == c->block)
        return fail(SDR_E_INVALID, "plls: run sdr_stereo_pre and sdr_rds_pre on a new block first");
    PllJobs jobs{};
    jobs.j[0] = stereo_job(c);
    jobs.j[1] = rds_job(c);
    const int r = launch_plls(c->flags & SDR_FLAG_PLL_LIBM, jobs, 2, c->info.block_if, c->nch, S(stream), false);
    if (r) return r;
    c->st_pll_done = c->rds_pll_done = c->block;
    return SDR_OK;
}

// the bookkeeping of a persistent launch: recover an abandoned previous launch, allocate the words
// and stamp arrays, reset this launch's stamps and error word (stream order on `stream`)
static int plls_prepare(sdr_ctx* c, int nblocks, hipStream_t s) {
    int dev_unused = 0;
    if (c->pers_signaled != c->pers_launched) {
        // blocks of the previous launch were never signalled: its waves give up on them after the
        // bounded wait (PLL_WAIT_TICKS) and still count them done. Let it drain, then resynchronise
        // the host's sequence numbers with the device words so this launch starts clean.
        HIP_TRY(hipStreamSynchronize(c->pers_stream));
        c->pers_signaled = c->pers_waited = c->pers_launched;
        HIP_TRY(hipMemcpyAsync(c->pers_words, &c->pers_launched, sizeof(uint32_t), hipMemcpyHostToDevice, s));
    } else if (c->pers_stream && c->pers_stream != s && c->pers_launched != 0 &&
               masked_stream(c->pers_stream, &dev_unused, nullptr)) {
        // every block of the previous launch is signalled, but its waves may still be stamping its
        // last blocks or setting its error word: the resets below wait for that launch in `s`'s order
        // (a PLL stream destroyed since has completed its work: hipStreamDestroy waits for it)
        if (!c->pers_ev) HIP_TRY(hipEventCreateWithFlags(&c->pers_ev, hipEventDisableTiming));
        HIP_TRY(hipEventRecord(c->pers_ev, c->pers_stream));
        HIP_TRY(hipStreamWaitEvent(s, c->pers_ev, 0));
    }
    if (!c->pers_words) {
        void* w = nullptr;
        HIP_TRY(hipMalloc(&w, PLL_WORDS * sizeof(uint32_t)));
        c->allocs.push_back(w);
        c->pers_words = static_cast<uint32_t*>(w);
        HIP_TRY(hipMemsetAsync(c->pers_words, 0, PLL_WORDS * sizeof(uint32_t), s));
    }
    if (c->pers_tcap < nblocks) {
        // timestamp arrays: allocated once with room for long phases (a later, longer launch
        // grows them here, outside any timed loop that reuses the capacity)
        const int cap = std::max(nblocks, 4096);
        if (c->pers_tcap > 0) HIP_TRY(hipStreamSynchronize(c->pers_stream));   // the last launch still writes them
        void *a = nullptr, *b = nullptr, *cy = nullptr;
        HIP_TRY(hipMalloc(&a, (size_t)cap * sizeof(unsigned long long)));
        c->allocs.push_back(a);
        HIP_TRY(hipMalloc(&b, (size_t)cap * sizeof(unsigned long long)));
        c->allocs.push_back(b);
        HIP_TRY(hipMalloc(&cy, (size_t)cap * 2 * sizeof(unsigned long long)));
        c->allocs.push_back(cy);
        c->pers_t0 = static_cast<unsigned long long*>(a);
        c->pers_t1 = static_cast<unsigned long long*>(b);
        c->pers_cyc = static_cast<unsigned long long*>(cy);
        c->pers_tcap = cap;
    }
    HIP_TRY(hipMemsetAsync(c->pers_t0, 0xFF, (size_t)nblocks * sizeof(unsigned long long), s));
    HIP_TRY(hipMemsetAsync(c->pers_t1, 0, (size_t)nblocks * sizeof(unsigned long long), s));
    HIP_TRY(hipMemsetAsync(c->pers_cyc, 0, (size_t)nblocks * 2 * sizeof(unsigned long long), s));
    // err of this launch: cleared after every post stream that read the previous launch's (their
    // queued stages would otherwise poison by a word that no longer says so, or read a clear word for a
    // block the old launch never computed)
    if (c->pers_nreaders > sdr_ctx::PERS_READERS) {
        HIP_TRY(hipDeviceSynchronize());
    } else {
        for (int i = 0; i < c->pers_nreaders; i++)   // recorded by the readers (pers_reader_mark)
            if (c->pers_reader_ev[i]) HIP_TRY(hipStreamWaitEvent(s, c->pers_reader_ev[i], 0));
    }
    c->pers_nreaders = 0;
    HIP_TRY(hipMemsetAsync(c->pers_words + 1, 0, sizeof(uint32_t), s));
    c->pers_prepared = nblocks;
    c->pers_prepared_launch = c->pers_launched;
    return SDR_OK;
}

int sdr_plls_prepare(sdr_ctx* c, int nblocks, void* stream) {
    if (!c || nblocks <= 0) return fail(SDR_E_INVALID, "plls_prepare: bad arguments");
    if (c->flags & SDR_FLAG_PLL_LIBM) return fail(SDR_E_INVALID, "plls_prepare: not with SDR_FLAG_PLL_LIBM");
    HIP_TRY(hipSetDevice(c->device));
    return plls_prepare(c, nblocks, S(stream));
}

// the persistent launch's jobs: the selected PLLs (SDR_PLLS_STEREO, SDR_PLLS_RDS; in that order in
// j[]) of the two parities, p[0] = the parity the next sdr_frontend switches to
static PllJobs2 plls_jobs(sdr_ctx* c, int which, int* njobs) {
    PllJobs2 jobs{};
    const int first_parity = c->parity ^ 1;
    for (int k = 0; k < 2; k++) {
        const int saved = c->parity;
        c->parity = first_parity ^ k;
        int q = 0;
        if (which & SDR_PLLS_STEREO) jobs.p[k].j[q++] = stereo_job(c);
        if (which & SDR_PLLS_RDS) jobs.p[k].j[q++] = rds_job(c);
        *njobs = q;
        c->parity = saved;
    }
    return jobs;
}

static int plls_which_ok(const sdr_ctx* c, int which, const char* what) {
    if (which != SDR_PLLS_STEREO && which != SDR_PLLS_RDS && which != SDR_PLLS_BOTH)
        return fail(SDR_E_INVALID, "%s: which = %d (SDR_PLLS_STEREO, SDR_PLLS_RDS or SDR_PLLS_BOTH)", what, which);
    if ((which & SDR_PLLS_RDS) && !c->rds_on) return fail(SDR_E_INVALID, "%s: the RDS PLL needs rds_on", what);
    return SDR_OK;
}

int sdr_plls_fits(sdr_ctx* c, int which, int first_cu, int n_cu, int* waves, long long* groups, long long* resident) {
    if (!c || !waves || !groups || !resident) return fail(SDR_E_INVALID, "plls_fits: bad arguments");
    if (const int r = plls_which_ok(c, which, "plls_fits")) return r;
    hipDeviceProp_t prop;
    HIP_TRY(hipGetDeviceProperties(&prop, c->device));
    const int ncu = prop.multiProcessorCount;
    if (first_cu < 0 || n_cu <= 0 || first_cu + n_cu > ncu)
        return fail(SDR_E_INVALID, "plls_fits: CUs [%d, %d) outside [0, %d)", first_cu, first_cu + n_cu, ncu);
    int nset = 0;
    const std::vector<uint32_t> mask = cu_range_mask(ncu, first_cu, n_cu, 0, &nset);
    const CuPlacement pl = cu_placement(mask.data(), (int)mask.size(), ncu, device_xccs(c->device));
    HIP_TRY(hipSetDevice(c->device));
    int njobs = 0;
    const PllJobs2 jobs = plls_jobs(c, which, &njobs);
    PllMultiPlan P;
    if (const int r = pll_multi_plan(jobs, njobs, c->info.block_if, c->nch, pl, &P)) return r;
    *waves = (int)P.waves;
    *groups = P.groups;
    *resident = P.resident;
    return SDR_OK;
}

int sdr_plls_launch(sdr_ctx* c, int nblocks, void* stream) { return sdr_plls_launch_sel(c, nblocks, SDR_PLLS_BOTH, stream); }

int sdr_plls_launch_sel(sdr_ctx* c, int nblocks, int which, void* stream) {
    if (!c || nblocks <= 0) return fail(SDR_E_INVALID, "plls_launch: bad arguments");
    if (const int rf_ = check_failed(c, "plls_launch")) return rf_;
    if (c->flags & SDR_FLAG_PLL_LIBM) return fail(SDR_E_INVALID, "plls_launch: not with SDR_FLAG_PLL_LIBM");
    if (const int r = plls_which_ok(c, which, "plls_launch")) return r;
    hipStream_t s = S(stream);
    // the launch's waves spin until later dispatches on other streams publish each block, so the
    // PLL stream must own its hardware queue (pool streams share GPU_MAX_HW_QUEUES queues with the
    // streams that signal) and every workgroup must be resident on the stream's CUs at once: refused
    // before anything is enqueued otherwise (a waiting launch could never finish, and its blocks would
    // time out)
    int sdev = -1;
    CuPlacement pl;
    if (!masked_stream(s, &sdev, &pl))
        return fail(SDR_E_INVALID, "plls_launch: the PLL stream was not made by sdr_stream_create_cu_range (a "
                                   "persistent launch needs a stream with its own hardware queue; use sdr_plls)");
    if (sdev != c->device)
        return fail(SDR_E_INVALID, "plls_launch: the PLL stream is on device %d, the context on %d", sdev, c->device);
    HIP_TRY(hipSetDevice(c->device));
    const int n = c->info.block_if, nch = c->nch;
    int njobs = 0;
    const PllJobs2 jobs = plls_jobs(c, which, &njobs);
    {
        PllMultiPlan P;
        if (const int r = pll_multi_plan(jobs, njobs, n, nch, pl, &P)) return r;
        if (P.groups > P.resident)
            return fail(SDR_E_INVALID, "plls_launch: %u waves do not fit the stream's %d CUs: %lld of %lld workgroups "
                        "of %d waves resident at once (%d per CU, %d XCCs x %d SE-balanced CU slots; use sdr_plls, "
                        "a stream over more CUs, or sdr_plls_fits to pick one)", P.waves, pl.ncu, P.resident,
                        P.groups, P.WG, P.per_cu, pl.xcc_active, pl.min_units);
    }
    // prepared ahead (sdr_plls_prepare, same nblocks, no launch since): only the launch is left
    if (!(c->pers_prepared == nblocks && c->pers_prepared_launch == c->pers_launched &&
          c->pers_signaled == c->pers_launched)) {
        const int r = plls_prepare(c, nblocks, s);
        if (r) return r;
    }
    c->pers_prepared = 0;
    uint32_t waves = 0;
    const int r = launch_pll_multi(jobs, njobs, n, nch, nblocks, c->pers_words, c->pers_launched, c->pers_t0,
                                   c->pers_t1, c->pers_cyc, &waves, s, pl, FRB_TILE);
    if (r) return r;
    c->pers_which = which;
    c->pers_failed = false;   // this launch's error word was cleared by its prepare
    c->pers_waves = waves;
    c->pers_base = c->pers_launched;
    c->pers_first_block = c->block + 1;       // the block the next sdr_frontend produces
    c->pers_stream = s;
    c->pers_launched += (uint32_t)nblocks;
    c->pers_last_n = nblocks;
    return SDR_OK;
}

extern "C++" {
namespace {
// may `block` be signalled next to the pending persistent launch?
int plls_signal_check(const sdr_ctx* c, long long block, const char* what) {
    if (c->pers_signaled == c->pers_launched)
        return fail(SDR_E_INVALID, "%s: no sdr_plls_launch covers this block", what);
    // the launch fixed block j's buffer parity as (first block's parity) ^ j: only the blocks that
    // follow the launch, in order, may be signalled
    const long long want_block = c->pers_first_block + (long long)(c->pers_signaled - c->pers_base);
    if (block != want_block)
        return fail(SDR_E_INVALID, "%s: block %lld, but the launch expects block %lld next", what, block, want_block);
    // a block's done slot is reused PLL_DONE_RING sequence numbers later: every block must have been
    // waited for (sdr_plls_wait) before the one that reuses its slot is signalled
    if (c->pers_signaled - c->pers_waited >= PLL_DONE_RING)
        return fail(SDR_E_INVALID, "%s: %u blocks signalled but not waited for (at most %u in flight)", what,
                    c->pers_signaled - c->pers_waited, PLL_DONE_RING);
    return SDR_OK;
}
}  // namespace
}  // extern "C++"

int sdr_frontend_pre_parts(sdr_ctx* c, const uint8_t* iq, size_t iq_stride, int nparts, void* stream) {
    if (!c || !iq || nparts < 1) return fail(SDR_E_INVALID, "frontend_pre_parts: bad arguments");
    if (const int rf_ = check_failed(c, "frontend_pre_parts")) return rf_;
    if (const int r = check_iq(c, iq, iq_stride)) return r;
    if (!c->rds_on || c->ntaps != FRB_T || (c->flags & SDR_FLAG_FAST_FRONTEND))
        return fail(SDR_E_INVALID, "frontend_pre_parts: needs rds_on, 101 taps and the exact front end");
    if (c->pers_signaled != c->pers_base)
        return fail(SDR_E_INVALID, "frontend_pre_parts: only the first block of a persistent launch comes in parts");
    if (c->pers_which != SDR_PLLS_BOTH)
        return fail(SDR_E_INVALID, "frontend_pre_parts: the launch must cover both PLLs (sdr_plls_launch)");
    if (const int r = plls_signal_check(c, c->block + 1, "frontend_pre_parts")) return r;
    hipStream_t s = S(stream);
    const int n = c->info.block_if, ntiles = cdiv(n, FRB_TILE), fe_tiles = frontend_tiles(n);
    nparts = std::min(nparts, ntiles);
    const int p = c->parity ^ 1;
    const FrontendArgs a = frontend_args(c, iq, iq_stride, p);
    if (const int rw = release_wait(c, p, REL_MONO | REL_STEREO | REL_RDS, s)) return rw;
    const int parity0 = c->parity;
    const long long block0 = c->block;
    c->parity = p;                 // the block's buffers (the pre-PLL FIRs read c->parity)
    c->block++;
    // a launch that fails part-way leaves the context on the previous block (nothing was signalled)
    auto undo = [&](int r) { c->parity = parity0; c->block = block0; return r; };
    // part q: the FIR tiles [x0, x1) and the front-end tiles their windows need (tile j writes
    // outputs [adv j, adv j + adv), adv = 64 R - 1); after each part but the last, the count of
    // published tiles. The front end runs in two launches (SDR_FILL_FE_PARTS 0): the first part's
    // tiles, then all the rest with the second part -- one launch fills the chip where three part
    // launches did not, so the block's front end ends ~0.1 ms earlier and the next block's (which
    // continues its I/Q tail) can start (profiles/r06/fill_fe/ab.txt); SDR_FILL_FE_PARTS 1: one
    // front-end launch per part (round 4)
    const int fe_adv = 64 * frontend_tab_r() - 1;
    int fe_done = 0;
    for (int q = 0; q < nparts; q++) {
        const int x0 = q * ntiles / nparts, x1 = (q + 1) * ntiles / nparts;
        const bool fe_split = q < nparts - 1 && (SDR_FILL_FE_PARTS || q == 0);
        const int fe_end = fe_split ? std::min(fe_tiles, cdiv(std::min(x1 * FRB_TILE, n), fe_adv)) : fe_tiles;
        int r = SDR_OK;
        if (fe_end > fe_done) r = frontend_launch(a, s, fe_done, fe_end - fe_done);
        fe_done = std::max(fe_done, fe_end);
        if (!r) r = pre_launch(c, s, x0, x1 - x0);
        // (capped below PLL_SUB_SCALE: a count above it would reach the values of a later launch)
        if (!r && q < nparts - 1)
            r = launch_flag_store(c->pers_words + PLL_WORD_SUB,
                                  c->pers_base * PLL_SUB_SCALE + std::min((uint32_t)x1, PLL_SUB_SCALE - 1u), s);
        if (r) return undo(r);
    }
    c->st_pre_done = c->rds_pre_done = c->block;
    return sdr_plls_signal(c, stream);   // the whole block: the launch's flag
}

int sdr_plls_signal(sdr_ctx* c, void* stream) {
    if (!c) return fail(SDR_E_INVALID, "null context");
    if (const int rf_ = check_failed(c, "plls_signal")) return rf_;
    const bool st = (c->pers_which & SDR_PLLS_STEREO) != 0, rd = (c->pers_which & SDR_PLLS_RDS) != 0;
    if ((st && (c->st_pre_done != c->block || c->st_pll_done == c->block)) ||
        (rd && (c->rds_pre_done != c->block || c->rds_pll_done == c->block)))
        return fail(SDR_E_INVALID, "plls_signal: run the pre part of every PLL the launch covers (sdr_stereo_pre, "
                                   "sdr_rds_pre) on a new block first");
    if (const int rc = plls_signal_check(c, c->block, "plls_signal")) return rc;
    const int r = launch_flag_store(c->pers_words, c->pers_signaled + 1u, S(stream));
    if (r) return r;
    c->pers_block = c->block;
    c->pers_block_seq = c->pers_signaled;
    c->pers_signaled++;
    if (st) c->st_pll_done = c->block;
    if (rd) c->rds_pll_done = c->block;
    return SDR_OK;
}

int sdr_plls_wait(sdr_ctx* c, void* stream) {
    if (!c) return fail(SDR_E_INVALID, "null context");
    if (const int rf_ = check_failed(c, "plls_wait")) return rf_;
    if (c->pers_block != c->block) return fail(SDR_E_INVALID, "plls_wait: sdr_plls_signal this block first");
    // every wave has finished this block's sequence number (its slot of the done ring)
    const uint32_t seq = c->pers_block_seq;
    const uint32_t want = c->pers_waves * (seq / PLL_DONE_RING + 1u);
    if ((int32_t)(seq + 1u - c->pers_waited) > 0) c->pers_waited = seq + 1u;
    // this stream's post stages read the launch's error word: the next prepare orders its reset after
    // them (a post stream not in the list -- more than PERS_READERS of them -- falls back to a device
    // synchronisation there)
    hipStream_t ws = S(stream);
    if (const int r = launch_flag_wait(c->pers_words + PLL_WORDS_DONE + seq % PLL_DONE_RING, want, c->pers_words + 1, ws))
        return r;
    return pers_reader_mark(c, ws);
}

int sdr_plls_report(sdr_ctx* c, double* block_ms, int max_blocks, int* nblocks, void* stream) {
    if (!c || !c->pers_words) return fail(SDR_E_INVALID, "plls_report: no persistent launch");
    hipStream_t s = S(stream);
    const int n = std::min(c->pers_last_n, std::max(max_blocks, 0));
    std::vector<unsigned long long> t0((size_t)std::max(n, 1)), t1((size_t)std::max(n, 1));
    uint32_t words[PLL_WORDS] = {};
    HIP_TRY(hipMemcpyAsync(words, c->pers_words, sizeof(words), hipMemcpyDeviceToHost, s));
    if (n > 0) {
        HIP_TRY(hipMemcpyAsync(t0.data(), c->pers_t0, n * sizeof(unsigned long long), hipMemcpyDeviceToHost, s));
        HIP_TRY(hipMemcpyAsync(t1.data(), c->pers_t1, n * sizeof(unsigned long long), hipMemcpyDeviceToHost, s));
    }
    HIP_TRY(hipStreamSynchronize(s));
    // block j's PLL time: from when both its input was signalled and the previous block was done
    // (waves drift apart, so the first wave's start can precede the slowest wave's previous end)
    // to its last wave's end, from the 100 MHz s_memrealtime stamps
    for (int j = 0; j < n && block_ms; j++) {
        const unsigned long long from = j > 0 ? std::max(t0[j], t1[j - 1]) : t0[j];
        block_ms[j] = (t1[j] >= from) ? (double)(t1[j] - from) * 1e-5 : -1.0;
    }
    if (nblocks) *nblocks = n;
    if (words[1]) {
        c->pers_failed = true;
        return fail(SDR_E_HIP, "plls_report: a persistent PLL wait timed out (outputs invalid): err %u, flag %u, "
                    "signalled %u, launched %u, waves %u", words[1], words[0], c->pers_signaled, c->pers_launched,
                    c->pers_waves);
    }
    return SDR_OK;
}

int sdr_plls_timeline(sdr_ctx* c, unsigned long long* t_start, unsigned long long* t_end, int max_blocks, int* nblocks,
                      void* stream) {
    if (!c || !c->pers_words) return fail(SDR_E_INVALID, "plls_timeline: no persistent launch");
    hipStream_t s = S(stream);
    const int n = std::min(c->pers_last_n, std::max(max_blocks, 0));
    if (n > 0 && t_start)
        HIP_TRY(hipMemcpyAsync(t_start, c->pers_t0, n * sizeof(unsigned long long), hipMemcpyDeviceToHost, s));
    if (n > 0 && t_end)
        HIP_TRY(hipMemcpyAsync(t_end, c->pers_t1, n * sizeof(unsigned long long), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    if (nblocks) *nblocks = n;
    return SDR_OK;
}

int sdr_plls_cycles(sdr_ctx* c, double* cycles_per_step, double* clock_mhz, void* stream) {
    if (!c || !c->pers_cyc || c->pers_last_n <= 0) return fail(SDR_E_INVALID, "plls_cycles: no persistent launch");
    hipStream_t s = S(stream);
    const int n = c->pers_last_n;
    std::vector<unsigned long long> v((size_t)2 * n);
    HIP_TRY(hipMemcpyAsync(v.data(), c->pers_cyc, v.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    double cyc = 0.0, ticks = 0.0;
    for (int j = 0; j < n; j++) {
        cyc += (double)v[2 * j];
        ticks += (double)v[2 * j + 1];
    }
    const double steps = (double)c->pers_waves * n * c->info.block_if;
    if (cycles_per_step) *cycles_per_step = steps > 0 ? cyc / steps : -1.0;
    if (clock_mhz) *clock_mhz = ticks > 0 ? cyc / ticks * 100.0 : -1.0;   // s_memrealtime runs at 100 MHz
    return SDR_OK;
}

int sdr_plls_block_cycles(sdr_ctx* c, double* cycles_per_step, double* clock_mhz, int max, int* n_out, void* stream) {
    if (!c || !c->pers_cyc || c->pers_last_n <= 0) return fail(SDR_E_INVALID, "plls_block_cycles: no persistent launch");
    hipStream_t s = S(stream);
    const int n = c->pers_last_n;
    std::vector<unsigned long long> v((size_t)2 * n);
    HIP_TRY(hipMemcpyAsync(v.data(), c->pers_cyc, v.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    const double steps = (double)c->pers_waves * c->info.block_if;
    for (int j = 0; j < n && j < max; j++) {
        if (cycles_per_step) cycles_per_step[j] = steps > 0 ? (double)v[2 * j] / steps : -1.0;
        if (clock_mhz) clock_mhz[j] = v[2 * j + 1] ? (double)v[2 * j] / (double)v[2 * j + 1] * 100.0 : -1.0;
    }
    if (n_out) *n_out = n;
    return SDR_OK;
}

int sdr_rds_post(sdr_ctx* c, float* rds_clean, size_t rds_stride, void* stream) {
    if (!c) return fail(SDR_E_INVALID, "null context");
    if (const int rf_ = check_failed(c, "rds_post")) return rf_;
    if (c->rds_pll_done != c->block || c->rds_dsp_done == c->block)
        return fail(SDR_E_INVALID, "rds_post: run sdr_rds_pll on a new block first");
    if (const int rf = check_pers_failed(c, "rds_post")) return rf;
    const sdr_info& in = c->info;
    hipStream_t s = S(stream);
    const int n = in.block_if, T = c->ntaps, p = c->parity;
    float* rband = c->rband + p * c->fm_par;
    float* rdc = c->rdc + p * c->fm_par;
    float* rfilt = c->rfilt + p * c->rf_par;
    if (!(c->flags & SDR_FLAG_KEEP_INTERMEDIATES)) {
        // NCO (rds.cpp:119, pll.cpp:52) + delay (:122) + mixer (:125-127) in one pass (k_rds_mix)
        RdsMix a{};
        a.rband = rband;
        a.t = c->plain(c->t_rds);
        a.fm_stride = c->fm_stride;
        a.plain_stride = c->plain_stride;
        a.car = c->pllbuf(c->ipll);
        a.car_prev = c->ipll + (p ^ 1) * c->pll_par;
        a.car_stride = c->pll_stride;
        a.st = c->rds_pll;
        a.ncoScale = 0.5f;                          // rds.cpp:119: fmpll(..., 0.5, 0, 0.001)
        a.phaseAdjust = 0.0f;
        a.rdc = rdc;
        a.rdc_prev = c->rdc + (p ^ 1) * c->fm_par;
        a.rfilt = rfilt;                            // the resampler's history (below)
        a.rfilt_prev = c->rfilt + (p ^ 1) * c->rf_par;
        a.rf_stride = c->rf_stride;
        a.n = n;
        a.n_rds = in.n_rds;
        hipLaunchKernelGGL(k_rds_mix, dim3(cdiv(n + 1, BLK * MIX_R), c->nch), dim3(BLK), 0, s, a);
        LAUNCH_CHECK();
        if (const int rr = release_record(c, REL_RDS, s)) return rr;   // rband, t_rds, ipll read
    } else {
        {
            PllJobs jobs{};
            jobs.j[0] = rds_job(c);                   // NCO output of this block's PLL (rds.cpp:119)
            const int r = launch_nco(jobs, 1, n, c->nch, s);
            if (r) return r;
        }
        // delay (rds.cpp:122) + mixer (:125-127) into the extended rds_dc stream
        hipLaunchKernelGGL(k_mix<true>, dim3(cdiv(n, BLK), c->nch), dim3(BLK), 0, s, rband, c->fm_stride,
                           c->pllbuf(c->ipll), c->pll_stride, n, rdc, c->rdc + (p ^ 1) * c->fm_par, c->fm_stride, 50);
        LAUNCH_CHECK();
        if (const int rr = release_record(c, REL_RDS, s)) return rr;
        hipLaunchKernelGGL(k_hist_copy, dim3(c->nch), dim3(HIST), 0, s, rfilt, c->rfilt + (p ^ 1) * c->rf_par,
                           c->rf_stride, in.n_rds);
        LAUNCH_CHECK();
    }
    // 247/640 resampler (:130) into the extended rds_filt stream (history: k_rds_mix / k_hist_copy above)
    if (resample_lc_span(c->rdsbb_L, 247, 640) > 64 * RLC_XL || ((c->rdsbb_L + 3) & ~3) > 64 * RLC_HL)
        return fail(SDR_E_INVALID, "rds_post: resampler tile does not fit (L = %d)", c->rdsbb_L);
    dim3 gr(cdiv(in.n_rds, RLC_TN), cdiv(c->nch, 64));
    auto kr = c->rdsbb_all101 ? k_resample_lc<101> : k_resample_lc<0>;
    hipLaunchKernelGGL(kr, gr, dim3(RLC_BLK), resample_lc_lds_bytes(c->rdsbb_L, 247, 640, !c->rdsbb_all101), s, rdc,
                       c->fm_stride, -HIST, c->rdsbb_pp, c->rdsbb_cnt, c->rdsbb_L, c->rds_ptq, in.n_rds, c->nch,
                       rfilt, c->rf_stride);
    LAUNCH_CHECK();
    // RRC (:133) into the context's rds_clean (sdr_rds_bits reads it) and the caller's buffer
    if (T != FRB_T) return fail(SDR_E_INVALID, "rds_post: %d taps", T);
    {
        FirRb f{};
        f.h[0] = c->rrc_h;
        f.y[0] = c->rds_clean;
        f.y_stride[0] = c->clean_stride;
        f.ydup = rds_clean;
        f.ydup_stride = rds_stride;
        f.err = block_poison(c);                    // NaN rows after a persistent PLL or release timeout
        const int r = fir_rb<1, false>(c, rfilt, c->rf_stride, in.n_rds, f, s);
        if (r) return r;
    }
    c->rds_dsp_done = c->block;
    return pers_reader_mark(c, s);
}

int sdr_rds_dsp(sdr_ctx* c, float* rds_clean, size_t rds_stride, void* stream) {
    if (!c) return fail(SDR_E_INVALID, "null context");
    if (c->block < 0 || c->rds_dsp_done == c->block) return fail(SDR_E_INVALID, "rds: no new block");
    int r = sdr_rds_pre(c, stream);
    if (!r) r = sdr_rds_pll(c, stream);
    if (!r) r = sdr_rds_post(c, rds_clean, rds_stride, stream);
    return r;
}

int sdr_rds_bits(sdr_ctx* c, int32_t* offset, int32_t* nsym, uint8_t* symbols, size_t sym_stride, int32_t* nbits,
                 uint8_t* bits, size_t bits_stride, void* stream) {
    if (!c) return fail(SDR_E_INVALID, "null context");
    if (const int rf_ = check_failed(c, "rds_bits")) return rf_;
    if (c->rds_dsp_done != c->block || c->rds_bits_done == c->block)
        return fail(SDR_E_INVALID, "rds_bits: run sdr_rds_dsp on a new block first");
    if (const int rf = check_pers_failed(c, "rds_bits")) return rf;
    const sdr_info& in = c->info;
    hipLaunchKernelGGL(k_rds_bits, dim3(c->nch), dim3(64), (size_t)in.n_rds * sizeof(float),
                       S(stream), c->rds_clean,
                       c->clean_stride, in.n_rds, in.symbol_Fs, c->rds_on, c->dec, offset, nsym, symbols,
                       sym_stride, nbits, bits, bits_stride, block_poison(c),
                       (reinterpret_cast<uintptr_t>(c->rds_clean) % 16 == 0 && c->clean_stride % 4 == 0) ? 1 : 0);
    LAUNCH_CHECK();
    c->rds_bits_done = c->block;
    return pers_reader_mark(c, S(stream));
}

int sdr_ctx_buffer(sdr_ctx* c, const char* name, const float** ptr, size_t* stride, int* len) {
    if (!c || !name || !ptr || !stride || !len) return fail(SDR_E_INVALID, "null argument");
    const sdr_info& in = c->info;
    const int p = c->parity;
    struct E { const char* n; const float* p; size_t s; int l; } tab[] = {
        {"fm", c->fm_cur(), c->fm_stride, in.block_if},
        {"pilot", c->plain(c->pilot), c->plain_stride, in.block_if},
        {"carrier", c->pllbuf(c->carrier), c->pll_stride, in.block_if + 1},
        {"band", c->plain(c->band), c->plain_stride, in.block_if},
        {"stereo_dc", c->sdc + p * c->fm_par, c->fm_stride, in.block_if},
        {"rds_band", c->rband + p * c->fm_par, c->fm_stride, in.block_if},
        {"gen_pilot", c->plain(c->gpilot), c->plain_stride, in.block_if},
        {"ipll", c->pllbuf(c->ipll), c->pll_stride, in.block_if + 1},
        {"rds_dc", c->rdc + p * c->fm_par, c->fm_stride, in.block_if},
        {"rds_filt", c->rfilt + p * c->rf_par, c->rf_stride, in.n_rds},
        {"rds_clean", c->rds_clean, c->clean_stride, in.n_rds},
    };
    for (const E& e : tab) {
        if (std::strcmp(e.n, name) == 0) {
            *ptr = e.p;
            *stride = e.s;
            *len = e.l;
            return SDR_OK;
        }
    }
    return fail(SDR_E_INVALID, "unknown buffer %s", name);
}

// ------------------------------------------------------------------ batched primitives
int sdr_convolve_fir(float* y, size_t y_stride, const float* x, size_t x_stride, int nch, int nx, const float* h,
                     int ntaps, float* state, int nstate, int D, void* stream) {
    if (!y || !x || !h || !state || nch <= 0 || nx <= 0 || ntaps <= 0 || D <= 0 || nstate < ntaps - 1)
        return fail(SDR_E_INVALID, "convolve_fir: bad arguments (nstate must be >= ntaps-1)");
    const int ny = nx / D;
    if (ny > 0) {
        const int tile = FIR_TILE;
        const size_t lds = fir_lds_bytes(ntaps, 1, tile, D);
        if (lds > 160 * 1024) return fail(SDR_E_INVALID, "convolve_fir: ntaps*D too large for one tile");
        hipLaunchKernelGGL((k_fir<1, false>), dim3(cdiv(ny, tile), nch), dim3(BLK), lds, S(stream), x, x_stride,
                           state + nstate, (size_t)nstate, h, nullptr, ntaps, D, ny, tile, y, nullptr, y_stride, nullptr, 0);
        LAUNCH_CHECK();
    }
    hipLaunchKernelGGL(k_state_update, dim3(nch), dim3(256), 0, S(stream), state, nstate, x, x_stride, nx);
    LAUNCH_CHECK();
    return SDR_OK;
}

namespace {
// polyphase tables of the taps the primitive resampler has been called with, keyed by (U, tap
// values): the reference's callers use a few fixed filters, so entries are kept (never freed
// under a kernel still in flight) and the set is only dropped, after a device sync, if it grows
struct PPEntry {
    int U = 0;
    std::vector<float> host;
    float* table = nullptr;
    int* cnt = nullptr;
    int L = 0;
};
struct PPCache {
    std::mutex m;
    std::vector<PPEntry> e;
};
PPCache g_pp;
constexpr size_t PP_CACHE_MAX = 16;
}  // namespace

int sdr_convolve_fir_resample(float* y, size_t y_stride, const float* x, size_t x_stride, int nch, int nx,
                              const float* h, int ntaps, float* state, int nstate, int U, int D, void* stream) {
    if (!y || !x || !h || !state || nch <= 0 || nx <= 0 || ntaps <= 0 || U <= 0 || D <= 0)
        return fail(SDR_E_INVALID, "convolve_fir_resample: bad arguments");
    const int ny = (int)(((long long)nx * U) / D);
    // polyphase table of the (device) taps; the taps are read on the caller's stream so that a
    // preceding asynchronous upload of them on that stream is complete
    std::vector<float> hh(ntaps);
    HIP_TRY(hipMemcpyAsync(hh.data(), h, ntaps * sizeof(float), hipMemcpyDeviceToHost, S(stream)));
    HIP_TRY(hipStreamSynchronize(S(stream)));
    std::lock_guard<std::mutex> lk(g_pp.m);
    const PPEntry* pe = nullptr;
    for (const PPEntry& e : g_pp.e)
        if (e.U == U && e.host == hh) { pe = &e; break; }
    if (!pe) {
        if (g_pp.e.size() >= PP_CACHE_MAX) {
            HIP_TRY(hipDeviceSynchronize());
            for (PPEntry& e : g_pp.e) { (void)hipFree(e.table); (void)hipFree(e.cnt); }
            g_pp.e.clear();
        }
        Polyphase pp = make_polyphase(hh, U);
        PPEntry ne;
        ne.U = U; ne.host = hh; ne.L = pp.L;
        HIP_TRY(hipMalloc(&ne.table, pp.table.size() * sizeof(float)));
        HIP_TRY(hipMalloc(&ne.cnt, pp.cnt.size() * sizeof(int)));
        HIP_TRY(hipMemcpy(ne.table, pp.table.data(), pp.table.size() * sizeof(float), hipMemcpyHostToDevice));
        HIP_TRY(hipMemcpy(ne.cnt, pp.cnt.data(), pp.cnt.size() * sizeof(int), hipMemcpyHostToDevice));
        g_pp.e.push_back(std::move(ne));
        pe = &g_pp.e.back();
    }
    // the deepest look-back is output 0: x[-(ceil(ntaps/U)-1)] (100 in every mode)
    const int lookback = (ntaps + U - 1) / U - 1;
    if (nstate < lookback)
        return fail(SDR_E_INVALID, "convolve_fir_resample: nstate %d < look-back %d", nstate, lookback);
    if (ny > 0) {
        const int tile = 256;
        const size_t lds = resample_lds_bytes(pe->L, U, D, tile, 1);
        hipLaunchKernelGGL(k_resample<0>, dim3(cdiv(ny, tile), nch), dim3(BLK), lds, S(stream), x, state + nstate,
                           x_stride, (size_t)nstate, nullptr, nullptr, (size_t)0, (size_t)0, pe->table, pe->cnt,
                           pe->L, U, D, ny, tile, -nstate, (void*)y, y_stride);
        LAUNCH_CHECK();
    }
    hipLaunchKernelGGL(k_state_update, dim3(nch), dim3(256), 0, S(stream), state, nstate, x, x_stride, nx);
    LAUNCH_CHECK();
    return SDR_OK;
}

int sdr_fm_demod(float* out, size_t out_stride, const float* I, const float* Q, size_t iq_stride, int nch, int n,
                 float* prev, void* stream) {
    if (!out || !I || !Q || !prev || nch <= 0 || n <= 0) return fail(SDR_E_INVALID, "fm_demod: bad arguments");
    hipLaunchKernelGGL(k_demod, dim3(cdiv(n, BLK), nch), dim3(BLK), 0, S(stream), out, out_stride, I, Q, iq_stride, n,
                       reinterpret_cast<const float2*>(prev));
    LAUNCH_CHECK();
    hipLaunchKernelGGL(k_demod_prev, dim3(cdiv(nch, 64)), dim3(64), 0, S(stream), reinterpret_cast<float2*>(prev), I,
                       Q, iq_stride, n, nch);
    LAUNCH_CHECK();
    return SDR_OK;
}

int sdr_fmpll(float* out, size_t out_stride, const float* in, size_t in_stride, int nch, int n, float freq, float Fs,
              sdr_pll_state* state, float ncoScale, float phaseAdjust, float normBandwidth, void* stream) {
    if (!out || !in || !state || nch <= 0 || n < 0) return fail(SDR_E_INVALID, "fmpll: bad arguments");
    const size_t ts = round_up((size_t)std::max(n, 1), 4);
    // scratch: input reciprocals (f64), phases and -in (f32), each [nch][ts]
    const size_t rx_bytes = ts * nch * sizeof(double), t_bytes = 2 * ts * nch * sizeof(float);
    hipStream_t s = S(stream);
    // one scratch buffer per stream, reused in that stream's order (buffers from the
    // stream-ordered pool, hipMallocAsync / hipFreeAsync per call, came back wrong)
    void* scratch = nullptr;
    std::unique_lock<std::mutex> lk(g_scratch_mu);   // held until the PLL kernels are enqueued
    {
        const int rc = stream_scratch(s, rx_bytes + t_bytes, &scratch);
        if (rc != SDR_OK) return rc;
    }
    double* rxbuf = static_cast<double*>(scratch);
    float* tbuf = reinterpret_cast<float*>(rxbuf + ts * nch);
    return launch_pll(false, in, in_stride, n, nch, freq, Fs, tbuf, ts, rxbuf, tbuf + ts * nch, out, out_stride,
                      state, ncoScale, phaseAdjust, normBandwidth, s);
}

int sdr_cdr(int32_t* offset, const float* x, size_t x_stride, int nch, int n, int sps, void* stream) {
    if (!offset || !x || nch <= 0 || n < 0 || sps <= 0 || sps > 64) return fail(SDR_E_INVALID, "cdr: bad arguments");
    hipLaunchKernelGGL(k_cdr, dim3(nch), dim3(64), 0, S(stream), offset, x, x_stride, n, sps);
    LAUNCH_CHECK();
    return SDR_OK;
}

int sdr_manchester_decode(uint8_t* bits, size_t bits_stride, int32_t* nbits, const uint8_t* symbols, size_t sym_stride,
                          const int32_t* nsym, int nch, int block_count, int32_t* state, void* stream) {
    if (!bits || !nbits || !symbols || !nsym || !state || nch <= 0) return fail(SDR_E_INVALID, "manchester: bad arguments");
    hipLaunchKernelGGL(k_manchester, dim3(cdiv(nch, 64)), dim3(64), 0, S(stream), bits, bits_stride, nbits, symbols,
                       sym_stride, nsym, nch, block_count, state);
    LAUNCH_CHECK();
    return SDR_OK;
}

int sdr_differential_decode(uint8_t* out, size_t out_stride, const uint8_t* bits, size_t bits_stride,
                            const int32_t* nbits, int nch, int block_num, int32_t* last_bit, void* stream) {
    if (!out || !bits || !nbits || !last_bit || nch <= 0) return fail(SDR_E_INVALID, "differential: bad arguments");
    hipLaunchKernelGGL(k_differential, dim3(cdiv(nch, 64)), dim3(64), 0, S(stream), out, out_stride, bits, bits_stride,
                       nbits, nch, block_num, last_bit);
    LAUNCH_CHECK();
    return SDR_OK;
}

int sdr_push_fm_demod(sdr_ctx* c, const float* fm, size_t fm_stride, void* stream) {
    if (!c || !fm) return fail(SDR_E_INVALID, "null argument");
    if (const int rf_ = check_failed(c, "push_fm_demod")) return rf_;
    const sdr_info& in = c->info;
    const int p = c->parity ^ 1;
    float* dst = c->fm + p * c->fm_par;
    if (const int rw = release_wait(c, p, REL_MONO | REL_STEREO, S(stream))) return rw;
    if (const int r = copy_rows(dst, c->fm_stride, fm, fm_stride, in.block_if, c->nch, c->fm + (p ^ 1) * c->fm_par,
                                S(stream)))
        return r;
    c->parity = p;
    c->block++;
    return SDR_OK;
}

}  // extern "C"

