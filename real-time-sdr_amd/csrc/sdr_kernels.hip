// sdr_kernels.hip -- MI355X (gfx950) kernels, launchers and C ABI of the FM/RDS DSP hot path.
//
// Hot path of TheZxc07/real-time-SDR recast as batched kernels over many independent channels:
//   front end   u8 I/Q -> 101-tap FIR /10 on I and Q -> FM discriminator    rffrontend.cpp:58-71
//   mono        101-tap resampler U/D -> int16                            mono.cpp:34-42
//   stereo      pilot BPF -> PLL(19k, x2) ; band BPF ; mixer ; delay ; 2 resamplers -> L/R
//                                                                          stereo.cpp:74-107
//   rds DSP     BPF -> square -> BPF -> PLL(114k, x0.5) ; delay ; mixer -> 247/640 resampler
//               -> RRC                                                     rds.cpp:105-133
//   rds bits    cdr -> slicer -> Manchester -> differential               rds.cpp:135-167
//
// Numerics ("exact" mode, default): every kernel keeps the reference's rounding points --
// f32 product then f32 add in tap order (no contraction: `fp contract(off)` below), the
// discriminator's f64 denominator/division, the PLL's f64 atan2/sin/cos on f32 arguments.
//
// Layout: channel-major [nch][len]. Every f32 stream that a later FIR/resampler reads with
// look-back is kept "extended": [2 parities][nch][HIST + len], the first HIST samples being the
// previous block's last HIST samples, so a kernel reads x[-HIST..len) with no branch; the
// producer of block b copies the history from the parity of block b-1.

#include <hip/hip_runtime.h>

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

#pragma clang fp contract(off)

namespace {

constexpr int HIST = 160;        // history samples in front of every extended f32 stream (>= 150)
constexpr int BLK = 256;         // threads per workgroup for the streaming kernels
constexpr int FIR_TILE = 512;    // outputs per workgroup for the 101-tap FIRs
constexpr int DEC_STATE = 8;     // ints of RDS decoder state per channel

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

#define HIP_TRY(expr)                                                                       \
    do {                                                                                    \
        hipError_t e_ = (expr);                                                             \
        if (e_ != hipSuccess) return fail(SDR_E_HIP, "%s: %s", #expr, hipGetErrorString(e_)); \
    } while (0)

#define LAUNCH_CHECK()                                                                              \
    do {                                                                                            \
        hipError_t e_ = hipGetLastError();                                                          \
        if (e_ != hipSuccess) return fail(SDR_E_HIP, "launch failed at %s:%d: %s", __FILE__, __LINE__, \
                                          hipGetErrorString(e_));                                   \
    } while (0)

// static_cast<short>(float) as g++/x86-64 lowers it (mono.cpp:41, stereo.cpp:101-102):
// cvttss2si (INT_MIN when out of range or NaN), then the low 16 bits.
__device__ __forceinline__ int32_t cvt_i32_x86(float v) {
    return (v >= -2147483648.0f && v < 2147483648.0f) ? (int32_t)v : INT32_MIN;
}
__device__ __forceinline__ int16_t cvt_i16_x86(float v) {
    return (int16_t)(uint16_t)((uint32_t)cvt_i32_x86(v) & 0xFFFFu);
}

// ------------------------------------------------------------------------------------------
// Front end: u8 I/Q -> decimating FIR on I and Q -> discriminator (rffrontend.cpp:58-71,
// filter.cpp:106-121, demod.cpp:3-24). Grid (tiles, nch). A tile computes decimated outputs
// [c0, n1) (c0 = n0-1 so the discriminator has its previous sample) from an LDS window of
// converted I/Q pairs, then writes fm_demod[n0, n1).
// State: tail = last (ntaps-1) I/Q pairs of the previous block (u8, 128 == 0.0f),
//        prev = last decimated (I, Q) of the previous block. Both double-buffered by parity.
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(BLK) void k_frontend(
    const uint8_t* __restrict__ iq, size_t iq_stride, const uint8_t* __restrict__ tail_in,
    uint8_t* __restrict__ tail_out, const float2* __restrict__ prev_in, float2* __restrict__ prev_out,
    const float* __restrict__ h, int ntaps, int D, int block_iq, int block_if, int tile,
    float* __restrict__ fm, const float* __restrict__ fm_other, size_t fm_stride) {
    extern __shared__ float4 smem4[];
    const int ntaps_pad = (ntaps + 3) & ~3;
    float* sh = reinterpret_cast<float*>(smem4);
    const int ch = blockIdx.y;
    const int tid = threadIdx.x;
    const int n0 = blockIdx.x * tile;
    const int n1 = min(n0 + tile, block_if);
    const int c0 = max(n0 - 1, 0);
    const int m0 = c0 * D - (ntaps - 1);
    const int m1 = (n1 - 1) * D;
    const int W = m1 - m0 + 1;
    float2* sx = reinterpret_cast<float2*>(sh + ntaps_pad);
    float2* sds = sx + ((W + 1) & ~1);
    const int hist_pairs = ntaps - 1;
    const uint16_t* src = reinterpret_cast<const uint16_t*>(iq + (size_t)ch * iq_stride);
    const uint16_t* tin = reinterpret_cast<const uint16_t*>(tail_in + (size_t)ch * 2 * hist_pairs);

    for (int i = tid; i < ntaps; i += BLK) sh[i] = h[i];
    for (int i = tid; i < W; i += BLK) {
        const int m = m0 + i;
        const uint32_t pr = (m < 0) ? tin[hist_pairs + m] : src[m];
        // float(((u - 128.0) / 128.0)) is exactly (u - 128) * 2^-7
        sx[i] = make_float2(((float)(pr & 0xFFu) - 128.0f) * 0.0078125f, ((float)(pr >> 8) - 128.0f) * 0.0078125f);
    }
    __syncthreads();
    for (int c = c0 + tid; c < n1; c += BLK) {
        const int base = c * D - m0;
        float aI = 0.0f, aQ = 0.0f;
        for (int k = 0; k < ntaps; k++) {
            const float hk = sh[k];
            const float2 v = sx[base - k];
            aI = aI + hk * v.x;
            aQ = aQ + hk * v.y;
        }
        sds[c - c0] = make_float2(aI, aQ);
    }
    __syncthreads();
    float* out = fm + (size_t)ch * fm_stride;
    for (int n = n0 + tid; n < n1; n += BLK) {
        const float2 cur = sds[n - c0];
        const float2 pv = (n == 0) ? prev_in[ch] : sds[n - 1 - c0];
        float r;
        if ((cur.x == 0) & (cur.y == 0)) {
            r = 0.0f;
        } else {
            const float num = cur.x * (cur.y - pv.y) - cur.y * (cur.x - pv.x);
            const double den = (double)cur.x * (double)cur.x + (double)cur.y * (double)cur.y;
            r = (float)((double)num / den);
        }
        out[n] = r;
    }
    if (n1 == block_if && tid == 0) prev_out[ch] = sds[n1 - 1 - c0];
    if (blockIdx.x == 0) {
        const uint16_t* last = src + (block_iq - hist_pairs);
        uint16_t* tout = reinterpret_cast<uint16_t*>(tail_out + (size_t)ch * 2 * hist_pairs);
        for (int i = tid; i < hist_pairs; i += BLK) tout[i] = last[i];
        const float* o = fm_other + (size_t)ch * fm_stride;
        for (int i = tid; i < HIST; i += BLK) out[i - HIST] = o[block_if - HIST + i];
    }
}

// ------------------------------------------------------------------------------------------
// Front end v2 (register-blocked). Each thread computes R consecutive decimated outputs (I and Q
// as one packed f32 pair) by streaming its input window in DESCENDING sample order: every output
// then still accumulates its taps in ascending k (filter.cpp:110-116), while each input sample is
// converted once and feeds up to R outputs. Conversion: u8 -> signed byte (u ^ 0x80 = u - 128)
// -> f32 m via SDWA sext; with taps pre-scaled by 2^-7 (hs = h/128, exact) the product
// fl(hs*m) equals the reference's fl(h*x), x = (u-128)/128, bit for bit.
//   exact: v_pk_mul_f32 + v_pk_add_f32 (separate roundings, like filter.cpp:115)
//   FAST:  v_pk_fma_f32 (one rounding per tap; fm_demod within ~1e-6 relative)
// A tile computes TILE = 256*R outputs starting one before the first fm_demod sample it writes
// (the discriminator's carry, demod.cpp:16), so tiles advance by TILE-1. The u8 window is staged
// in LDS with coalesced dword loads (D even) or u16 loads (D odd).
// ------------------------------------------------------------------------------------------
typedef float f32x2 __attribute__((ext_vector_type(2)));

// One input sample S (descending) of the register-blocked FIR: up to R independent packed MACs,
// then recursion to S-1 -- complete unrolling with compile-time chunk and tap indices. A
// sched_barrier closes every sample so the scheduler keeps the sample-major order (ILP across the
// R accumulators, each product next to its add) instead of hoisting products or serialising one
// output's chain; the LDS chunk two chunks ahead is read at each chunk boundary.
#ifndef SDR_FE_PF
#define SDR_FE_PF 5
#endif
#ifndef SDR_FE_CVT_MID
#define SDR_FE_CVT_MID 0   // 1: conversion between the products (more hazard wait states: not adopted)
#endif
constexpr int FE_PF = SDR_FE_PF;   // tap rows prefetched this many samples ahead (rotating SGPR ring)

// {h, h} * m with h one half (HI) of an SGPR pair: v_pk_mul_f32 with a scalar operand whose half
// is broadcast to both lanes by op_sel / op_sel_hi (no VGPR copy of the tap)
__device__ __forceinline__ f32x2 fe_mul_v(double hpair, int hi, f32x2 m) {
    f32x2 r;
    if (hi) asm volatile("v_pk_mul_f32 %0, %1, %2 op_sel:[1,0] op_sel_hi:[1,1]" : "=v"(r) : "s"(hpair), "v"(m));
    else asm volatile("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[0,1]" : "=v"(r) : "s"(hpair), "v"(m));
    return r;
}
// (I, Q) of one sample, sign-extended from the bytes of a dword that holds two samples
// (u8 ^ 0x80 == u8 - 128 as int8), converted in program order (volatile asm)
#ifndef SDR_FE_CVT_C
#define SDR_FE_CVT_C 0
#endif
template <int HALF>
__device__ __forceinline__ f32x2 fe_cvt_v(uint32_t w) {
    f32x2 r;
#if SDR_FE_CVT_C
    // plain C++ (the SDWA peephole forms the same sext-byte conversions): no inline-asm hazard
    r.x = (float)(int)(int8_t)(uint8_t)(w >> (16 * HALF));
    r.y = (float)(int)(int8_t)(uint8_t)(w >> (16 * HALF + 8));
    return r;
#endif
    if (HALF) {
        asm volatile("v_cvt_f32_i32_sdwa %0, sext(%2) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_2\n\t"
                     "v_cvt_f32_i32_sdwa %1, sext(%2) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_3"
                     : "=&v"(r.x), "=v"(r.y) : "v"(w));
    } else {
        asm volatile("v_cvt_f32_i32_sdwa %0, sext(%2) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_0\n\t"
                     "v_cvt_f32_i32_sdwa %1, sext(%2) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1"
                     : "=&v"(r.x), "=v"(r.y) : "v"(w));
    }
    return r;
}
#ifndef SDR_FE_ADD_C
#define SDR_FE_ADD_C 0
#endif
__device__ __forceinline__ f32x2 fe_add_v(f32x2 a, f32x2 b) {
#if SDR_FE_ADD_C
    return a + b;   // v_pk_add_f32, ordered by its operands (no inline-asm hazard wait after the products)
#else
    f32x2 r;
    asm volatile("v_pk_add_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
#endif
}
__device__ __forceinline__ f32x2 fe_fma(double hpair, int hi, f32x2 m, f32x2 acc) {
    f32x2 r;
    if (hi) asm volatile("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,0,0] op_sel_hi:[1,1,1]" : "=v"(r) : "s"(hpair), "v"(m), "v"(acc));
    else asm volatile("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[0,1,1]" : "=v"(r) : "s"(hpair), "v"(m), "v"(acc));
    return r;
}

// ------------------------------------------------------------------------------------------
// Fast-mode front end on the matrix cores (SDR_FLAG_FAST_FRONTEND): the decimating FIR as an
// integer GEMM. A wave owns a tile of NB (16, 24 or 32; default 32) blocks of 16 consecutive decimated outputs of one
// channel. Block b's outputs need a 256-sample window w_b (x[D*c_b - 100 + s], s < 256, of which
// 15*D + 101 are used) and y[c_b + i] = sum_s W[i][s] * w_b[s] with the Toeplitz tap matrix
// W[i][s] = h[D*i + 100 - s]. Samples are exact int8 (u8 - 128); the taps are fixed point with
// 2^-(31 - ceil(log2 max|h|)) resolution split into FT_ND = 4 balanced base-256 digits, so
// v_mfma_i32_16x16x64_i8 (rows = 16 outputs, columns = 8 blocks x {I, Q}, K = 4 x 64) accumulates
// each digit plane exactly in int32 and the planes combine exactly in f64: y is the correctly
// rounded f32 of the convolution with the quantised taps (<= ~1e-8 absolute from the exact one,
// so ~1e-6 relative even at 1-LSB input amplitude; 3 digits measured 1e-4 on a filter start-up
// transient). North-star tolerance 1e-5 relative on fm_demod, RDS bits bit-exact: tested.
// Staging: u8 I/Q pairs -> planar int8 I and Q rows in LDS (v_perm deinterleave); each B
// fragment is then one ds_read_b128 (16 consecutive samples of one component).
// ------------------------------------------------------------------------------------------
typedef int v4i __attribute__((ext_vector_type(4)));
// NB = 16-output blocks per wave tile (NB/8 C tiles of 8 blocks). Tile j computes outputs
// c0 .. c0 + 16*NB - 1 with c0 = j*ADV - CARRY and writes the ADV outputs from c0 + CARRY on (the
// CARRY >= 1 before them feed the discriminator). (ADV, CARRY) per D make the first staged sample
// m0 = c0*D - 100 a multiple of 8 (16-byte I/Q groups) on every tile.
constexpr int ft_adv(int D, int NB) { return D == 3 ? 16 * NB - 8 : 16 * NB - 4; }
constexpr int ft_carry(int D) { return D == 10 ? 2 : D == 4 ? 1 : 4; }
constexpr int FT_ND = 4;                  // digit planes (32-bit fixed-point taps)
constexpr int FT_AFRAGS = 4 * FT_ND;      // K steps x digit planes
constexpr int ft_win(int D, int NB) { return 16 * D * (NB - 1) + 256; }
constexpr int FT_NB_DEFAULT = 32;
#ifndef FT_RECOMB_F64
#define FT_RECOMB_F64 0
#endif
#ifndef FT_DIAG
#define FT_DIAG 0   // timing-only diagnosis of k_frontend_mfma (1: no compute, 2: no tap loads)
#endif
#ifndef FT_CT_UNROLL
#define FT_CT_UNROLL 1
#endif

// One wave tile of the MFMA front end: NB blocks of 16 outputs (c0 + 16*bb + row) from the staged
// window in LDS, written to out[lo, hi). Shared by the one-tile-per-workgroup kernel (planar image)
// and the persistent LDS-DMA kernel (raw image).
template <int D, int NB, bool RAW>
__device__ __forceinline__ void ft_tile(const int8_t* __restrict__ lds, const v4i (&A)[FT_AFRAGS], double yscale,
                                        int c0, int ch, float2 prev_in_ch,
                                        float2* __restrict__ prev_out, int block_if, float* __restrict__ out) {
    constexpr int WIN = ft_win(D, NB), ADV = ft_adv(D, NB), CARRY = ft_carry(D);
    const float ys = (float)yscale;                   // 2^-(F+7): exact in f32
    const int t = threadIdx.x;
    // C layout of v_mfma_i32_16x16x64_i8: lane t holds rows 4g..4g+3 (g = t>>4) of column n = t&15;
    // column n = block 8*ct + (n>>1), component n&1 (I even, Q odd)
    const int n = t & 15, g = t >> 4, comp = n & 1;
    // B operand: 16 consecutive samples of this lane's component. Planar image (RAW false): one
    // 16-byte read of the signed I or Q plane. Raw image (RAW true: the interleaved u8 I/Q bytes as
    // the LDS-DMA lands them): two 16-byte reads, de-interleaved by v_perm and made signed (u8 ^ 0x80).
    const int8_t* prow = RAW ? lds : lds + comp * WIN;
    const uint32_t psel = comp ? 0x07050301u : 0x06040200u;
    const int lo = max(c0 + CARRY, 0), hi = min(c0 + CARRY + ADV, block_if);
    float carry_i = 0.0f, carry_q = 0.0f;             // last output of the previous C tile
#pragma unroll FT_CT_UNROLL
    for (int ct = 0; ct < NB / 8; ct++) {
        const int bb = 8 * ct + (n >> 1);             // this lane's block
        v4i acc[FT_ND];
#pragma unroll
        for (int p = 0; p < FT_ND; p++) acc[p] = v4i{0, 0, 0, 0};
#pragma unroll
        for (int kk = 0; kk < 4; kk++) {
            v4i B;
            if (RAW) {
                const uint4* rp = reinterpret_cast<const uint4*>(prow + 2 * (16 * D * bb + 64 * kk + 16 * g));
                const uint4 r0 = rp[0], r1 = rp[1];
                B = v4i{(int)(__builtin_amdgcn_perm(r0.y, r0.x, psel) ^ 0x80808080u),
                        (int)(__builtin_amdgcn_perm(r0.w, r0.z, psel) ^ 0x80808080u),
                        (int)(__builtin_amdgcn_perm(r1.y, r1.x, psel) ^ 0x80808080u),
                        (int)(__builtin_amdgcn_perm(r1.w, r1.z, psel) ^ 0x80808080u)};
            } else {
                B = *reinterpret_cast<const v4i*>(prow + 16 * D * bb + 64 * kk + 16 * g);
            }
#pragma unroll
            for (int p = 0; p < FT_ND; p++)
                acc[p] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A[FT_ND * kk + p], B, acc[p], 0, 0, 0);
        }
        // recombination of the digit planes: y = this lane's component of rows 4g..4g+3, yo = the
        // other component (DPP quad_perm 1,0,3,2)
        static_assert(FT_ND == 4, "pairwise recombination assumes 4 digit planes");
        float y[4], yo[4];
#if FT_RECOMB_F64
        (void)ys;
#endif
#pragma unroll
        for (int r = 0; r < 4; r++) {
            // digits pair up exactly in int32 (|acc| <= 101 * 128 * 128 < 2^21)
            const int hi2 = (acc[0][r] << 8) + acc[1][r], lo2 = (acc[2][r] << 8) + acc[3][r];
#if FT_RECOMB_F64
            // exact in f64 (|sum| < 2^53), one rounding to f32
            y[r] = (float)(((double)hi2 * 65536.0 + (double)lo2) * yscale);
#else
            // f32: hi2 rounds once (< 2^-24 relative), the power-of-two scalings are exact, one fma:
            // within ~1 ulp of the exact sum at a quarter of the f64 issue cost
            y[r] = __builtin_fmaf((float)hi2, ys * 65536.0f, (float)lo2 * ys);
#endif
            yo[r] = __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, y[r]), 0xB1, 0xF,
                                                                       0xF, false));
        }
        const float I3 = comp ? yo[3] : y[3], Q3 = comp ? y[3] : yo[3];
        // previous output of row 4g: row 4g-1 of the same block (lane t-16), or row 15 of block bb-1
        // (lane t-2+48), or for the first block of the C tile the carry from the previous one
        const int src_lane = g > 0 ? t - 16 : ((n >> 1) > 0 ? t - 2 + 48 : t);
        const float sI = __shfl(I3, src_lane), sQ = __shfl(Q3, src_lane);
        const bool first = (g == 0 && (n >> 1) == 0);
        const float pI = first ? carry_i : sI, pQ = first ? carry_q : sQ;
        carry_i = __shfl(I3, 62);
        carry_q = __shfl(Q3, 62);
        // the discriminator is split over the lane pair: the I lane takes rows 0, 1, the Q lane rows 2, 3
        const int cb = c0 + 16 * bb + 4 * g + 2 * comp;   // output index of this lane's first row
        float aI[3], aQ[3];                               // prev, row, row+1
        {
            const float I0 = comp ? yo[0] : y[0], Q0 = comp ? y[0] : yo[0];
            const float I1 = comp ? yo[1] : y[1], Q1 = comp ? y[1] : yo[1];
            const float I2 = comp ? yo[2] : y[2], Q2 = comp ? y[2] : yo[2];
            aI[0] = comp ? I1 : pI; aQ[0] = comp ? Q1 : pQ;
            aI[1] = comp ? I2 : I0; aQ[1] = comp ? Q2 : Q0;
            aI[2] = comp ? I3 : I1; aQ[2] = comp ? Q3 : Q1;
        }
        float v[2];
#pragma unroll
        for (int r = 0; r < 2; r++) {
            const int c = cb + r;
            float qI = aI[r], qQ = aQ[r];
            if (c == 0) {
                const float2 pv = prev_in_ch;
                qI = pv.x;
                qQ = pv.y;
            }
            const float cI = aI[r + 1], cQ = aQ[r + 1];
            // demod.cpp:8-19 (numerator as the reference; fast mode only: f32 denominator and a
            // v_rcp_f32 quotient, a few f32 ulps from the reference's f64 division)
            const float num = cI * (cQ - qQ) - cQ * (cI - qI);
            const float den = cI * cI + cQ * cQ;
            const float q = num * __builtin_amdgcn_rcpf(den);
            v[r] = ((cI == 0.0f) & (cQ == 0.0f)) ? 0.0f : q;
            if (c == block_if - 1) prev_out[ch] = make_float2(cI, cQ);
        }
        if (cb >= lo && cb + 1 < hi && ((cb & 1) == 0)) {
            *reinterpret_cast<float2*>(out + cb) = make_float2(v[0], v[1]);
        } else {
#pragma unroll
            for (int r = 0; r < 2; r++)
                if (cb + r >= lo && cb + r < hi) out[cb + r] = v[r];
        }
    }
}

// The same wave tile with I and Q of one block in ONE lane (FT_IQLANE, NB a multiple of 16): a
// C tile is 16 blocks, columns = blocks, and the I and Q planes are two MFMA groups with the same A
// fragments, so lane t holds rows 4g..4g+3 of block 16*ct + (t & 15) for both components. The
// discriminator then needs no DPP exchange or component selects, each lane finishes 4 outputs, and
// one pair of shuffles per C tile brings the previous row (lane t-16, or row 15 of the previous block).
template <int D, int NB>
__device__ __forceinline__ void ft_tile_iq(const int8_t* __restrict__ lds, const v4i (&A)[FT_AFRAGS], double yscale,
                                           int c0, int ch, float2 prev_in_ch, float2* __restrict__ prev_out,
                                           int block_if, float* __restrict__ out) {
    static_assert(NB % 16 == 0, "whole 16-block C tiles");
    constexpr int WIN = ft_win(D, NB), ADV = ft_adv(D, NB), CARRY = ft_carry(D);
    const float ys = (float)yscale;
    const int t = threadIdx.x;
    const int n = t & 15, g = t >> 4;
    const int lo = max(c0 + CARRY, 0), hi = min(c0 + CARRY + ADV, block_if);
    // row 4g - 1 of this block (lane t - 16) or row 15 of the previous block (lane 48 + n - 1)
    const int src_lane = g > 0 ? t - 16 : (n > 0 ? t + 47 : t);
    float carry_i = 0.0f, carry_q = 0.0f;             // row 15 of the previous C tile's last block
#pragma unroll FT_CT_UNROLL
    for (int ct = 0; ct < NB / 16; ct++) {
        const int bb = 16 * ct + n;
        v4i aI[FT_ND], aQ[FT_ND];
#pragma unroll
        for (int p = 0; p < FT_ND; p++) { aI[p] = v4i{0, 0, 0, 0}; aQ[p] = v4i{0, 0, 0, 0}; }
#pragma unroll
        for (int kk = 0; kk < 4; kk++) {
            const int off = 16 * D * bb + 64 * kk + 16 * g;
            const v4i BI = *reinterpret_cast<const v4i*>(lds + off);
            const v4i BQ = *reinterpret_cast<const v4i*>(lds + WIN + off);
#pragma unroll
            for (int p = 0; p < FT_ND; p++) {
                aI[p] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A[FT_ND * kk + p], BI, aI[p], 0, 0, 0);
                aQ[p] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A[FT_ND * kk + p], BQ, aQ[p], 0, 0, 0);
            }
        }
        static_assert(FT_ND == 4, "pairwise recombination assumes 4 digit planes");
        float yI[4], yQ[4];
#pragma unroll
        for (int r = 0; r < 4; r++) {
            // digits pair up exactly in int32, then one fma in f32 (as ft_tile)
            const int hI = (aI[0][r] << 8) + aI[1][r], lI = (aI[2][r] << 8) + aI[3][r];
            const int hQ = (aQ[0][r] << 8) + aQ[1][r], lQ = (aQ[2][r] << 8) + aQ[3][r];
            yI[r] = __builtin_fmaf((float)hI, ys * 65536.0f, (float)lI * ys);
            yQ[r] = __builtin_fmaf((float)hQ, ys * 65536.0f, (float)lQ * ys);
        }
        const float sI = __shfl(yI[3], src_lane), sQ = __shfl(yQ[3], src_lane);
        const bool first = (t == 0);
        const float pI = first ? carry_i : sI, pQ = first ? carry_q : sQ;
        carry_i = __shfl(yI[3], 63);
        carry_q = __shfl(yQ[3], 63);
        const int cb = c0 + 16 * bb + 4 * g;          // output index of this lane's first row
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; r++) {
            const int c = cb + r;
            float qI = r == 0 ? pI : yI[r > 0 ? r - 1 : 0], qQ = r == 0 ? pQ : yQ[r > 0 ? r - 1 : 0];
            if (c == 0) {
                qI = prev_in_ch.x;
                qQ = prev_in_ch.y;
            }
            const float cI = yI[r], cQ = yQ[r];
            // demod.cpp:8-19 (fast mode: f32 denominator and a v_rcp_f32 quotient, as ft_tile)
            const float num = cI * (cQ - qQ) - cQ * (cI - qI);
            const float den = cI * cI + cQ * cQ;
            const float q = num * __builtin_amdgcn_rcpf(den);
            v[r] = ((cI == 0.0f) & (cQ == 0.0f)) ? 0.0f : q;
            if (c == block_if - 1) prev_out[ch] = make_float2(cI, cQ);
        }
        if (cb >= lo && cb + 3 < hi && ((cb & 1) == 0)) {
            *reinterpret_cast<float2*>(out + cb) = make_float2(v[0], v[1]);
            *reinterpret_cast<float2*>(out + cb + 2) = make_float2(v[2], v[3]);
        } else {
#pragma unroll
            for (int r = 0; r < 4; r++)
                if (cb + r >= lo && cb + r < hi) out[cb + r] = v[r];
        }
    }
}
#ifndef FT_IQLANE
#define FT_IQLANE 1   // I and Q of a block in one lane (ft_tile_iq) when NB is a multiple of 16
#endif
template <int D, int NB>
__device__ __forceinline__ void ft_tile_planar(const int8_t* __restrict__ lds, const v4i (&A)[FT_AFRAGS], double yscale,
                                               int c0, int ch, float2 prev_in_ch, float2* __restrict__ prev_out,
                                               int block_if, float* __restrict__ out) {
    if constexpr (FT_IQLANE && NB % 16 == 0)
        ft_tile_iq<D, NB>(lds, A, yscale, c0, ch, prev_in_ch, prev_out, block_if, out);
    else
        ft_tile<D, NB, false>(lds, A, yscale, c0, ch, prev_in_ch, prev_out, block_if, out);
}

template <int D, bool X4, int NB>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(4, 8))) void k_frontend_mfma(
    const uint8_t* __restrict__ iq, size_t iq_stride, const uint8_t* __restrict__ tail_in,
    uint8_t* __restrict__ tail_out, const float2* __restrict__ prev_in, float2* __restrict__ prev_out,
    const v4i* __restrict__ afrag, double yscale, int block_iq, int block_if,
    float* __restrict__ fm, const float* __restrict__ fm_other, size_t fm_stride, int tiles_ch,
    const uint32_t* __restrict__ pad) {
    static_assert(15 * D + 101 <= 256, "one block's window must fit K = 256");
    static_assert(NB % 8 == 0, "whole C tiles");
    constexpr int HP = 100, WIN = ft_win(D, NB), G = WIN / 8;
    constexpr int ADV = ft_adv(D, NB), CARRY = ft_carry(D);
    static_assert(CARRY >= 1 && CARRY + ADV <= 16 * NB && WIN % 8 == 0, "tile geometry");
    static_assert(((ADV * D) % 8) == 0 && (((-CARRY * D - HP) % 8) + 8) % 8 == 0, "m0 = 0 mod 8");
    __shared__ __attribute__((aligned(16))) int8_t plane[2][WIN];
    const int t = threadIdx.x;
    const int ch = blockIdx.x / tiles_ch;
    const int j = blockIdx.x - ch * tiles_ch;
    const uint8_t* src = iq + (size_t)ch * iq_stride;
    float* out = fm + (size_t)ch * fm_stride;
    const int c0 = j * ADV - CARRY;
    // ---- stage: groups of 8 I/Q pairs (16 bytes) -> 8 I bytes + 8 Q bytes, signed. All of a
    // lane's window loads are issued first (fully unrolled), then the taps' A fragments (constant,
    // L2-resident, lane-major: every load is 1 KiB contiguous).
    constexpr int GPL = (G + 63) / 64;                // groups per lane
    v4i A[FT_AFRAGS];
    {
        uint4 st[GPL];
        const int m0 = c0 * D - HP;                   // = 0 mod 8
        const uint2* g2 = reinterpret_cast<const uint2*>(src);
        const uint2* t2 = reinterpret_cast<const uint2*>(tail_in + (size_t)ch * 2 * HP);
        const uint2* p2 = reinterpret_cast<const uint2*>(pad);
        const bool interior = (m0 >= 0) && (m0 + WIN <= block_iq);
        if (interior && X4) {                         // 16-byte aligned rows: one dwordx4 per group
            typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
            const u32x4* gw = reinterpret_cast<const u32x4*>(src + 2 * m0);
#pragma unroll
            for (int k = 0; k < GPL; k++) {
                const int i = t + 64 * k;
                const u32x4 v = (k < GPL - 1 || i < G) ? __builtin_nontemporal_load(gw + i) : u32x4{0u, 0u, 0u, 0u};
                st[k] = uint4{v.x, v.y, v.z, v.w};
            }
        } else {                                      // 8-byte loads, each from the block, the tail or padding
#pragma unroll
            for (int k = 0; k < GPL; k++) {
                uint2 h[2];
#pragma unroll
                for (int hh = 0; hh < 2; hh++) {
                    const int mm = m0 + 8 * (t + 64 * k) + 4 * hh;
                    const uint2* pa = mm >= 0 ? (mm < block_iq ? g2 + (mm >> 2) : p2)
                                              : (mm >= -HP ? t2 + ((HP + mm) >> 2) : p2);
                    h[hh] = *pa;
                }
                st[k] = uint4{h[0].x, h[0].y, h[1].x, h[1].y};
            }
        }
        // taps after the window: in flight together, the window (older) is waited for first
#if FT_DIAG == 2
        // timing-only diagnosis (wrong results): constant A fragments, no tap loads
#pragma unroll
        for (int f = 0; f < FT_AFRAGS; f++) A[f] = v4i{f, t, 1, 2};
#else
#pragma unroll
        for (int f = 0; f < FT_AFRAGS; f++) A[f] = afrag[f * 64 + t];
#endif
        uint2* pi = reinterpret_cast<uint2*>(plane[0]);
        uint2* pq = reinterpret_cast<uint2*>(plane[1]);
#pragma unroll
        for (int k = 0; k < GPL; k++) {
            const int i = t + 64 * k;
            if (k < GPL - 1 || i < G) {
                const uint4 v = st[k];
                pi[i] = uint2{__builtin_amdgcn_perm(v.y, v.x, 0x06040200u) ^ 0x80808080u,
                              __builtin_amdgcn_perm(v.w, v.z, 0x06040200u) ^ 0x80808080u};
                pq[i] = uint2{__builtin_amdgcn_perm(v.y, v.x, 0x07050301u) ^ 0x80808080u,
                              __builtin_amdgcn_perm(v.w, v.z, 0x07050301u) ^ 0x80808080u};
            }
        }
    }
    __syncthreads();
#if FT_DIAG == 1
    // timing-only diagnosis (wrong results): staging and stores only, no MFMA / discriminator
    {
        const int lo = max(c0 + CARRY, 0), hi = min(c0 + CARRY + ADV, block_if);
        const int8_t v0 = plane[0][t];
        for (int c = lo + t; c < hi; c += 64) out[c] = (float)v0 + (float)A[0][0];
    }
#else
    ft_tile_planar<D, NB>(plane[0], A, yscale, c0, ch, prev_in[ch], prev_out, block_if, out);
#endif
    if (j == 0) {
        const uint16_t* last = reinterpret_cast<const uint16_t*>(src) + (block_iq - HP);
        uint16_t* tout = reinterpret_cast<uint16_t*>(tail_out + (size_t)ch * 2 * HP);
        for (int i = t; i < HP; i += 64) tout[i] = last[i];
        const float* o = fm_other + (size_t)ch * fm_stride;
        for (int i = t; i < HIST; i += 64) out[i - HIST] = o[block_if - HIST + i];
    }
}

// Persistent MFMA front end for 16-byte aligned rows: a grid of a few waves per CU (one wave per
// workgroup) walks tiles round-robin (tile = blockIdx.x + i*gridDim.x; a device-wide atomic queue
// saturates near 90 dequeues/us, far below the ~500 tiles/us needed), loads the taps' A fragments
// once, and keeps the NEXT tile's window in flight while it computes the current one: interior windows
// go HBM -> LDS by LDS-DMA (global_load_lds_dwordx4, no VGPRs) into the other of two LDS buffers,
// retired by a counted vmcnt; boundary tiles (the first of a channel reads the previous block's tail,
// the last runs into the padding) are staged synchronously with plain loads. The B fragments are
// read from the raw interleaved image (ft_tile<RAW>).
template <int D, int NB>
__global__ __launch_bounds__(64) void k_frontend_mfma_q(
    const uint8_t* __restrict__ iq, size_t iq_stride, const uint8_t* __restrict__ tail_in,
    uint8_t* __restrict__ tail_out, const float2* __restrict__ prev_in, float2* __restrict__ prev_out,
    const v4i* __restrict__ afrag, double yscale, int block_iq, int block_if,
    float* __restrict__ fm, const float* __restrict__ fm_other, size_t fm_stride, int tiles_ch, int total,
    const uint32_t* __restrict__ pad) {
    constexpr int HP = 100, WIN = ft_win(D, NB), RAWB = 2 * WIN;
    constexpr int ADV = ft_adv(D, NB), CARRY = ft_carry(D);
    constexpr int NGL = (RAWB + 1023) / 1024;          // LDS-DMA instructions per window (1 KiB each)
    constexpr int BUFB = NGL * 1024;
    static_assert(NGL <= 63, "vmcnt immediate (6 bits)");
    __shared__ __attribute__((aligned(16))) int8_t lds[2 * BUFB];
    const int t = threadIdx.x;
    v4i A[FT_AFRAGS];
#pragma unroll
    for (int f = 0; f < FT_AFRAGS; f++) A[f] = afrag[f * 64 + t];
    // window of tile tl starts at sample m0 = c0*D - 100 (= 0 mod 8); the DMA reads BUFB bytes
    auto m0_of = [&](int tl) { const int j = tl % tiles_ch; return (j * ADV - CARRY) * D - HP; };
    auto interior = [&](int tl) { const int m0 = m0_of(tl); return m0 >= 0 && 2 * m0 + BUFB <= 2 * block_iq; };
    auto issue = [&](int tl, int buf) {
        const uint8_t* g = iq + (size_t)(tl / tiles_ch) * iq_stride + 2 * (size_t)m0_of(tl) + 16 * t;
#pragma unroll
        for (int i = 0; i < NGL; i++)
            __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(g + 1024 * i),
                                             reinterpret_cast<__attribute__((address_space(3))) void*>(
                                                 reinterpret_cast<uintptr_t>(lds + buf * BUFB + 1024 * i)),
                                             16, 0, 0);
    };
    // boundary window: every 8-byte group (4 I/Q pairs) from the block, the previous block's tail or
    // the padding (u8 128 == 0.0f), plain loads -> ds_write
    auto stage_plain = [&](int tl, int buf) {
        const int ch = tl / tiles_ch, m0 = m0_of(tl);
        const uint2* g2 = reinterpret_cast<const uint2*>(iq + (size_t)ch * iq_stride);
        const uint2* t2 = reinterpret_cast<const uint2*>(tail_in + (size_t)ch * 2 * HP);
        const uint2* p2 = reinterpret_cast<const uint2*>(pad);
        uint2* d = reinterpret_cast<uint2*>(lds + buf * BUFB);
        for (int i = t; i < RAWB / 8; i += 64) {
            const int mm = m0 + 4 * i;
            const uint2* pa = mm >= 0 ? (mm < block_iq ? g2 + (mm >> 2) : p2) : (mm >= -HP ? t2 + ((HP + mm) >> 2) : p2);
            d[i] = *pa;
        }
    };
    const int G = gridDim.x;
    int cur = blockIdx.x, nxt = cur + G;
    if (cur < total) {
        if (interior(cur)) issue(cur, 0);
        else stage_plain(cur, 0);
    }
    int b = 0;
    while (cur < total) {
        const bool dma_next = nxt < total && interior(nxt);
        if (dma_next) issue(nxt, b ^ 1);
        // retire cur's window (everything but the NGL younger DMA of nxt; vector memory operations
        // retire in issue order, the previous tile's fm stores included) and the boundary ds_writes
        if (dma_next) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" :: "n"(NGL) : "memory");
        else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        const int ch = cur / tiles_ch, j = cur - ch * tiles_ch;
        float* out = fm + (size_t)ch * fm_stride;
        ft_tile<D, NB, true>(lds + b * BUFB, A, yscale, j * ADV - CARRY, ch, prev_in[ch], prev_out, block_if, out);
        if (j == 0) {
            const uint8_t* src = iq + (size_t)ch * iq_stride;
            const uint16_t* last = reinterpret_cast<const uint16_t*>(src) + (block_iq - HP);
            uint16_t* tout = reinterpret_cast<uint16_t*>(tail_out + (size_t)ch * 2 * HP);
            for (int i = t; i < HP; i += 64) tout[i] = last[i];
            const float* o = fm_other + (size_t)ch * fm_stride;
            for (int i = t; i < HIST; i += 64) out[i - HIST] = o[block_if - HIST + i];
        }
        // the other buffer is free: every wave passed this tile's barrier after finishing the previous
        // tile (one wave per workgroup, so the barrier only orders this wave's own LDS traffic)
        if (nxt < total && !dma_next) stage_plain(nxt, b ^ 1);
        cur = nxt;
        nxt += G;
        b ^= 1;
    }
}

// Persistent MFMA front end with register prefetch (SDR_FE_MFMA_WPE = waves per SIMD): a grid of
// 4*WPE one-wave workgroups per CU walks tiles round-robin (tile = blockIdx.x + i*gridDim.x). Each
// wave loads the taps' A fragments once (16 KiB per wave instead of per tile) and keeps the NEXT
// tile's window in flight in registers (the same 16-byte I/Q group loads as k_frontend_mfma) while
// the current tile computes out of its single LDS image, so one image per wave lets more waves
// fit than the two-buffer LDS-DMA kernel. 16-byte aligned rows only (the launcher checks).
template <int D, int NB, int WPE>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(WPE, WPE))) void k_frontend_mfma_p(
    const uint8_t* __restrict__ iq, size_t iq_stride, const uint8_t* __restrict__ tail_in,
    uint8_t* __restrict__ tail_out, const float2* __restrict__ prev_in, float2* __restrict__ prev_out,
    const v4i* __restrict__ afrag, double yscale, int block_iq, int block_if,
    float* __restrict__ fm, const float* __restrict__ fm_other, size_t fm_stride, int tiles_ch, int total,
    const uint32_t* __restrict__ pad) {
    static_assert(15 * D + 101 <= 256 && NB % 8 == 0, "tile geometry");
    constexpr int HP = 100, WIN = ft_win(D, NB), G = WIN / 8;
    constexpr int ADV = ft_adv(D, NB), CARRY = ft_carry(D);
    constexpr int GPL = (G + 63) / 64;                // 16-byte groups per lane
    __shared__ __attribute__((aligned(16))) int8_t plane[2][WIN];
    const int t = threadIdx.x;
    int cur = blockIdx.x;
    if (cur >= total) return;
    v4i A[FT_AFRAGS];
#pragma unroll
    for (int f = 0; f < FT_AFRAGS; f++) A[f] = afrag[f * 64 + t];
    uint4 st[GPL];
    // window of tile tl -> st (lane t holds groups t, t+64, ...): interior windows as one dwordx4
    // per group, boundary windows (previous block's tail, padding past the block) per 8 bytes
    auto fetch = [&](int tl) {
        const int ch = tl / tiles_ch, j = tl - ch * tiles_ch;
        const int m0 = (j * ADV - CARRY) * D - HP;    // = 0 mod 8
        const uint8_t* src = iq + (size_t)ch * iq_stride;
        if (m0 >= 0 && m0 + WIN <= block_iq) {
            typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
            const u32x4* gw = reinterpret_cast<const u32x4*>(src + 2 * m0);
#pragma unroll
            for (int k = 0; k < GPL; k++) {
                const int i = t + 64 * k;
                const u32x4 v = (k < GPL - 1 || i < G) ? __builtin_nontemporal_load(gw + i) : u32x4{0u, 0u, 0u, 0u};
                st[k] = uint4{v.x, v.y, v.z, v.w};
            }
        } else {
            const uint2* g2 = reinterpret_cast<const uint2*>(src);
            const uint2* t2 = reinterpret_cast<const uint2*>(tail_in + (size_t)ch * 2 * HP);
            const uint2* p2 = reinterpret_cast<const uint2*>(pad);
#pragma unroll
            for (int k = 0; k < GPL; k++) {
                uint2 h[2];
#pragma unroll
                for (int hh = 0; hh < 2; hh++) {
                    const int mm = m0 + 8 * (t + 64 * k) + 4 * hh;
                    const uint2* pa = mm >= 0 ? (mm < block_iq ? g2 + (mm >> 2) : p2)
                                              : (mm >= -HP ? t2 + ((HP + mm) >> 2) : p2);
                    h[hh] = *pa;
                }
                st[k] = uint4{h[0].x, h[0].y, h[1].x, h[1].y};
            }
        }
    };
    fetch(cur);
    while (true) {
        {   // st -> planar signed I and Q rows
            uint2* pi = reinterpret_cast<uint2*>(plane[0]);
            uint2* pq = reinterpret_cast<uint2*>(plane[1]);
#pragma unroll
            for (int k = 0; k < GPL; k++) {
                const int i = t + 64 * k;
                if (k < GPL - 1 || i < G) {
                    const uint4 v = st[k];
                    pi[i] = uint2{__builtin_amdgcn_perm(v.y, v.x, 0x06040200u) ^ 0x80808080u,
                                  __builtin_amdgcn_perm(v.w, v.z, 0x06040200u) ^ 0x80808080u};
                    pq[i] = uint2{__builtin_amdgcn_perm(v.y, v.x, 0x07050301u) ^ 0x80808080u,
                                  __builtin_amdgcn_perm(v.w, v.z, 0x07050301u) ^ 0x80808080u};
                }
            }
        }
        const int ch = cur / tiles_ch, j = cur - ch * tiles_ch;
        const float2 prev = prev_in[ch];              // before the prefetch: its wait must not cover it
        __syncthreads();
        const int nxt = cur + (int)gridDim.x;
        if (nxt < total) fetch(nxt);                  // in flight during this tile's MFMA and discriminator
        float* out = fm + (size_t)ch * fm_stride;
        ft_tile_planar<D, NB>(plane[0], A, yscale, j * ADV - CARRY, ch, prev, prev_out, block_if, out);
        if (j == 0) {
            const uint8_t* src = iq + (size_t)ch * iq_stride;
            const uint16_t* last = reinterpret_cast<const uint16_t*>(src) + (block_iq - HP);
            uint16_t* tout = reinterpret_cast<uint16_t*>(tail_out + (size_t)ch * 2 * HP);
            for (int i = t; i < HP; i += 64) tout[i] = last[i];
            const float* o = fm_other + (size_t)ch * fm_stride;
            for (int i = t; i < HIST; i += 64) out[i - HIST] = o[block_if - HIST + i];
        }
        if (nxt >= total) break;
        cur = nxt;
        __syncthreads();                              // the LDS image is rewritten next
    }
}

// Persistent front end: each 64-lane workgroup walks tiles (channel-major, stride gridDim.x).
// The next tile's u8 window is loaded into registers (coalesced dwords) while the current tile
// computes out of LDS, then written to LDS -- global latency overlaps the FIR instead of
// stalling every wave at its start. One tile = 64*R decimated outputs starting one before the
// first fm_demod sample it writes (the discriminator's carry, demod.cpp:16); tiles advance by
// 64*R-1. Boundary tiles (the first, which reads the previous block's tail, and the last, padded
// with u8 128 = 0.0f) take a bytewise path.
// PF: a persistent grid (SDR_FE_WG_PER_CU) that prefetches its next tile into registers during the
// FIR; without it (the default, one tile per workgroup) the window registers die once the window is
// in LDS, which leaves the FIR fewer VGPRs and the SIMD more waves.
template <int R, int D, bool FAST, bool PF>
__global__ __launch_bounds__(64) void k_frontend2(
    const uint8_t* __restrict__ iq, size_t iq_stride, const uint8_t* __restrict__ tail_in,
    uint8_t* __restrict__ tail_out, const float2* __restrict__ prev_in, float2* __restrict__ prev_out,
    const float* __restrict__ hs, int block_iq, int block_if,
    float* __restrict__ fm, const float* __restrict__ fm_other, size_t fm_stride, int nch, int tiles_ch,
    const uint32_t* __restrict__ pad) {
    constexpr int NT = 101, HP = NT - 1, NTH = 64;
    constexpr int TILE = NTH * R;
    constexpr int ADV = TILE - 1;
    constexpr int WIN = (TILE - 1) * D + NT;          // staged samples (u8 I/Q pairs)
    constexpr int TWIN = (R - 1) * D + NT;            // samples one thread reads
    constexpr int TCH = (2 * TWIN + 15) / 16;         // 16-byte LDS chunks per thread window
    constexpr int NG = (2 * WIN + 3) / 4;             // dwords of one tile window
    constexpr int PER = (NG + NTH - 1) / NTH;         // dwords per lane
    constexpr int LDS_BYTES = ((2 * WIN + 15) / 16) * 16 + 32;
    __shared__ __attribute__((aligned(16))) uint8_t sw[LDS_BYTES];
    const int t = threadIdx.x;
    const int total = nch * tiles_ch;
    int tile = blockIdx.x;
    if (tile >= total) return;
    uint32_t pf[PER];
    bool pf_ok = true;
    // window of tile `tl` -> pf (lane t holds dwords t, t+64, ...). Every I/Q sample is one u16;
    // samples before the block come from the previous block's tail, samples past its end are
    // u8 128 (== 0.0f). With D even the window starts on an even sample, so each dword is wholly
    // in the block, in the tail or in the padding: one load (or constant) per dword on every tile.
    auto fetch = [&](int tl) {
        const int ch = tl / tiles_ch, j = tl - ch * tiles_ch;
        const int m0 = (j * ADV - 1) * D - HP;
        pf_ok = true;
        const uint8_t* src = iq + (size_t)ch * iq_stride;
        const uint8_t* tin = tail_in + (size_t)ch * 2 * HP;
        if (D % 2 == 0) {
            static_assert(D % 2 != 0 || D + HP < 2 * NTH, "boundary fetch assumes the tail lies in k == 0");
            const uint32_t* g = reinterpret_cast<const uint32_t*>(src + 2 * m0);
            if (m0 >= 0 && m0 + WIN <= block_iq) {
#pragma unroll
                for (int k = 0; k < PER; k++) {
                    const int i = t + NTH * k;
                    pf[k] = (k < PER - 1 || i < NG) ? __builtin_nontemporal_load(g + i) : 0u;
                }
            } else {
                pf_ok = false;   // boundary tile: staged straight into LDS when its turn comes
            }
        } else {
            const uint16_t* s16 = reinterpret_cast<const uint16_t*>(src);
            const uint16_t* t16 = reinterpret_cast<const uint16_t*>(tin);
#pragma unroll
            for (int k = 0; k < PER; k++) {
                uint32_t v = 0;
#pragma unroll
                for (int h = 0; h < 2; h++) {
                    const int m = m0 + 2 * (t + NTH * k) + h;
                    const uint16_t* pa = m >= 0 ? s16 + m : t16 + (HP + m);
                    if (m < -HP || m >= block_iq) pa = reinterpret_cast<const uint16_t*>(pad);
                    const uint32_t pr = *pa;
                    v |= pr << (16 * h);
                }
                pf[k] = v;
            }
        }
    };
    fetch(tile);
    while (tile < total) {
        const int next = tile + (int)gridDim.x;
        const int ch = tile / tiles_ch, j = tile - ch * tiles_ch;
        const int c0 = j * ADV - 1;                   // first decimated output (the carry)
        {
            uint32_t* sd = reinterpret_cast<uint32_t*>(sw);
            if (pf_ok) {
#pragma unroll
                for (int k = 0; k < PER; k++) {
                    const int i = t + NTH * k;
                    if (k < PER - 1 || i < NG) sd[i] = pf[k];
                }
            } else {
                // boundary tile (D even): each dword lives wholly in the block, in the previous
                // block's tail or in the padding (u8 128 == 0.0f); the address is chosen per dword
                const int m0 = c0 * D - HP;
                const uint32_t* gs = reinterpret_cast<const uint32_t*>(iq + (size_t)ch * iq_stride);
                const uint32_t* gt = reinterpret_cast<const uint32_t*>(tail_in + (size_t)ch * 2 * HP);
                for (int i = t; i < NG; i += NTH) {
                    const int mm = m0 + 2 * i;
                    const uint32_t* pa = mm >= 0 ? (mm < block_iq ? gs + (mm >> 1) : pad)
                                                 : (mm >= -HP ? gt + ((HP + mm) >> 1) : pad);
                    sd[i] = *pa;
                }
            }
        }
        __syncthreads();
        if (PF && next < total) fetch(next);          // in flight during the FIR
        // ---- FIR: R outputs per thread, samples in descending order ----
        uint4 chunk[TCH];
        const uint4* tw = reinterpret_cast<const uint4*>(sw + 2 * t * R * D);
        chunk[TCH - 1] = tw[TCH - 1];
        if (TCH >= 2) chunk[TCH - 2] = tw[TCH - 2];
        f32x2 acc[R];
#pragma unroll
        for (int r = 0; r < R; r++) acc[r] = f32x2{0.0f, 0.0f};
        // Taps live in SGPRs: row S of the table holds the R taps sample S meets (uniform across
        // the wave), fetched with scalar loads FE_PF samples ahead into a rotating ring and fed to
        // the packed MACs as scalar operands (op_sel picks the half of the SGPR pair), so the VALU
        // gets its taps without LDS or VGPR traffic.
        // the tap pointer is made opaque per tile (otherwise every loop-invariant tap load is
        // hoisted out of the tile loop and the 8*TWIN taps overflow the SGPR file), then declared
        // uniform again with readfirstlane so the loads stay scalar
        int zero = 0;
        asm volatile("" : "+s"(zero));
        zero = __builtin_amdgcn_readfirstlane(zero);
        const double* hsd = reinterpret_cast<const double*>(hs) + zero;
        double ring[FE_PF][R / 2];
#pragma unroll
        for (int jj = 0; jj < FE_PF; jj++) {
            const int S0 = TWIN - 1 - jj;
#pragma unroll
            for (int q = 0; q < R / 2; q++) ring[S0 % FE_PF][q] = hsd[S0 * (R / 2) + q];
        }
        // sample S's (I, Q) as f32 (u8 - 128, exact) from the LDS chunk registers
        auto sample = [&](int S) -> f32x2 {
            const uint4 c4 = chunk[S >> 3];
            const int dw = (S & 7) >> 1;
            const uint32_t w = (dw == 0 ? c4.x : dw == 1 ? c4.y : dw == 2 ? c4.z : c4.w) ^ 0x80808080u;
            return (S & 1) ? fe_cvt_v<1>(w) : fe_cvt_v<0>(w);
        };
        // one sample of look-ahead: sample S-1 is converted while sample S's MACs issue, so no MAC
        // waits on its conversion
        f32x2 m_next = sample(TWIN - 1);
#pragma unroll
        for (int S = TWIN - 1; S >= 0; S--) {
            const int slot = S % FE_PF;
            if (((S & 7) == 7 || S == TWIN - 1) && (S >> 3) >= 2) chunk[(S >> 3) - 2] = tw[(S >> 3) - 2];
            const f32x2 m = m_next;
            if (FAST) {
                // the next sample's conversion sits in the middle of this sample's FMAs
#pragma unroll
                for (int r = 0; r < R; r++) {
                    const int k = r * D + HP - S;
                    if (k >= 0 && k < NT) acc[r] = fe_fma(ring[slot][r >> 1], r & 1, m, acc[r]);
                    if (r == R / 2 - 1 && S > 0) m_next = sample(S - 1);
                }
            } else {
                // all products of the sample first, then the adds, in program order (volatile asm):
                // no add waits on the product issued just before it
                f32x2 prod[R];
#pragma unroll
                for (int r = 0; r < R; r++) {
                    const int k = r * D + HP - S;
                    if (k >= 0 && k < NT) prod[r] = fe_mul_v(ring[slot][r >> 1], r & 1, m);
#if SDR_FE_CVT_MID
                    // the next sample's conversion between the products (an inline-asm result
                    // read right after it costs a wait state; here nothing reads it until S - 1)
                    if (r == R / 2 - 1 && S > 0) m_next = sample(S - 1);
#endif
                }
#if !SDR_FE_CVT_MID
                if (S > 0) m_next = sample(S - 1);
#endif
#pragma unroll
                for (int r = 0; r < R; r++) {
                    const int k = r * D + HP - S;
                    if (k >= 0 && k < NT) acc[r] = fe_add_v(acc[r], prod[r]);
                }
            }
            if (S - FE_PF >= 0) {
#pragma unroll
                for (int q = 0; q < R / 2; q++) ring[slot][q] = hsd[(S - FE_PF) * (R / 2) + q];
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        // ---- discriminator (demod.cpp:8-19); the previous output of lane t's first comes from t-1
        const f32x2 left = f32x2{__shfl_up(acc[R - 1].x, 1), __shfl_up(acc[R - 1].y, 1)};
        float* out = fm + (size_t)ch * fm_stride;
        const int cbase = c0 + t * R;
#pragma unroll
        for (int r = 0; r < R; r++) {
            const int c = cbase + r;
            f32x2 pv = (r > 0) ? acc[r > 0 ? r - 1 : 0] : left;
            if (c == 0) {
                const float2 p = prev_in[ch];
                pv = f32x2{p.x, p.y};
            }
            const f32x2 cur = acc[r];
            float v;
            if ((cur.x == 0) & (cur.y == 0)) {
                v = 0.0f;
            } else {
                const float num = cur.x * (cur.y - pv.y) - cur.y * (cur.x - pv.x);
                const double den = (double)cur.x * (double)cur.x + (double)cur.y * (double)cur.y;
                v = (float)((double)num / den);
            }
            if (c > c0 && c >= 0 && c < block_if) out[c] = v;
            if (c == block_if - 1) prev_out[ch] = make_float2(cur.x, cur.y);
        }
        if (j == 0) {
            const uint8_t* src = iq + (size_t)ch * iq_stride;
            const uint16_t* last = reinterpret_cast<const uint16_t*>(src) + (block_iq - HP);
            uint16_t* tout = reinterpret_cast<uint16_t*>(tail_out + (size_t)ch * 2 * HP);
            for (int i = t; i < HP; i += NTH) tout[i] = last[i];
            const float* o = fm_other + (size_t)ch * fm_stride;
            for (int i = t; i < HIST; i += NTH) out[i - HIST] = o[block_if - HIST + i];
        }
        if (!PF) break;                               // one tile per workgroup
        __syncthreads();                              // LDS is rewritten by the next tile
        tile = next;
    }
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
// from LDS (16-byte reads), the taps are wave-uniform scalar loads, and every output still sums
// h[k] * x[n-k] in ascending k as an f32 product then an f32 add (no contraction). NT = 2: two tap
// sets over one window (the stereo pilot and band filters).
// ------------------------------------------------------------------------------------------
constexpr int FRB_T = 101;                 // taps (rf_taps, project.cpp:61)
constexpr int FRB_R = 8;                   // outputs per thread
constexpr int FRB_TILE = BLK * FRB_R;      // outputs per workgroup
constexpr int FRB_W = FRB_TILE + FRB_T - 1 + 3;   // staged samples (+3: whole 16-byte reads)

template <int NT, bool SQUARE>
__global__ __launch_bounds__(BLK) void k_fir_rb(const float* __restrict__ x, size_t x_stride,
                                                const float* __restrict__ hist, size_t hist_stride,
                                                const float* __restrict__ h0, const float* __restrict__ h1, int ny,
                                                float* __restrict__ y0, float* __restrict__ y1, size_t y_stride,
                                                double* __restrict__ rx0, size_t rx_stride) {
    constexpr int T = FRB_T, R = FRB_R;
    __shared__ __attribute__((aligned(16))) float sx[(FRB_W + 3) & ~3];
    const int ch = blockIdx.y, tid = threadIdx.x;
    const int n0 = blockIdx.x * FRB_TILE;
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
    __syncthreads();
    const int nb = n0 + tid * R;
    if (nb >= ny) return;
    // w[i] = x[nb - (T-1) + i]; output nb + j at tap k reads w[j + T-1 - k] (samples past the
    // staged window only feed outputs >= ny, which are not stored)
    float w[R + T - 1 + 3];
#pragma unroll
    for (int i = 0; i < (R + T - 1 + 3) / 4; i++) {
        const float4 v = reinterpret_cast<const float4*>(sx + tid * R)[i];
        w[4 * i] = v.x; w[4 * i + 1] = v.y; w[4 * i + 2] = v.z; w[4 * i + 3] = v.w;
    }
    float a0[R], a1[R];
#pragma unroll
    for (int j = 0; j < R; j++) { a0[j] = 0.0f; a1[j] = 0.0f; }
#pragma unroll
    for (int k = 0; k < T; k++) {
        const float c0 = h0[k];
        const float c1 = (NT == 2) ? h1[k] : 0.0f;
#pragma unroll
        for (int j = 0; j < R; j++) {
            const float v = w[j + T - 1 - k];
            a0[j] = a0[j] + c0 * v;                               // filter.cpp:115
            if (NT == 2) a1[j] = a1[j] + c1 * v;
            // keep the MACs scalar: packed f32 ops run at half rate (tools/microbench/valu_rate.hip)
            // and pairing neighbouring outputs costs register realignment and occupancy
            if (NT == 1 && (j & 1) == 0) asm volatile("" : "+v"(a0[j]));
        }
    }
    float* o0 = y0 + (size_t)ch * y_stride + nb;
    float* o1 = (NT == 2) ? y1 + (size_t)ch * y_stride + nb : nullptr;
    if (nb + R <= ny) {
#pragma unroll
        for (int j = 0; j < R; j += 4) {
            reinterpret_cast<float4*>(o0 + j)[0] = make_float4(a0[j], a0[j + 1], a0[j + 2], a0[j + 3]);
            if (NT == 2) reinterpret_cast<float4*>(o1 + j)[0] = make_float4(a1[j], a1[j + 1], a1[j + 2], a1[j + 3]);
        }
    } else {
#pragma unroll
        for (int j = 0; j < R; j++) {
            if (nb + j < ny) {
                o0[j] = a0[j];
                if (NT == 2) o1[j] = a1[j];
            }
        }
    }
    if (rx0) {                                                    // y0 feeds a PLL: its reciprocal
        double* r = rx0 + (size_t)ch * rx_stride + nb;
        if (nb + R <= ny) {
#pragma unroll
            for (int j = 0; j < R; j += 2)
                reinterpret_cast<double2*>(r + j)[0] = make_double2(pllm::pll_rx(a0[j]), pllm::pll_rx(a0[j + 1]));
        } else {
#pragma unroll
            for (int j = 0; j < R; j++)
                if (nb + j < ny) r[j] = pllm::pll_rx(a0[j]);
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
constexpr int RLC_TN = 32;     // outputs per workgroup (8 per wave)
constexpr int RLC_XL = 3;      // staged samples per lane and row: 64 * 3 >= the q span + look-back
constexpr int RLC_HL = 2;      // staged taps per lane and polyphase row: 64 * 2 >= L4

template <int NTAP>   // > 0: every polyphase row has exactly NTAP taps (fully unrolled sums)
__global__ __launch_bounds__(BLK) void k_resample_lc(const float* __restrict__ x, size_t x_stride, int hist_lo,
                                                     const float* __restrict__ hp, const int* __restrict__ cnt,
                                                     int L, const int* __restrict__ ptq, int ny, int nch,
                                                     float* __restrict__ y, size_t y_stride) {
    extern __shared__ float4 smem4[];
    float* smem = reinterpret_cast<float*>(smem4);
    constexpr int PW = RLC_TN / (BLK / 64);                  // outputs per wave
    const int c0 = blockIdx.y * 64, n0 = blockIdx.x * RLC_TN;
    const int nn = min(RLC_TN, ny - n0);
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int qlo = (ptq[n0] >> 8) - (L - 1);
    const int W = (ptq[n0 + nn - 1] >> 8) - qlo + 1;
    const int SW = W | 1;
    const int L4 = (L + 3) & ~3;
    float* sx = smem;                                        // [64][SW]
    float* sh = smem + ((64 * SW + 3) & ~3);                 // [RLC_TN][L4]
    // staging with every load of a wave in flight before its LDS writes: rows c = wave + 4u of the
    // x tile (lanes along the row, RLC_XL loads per row), then the polyphase rows of the outputs
    {
        constexpr int NR = 64 / (BLK / 64);
        float v[NR][RLC_XL];
#pragma unroll
        for (int u = 0; u < NR; u++) {
            const int ch = min(c0 + wave + u * (BLK / 64), nch - 1);
            const float* xc = x + (size_t)ch * x_stride;
#pragma unroll
            for (int k = 0; k < RLC_XL; k++) {
                const int i = lane + 64 * k, m = qlo + i;
                v[u][k] = (i < W && m >= hist_lo) ? xc[m] : 0.0f;
            }
        }
#pragma unroll
        for (int u = 0; u < NR; u++) {
            const int c = wave + u * (BLK / 64);
#pragma unroll
            for (int k = 0; k < RLC_XL; k++) {
                const int i = lane + 64 * k;
                if (i < W) sx[c * SW + i] = v[u][k];
            }
        }
        float hv[PW][RLC_HL];
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
    __syncthreads();
    const int ch = c0 + lane;
    float out[PW];
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

size_t resample_lc_lds_bytes(int L, int U, int D) {
    const int W = resample_lc_span(L, U, D);
    return (size_t)((((64 * (W | 1)) + 3) & ~3) + RLC_TN * ((L + 3) & ~3)) * sizeof(float);
}

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
};
struct PllJobs {
    PllJob j[2];
};

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
    uint32_t split = 0u;
    uint32_t tie = ~0u;
    float tmax = 0.0f;
};
#ifndef SDR_PLL_HI_FIRST
#define SDR_PLL_HI_FIRST 1
#endif
#ifndef SDR_PLL_PREWAIT
#define SDR_PLL_PREWAIT 0
#endif
#ifndef SDR_PLL_LF_SCALAR
#define SDR_PLL_LF_SCALAR 1   // the plain f32 loop filter (no inline asm): +1.2 %, profiles/r02/ab_pll_lf.txt
#endif
#ifndef SDR_PLL_EDHI
#define SDR_PLL_EDHI 0
#endif
// |e| bound of the fast phase detector (the wrap to [-pi, pi] is the reference's below it)
constexpr double PLL_EMAX = SDR_PLL_EDHI ? pllm::PI - 0x1p-30 - 0x1p-42 : pllm::PI - 0x1p-30;
constexpr double PLL_TAB_WT_MAX = 0x1.6p29;   // |w * trigOffset| bound of the table path (above)

#ifndef SDR_PLL_COUNT
#define SDR_PLL_COUNT 0   // diagnosis build: count the fast chunks and the redone ones (sdr_diag_pll_counts)
#endif
#if SDR_PLL_COUNT
// [lane-chunks, lane-chunks that failed their proof, wave-chunks, wave-chunks redone]
__device__ unsigned long long g_pll_counts[4];
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
#if SDR_PLL_EDHI
    // the bracket ed -/+ eps as fma(Y, rx, base -/+ eps): base -/+ eps is ready before the input,
    // so the rounded e is one operation closer to Y (same proof: each end moves < 2^-50.5, far
    // inside eps - |error of ed|); |ed| <= |ed + eps| + 2^-43 for the range test
    const double ed = pllm::fma_(Y, rx, base + pllm::EPS_ABS_E2);
    const float lo = (float)pllm::fma_(Y, rx, base - pllm::EPS_ABS_E2), hi = (float)ed;
#else
    const double ed = pllm::fma_(Y, rx, base);
#if SDR_PLL_HI_FIRST
    // hi (the value used) first: the loop filter's packed product can issue while lo, the range
    // and the split test fill its hazard wait states
    const float hi = (float)(ed + pllm::EPS_ABS_E2);
    const float lo = (float)(ed - pllm::EPS_ABS_E2);
#else
    const float lo = (float)(ed - pllm::EPS_ABS_E2), hi = (float)(ed + pllm::EPS_ABS_E2);
#endif
#endif
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
    // pll.cpp:41-42: integ += Ki e; phaseEst = (phaseEst + Kp e) + integ, with the two products
    // and the two first sums as one v_pk_mul_f32 + one v_pk_add_f32 (the same f32 roundings)
#if SDR_PLL_LF_SCALAR
    // scalar f32: 5 VALU, and no hazard wait states after packed-f32 results
    {
        float ki_e = Ki * e;
        if (SDR_PLL_LF_SCALAR == 2) asm("" : "+v"(ki_e));      // keeps the SLP vectoriser from packing
        const float integ = r.ip.x + ki_e;
        r.ip.y = (r.ip.y + Kp * e) + integ;
        r.ip.x = integ;
    }
#else
    r.ip = r.ip + f32x2{Ki, Kp} * f32x2{e, e};
    float ph = r.ip.y;                                        // in place (else a pk_add + move)
    asm("v_add_f32 %0, %0, %1" : "+v"(ph) : "v"(r.ip.x));
    r.ip.y = ph;
#endif
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
#ifndef SDR_PLL_W01
#define SDR_PLL_W01 0
#endif
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
#if SDR_PLL_PREWAIT
        // the first buffers land before the loop (one memory latency per block). Otherwise the
        // compiler's wait counts at the loop header merge these loads' positions with the back
        // edge's and the steady-state loop waits for loads and stores it does not need: vmcnt(4)
        // before every refill (the previous chunk's refill) and vmcnt(12) inside every chunk (the
        // stores just issued), exposing a memory latency per chunk.
        __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0), expcnt and lgkmcnt unconstrained (gfx9)
#endif
    }
#if SDR_PLL_W01
    double2 w01 = TAB ? reinterpret_cast<const double2*>(wtab)[0] : double2{0.0, 0.0};
#endif
    for (int c0 = 0; c0 < nmain; c0 += NB) {
#pragma unroll
        for (int u = 0; u < NB; u++) {
            const int i0 = (c0 + u) * C;
            double wv[C];
            if (TAB) {
                // the first two steps' table entries were read at the end of the previous chunk
                // (w01), so the chunk's first steps do not wait on the LDS latency
#if SDR_PLL_W01
                wv[0] = w01.x; wv[1] = w01.y;
#pragma unroll
                for (int k = 1; k < C / 2; k++) {
#else
#pragma unroll
                for (int k = 0; k < C / 2; k++) {
#endif
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
#if SDR_PLL_DIAG_L2
            // diagnosis only (wrong results): every refill re-reads the first chunks (L2-resident),
            // to measure what the HBM latency of the refills costs
            load_chunk(xb[u], rb[u], u * C);
#else
            load_chunk(xb[u], rb[u], min(c0 + u + NB, nmain - 1) * C);
#endif
#if SDR_PLL_W01
            if (TAB) w01 = reinterpret_cast<const double2*>(wtab)[min(i0 + C, n - 2) >> 1];
#endif
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

// VEC: x / rx rows and the t buffer are 16-byte aligned with strides that are multiples of 4
// (x, t) and 2 (rx), so a chunk's inputs are prefetched with 16-byte loads and the 16 phases are
// stored with 16-byte stores -- the unrolled chunk itself touches no memory.
// Dynamic LDS: n doubles when the launch allows the trigArg table (launch_plls), else none.
template <bool VEC>
__global__ __launch_bounds__(64) void k_pll(const PllJobs jobs, int n, int nch, int tab_ok) {
    extern __shared__ double wtab[];
    const int ch = blockIdx.x * blockDim.x + threadIdx.x;   // lane 0 always holds a channel
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
    if (tab) pll_run<VEC, true>(jb, n, ch, wtab);
    else pll_run<VEC, false>(jb, n, ch, nullptr);
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
struct PllJobs2 {
    PllJobs p[2];
};
constexpr unsigned long long PLL_WAIT_TICKS = 500000000ull;   // 5 s of s_memrealtime

template <bool VEC>
__global__ __launch_bounds__(64) void k_pll_multi(const PllJobs2 jobs, int n, int nch, int tab_ok, int nblocks,
                                                  const uint32_t* pre_flag, uint32_t pre_first,
                                                  uint32_t* done_count, uint32_t* err,
                                                  unsigned long long* t_start, unsigned long long* t_end,
                                                  int sys_acquire) {
    extern __shared__ double wtab[];
    const int ch = blockIdx.x * blockDim.x + threadIdx.x;
    const bool active = ch < nch;
    __builtin_amdgcn_s_setprio(3);
    bool dead = false;
    for (int j = 0; j < nblocks; j++) {
        const PllJob& jb = jobs.p[j & 1].j[blockIdx.y];   // p[0]: the parity of the launch's first block
        if (!dead) {
            const uint32_t want = pre_first + (uint32_t)j + 1u;
            const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
            while ((int32_t)((sys_acquire ? __hip_atomic_load(pre_flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM)
                                          : __hip_atomic_load(pre_flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT)) -
                             want) < 0) {
                __builtin_amdgcn_s_sleep(4);
                if (__builtin_amdgcn_s_memrealtime() - t0 > PLL_WAIT_TICKS) {
                    dead = true;
                    break;
                }
            }
            if (dead && threadIdx.x == 0) __hip_atomic_fetch_or(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (!dead) {
            if (threadIdx.x == 0)
                __hip_atomic_fetch_min(t_start + j, (unsigned long long)__builtin_amdgcn_s_memrealtime(),
                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const double toff0 = active ? jb.st[ch].trigOffset : 0.0;
            const double w = 2 * 3.14159265358979323846 * (jb.freq / jb.Fs);
            const double toff_l0 = __shfl(toff0, 0);
            const bool tab = tab_ok && __all(!active || toff0 == toff_l0) &&
                             __builtin_fabs(w) * (__builtin_fabs(toff_l0) + (double)n + 1.0) < PLL_TAB_WT_MAX;
            if (tab) {
                for (int k = threadIdx.x; k < n; k += 64) wtab[k] = w * (toff_l0 + (double)(k + 1));   // pll.cpp:46-47
                __syncthreads();
            }
            if (active) {
                if (tab) pll_run<VEC, true>(jb, n, ch, wtab);
                else pll_run<VEC, false>(jb, n, ch, nullptr);
            }
            __syncthreads();   // every lane's table reads and state/phase stores issued before the release
        }
        if (threadIdx.x == 0) {
            if (!dead)
                __hip_atomic_fetch_max(t_end + j, (unsigned long long)__builtin_amdgcn_s_memrealtime(),
                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_fetch_add(done_count, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

// The two ends of the persistent PLLs' hand-offs, as one-wave kernels so that HIP's in-order
// kernel dispatch (each dispatch starts after the previous one in its stream has completed and
// released its writes) orders them: k_flag_store publishes "block ready" after the pre-PLL
// kernels of the front-end stream; k_flag_wait holds the post stream until the PLL waves have
// released a block (bounded, like the PLL's own waits).
__global__ void k_flag_store(uint32_t* flag, uint32_t v) {
    if (threadIdx.x == 0) __hip_atomic_store(flag, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
}
__global__ void k_flag_wait(const uint32_t* ctr, uint32_t want, uint32_t* err) {
    if (threadIdx.x != 0) return;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while ((int32_t)(__hip_atomic_load(ctr, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) - want) < 0) {
        __builtin_amdgcn_s_sleep(4);
        if (__builtin_amdgcn_s_memrealtime() - t0 > PLL_WAIT_TICKS) {
            __hip_atomic_fetch_or(err, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            break;
        }
    }
}

// pll_rx of a PLL input with no fused producer (the batched sdr_fmpll primitive)
__global__ __launch_bounds__(BLK) void k_pll_rx(double* __restrict__ rx, size_t rx_stride, const float* __restrict__ x,
                                                size_t x_stride, int n) {
    const int ch = blockIdx.y;
    const int i = blockIdx.x * BLK + threadIdx.x;
    if (i < n) rx[(size_t)ch * rx_stride + i] = pllm::pll_rx(x[(size_t)ch * x_stride + i]);
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

// copy the previous parity's last HIST samples in front of this parity's stream
__global__ void k_hist_copy(float* __restrict__ y, const float* __restrict__ y_other, size_t stride, int n) {
    const int ch = blockIdx.x;
    for (int i = threadIdx.x; i < HIST; i += blockDim.x)
        y[(size_t)ch * stride + i - HIST] = y_other[(size_t)ch * stride + n - HIST + i];
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
// first maximum wins, 0 when every sum is 0. One wave per channel, one lane per offset.
__device__ __forceinline__ int cdr_wave(const float* x, int n, int sps, int* sums) {
    const int lane = threadIdx.x;
    const int nk = n / sps;
    for (int i = lane; i < sps; i += blockDim.x) {
        uint32_t s = 0;
        for (int k = 0; k < nk; k++) {
            const int32_t v = cvt_i32_x86(x[k * sps + i]);
            s += (uint32_t)(v < 0 ? -(uint32_t)v : (uint32_t)v);
        }
        sums[i] = (int32_t)s;
    }
    __syncthreads();
    int maxi = 0, maxv = 0;
    for (int i = 0; i < sps; i++) {
        if (sums[i] > maxv) {
            maxv = sums[i];
            maxi = i;
        }
    }
    return maxi;
}

__global__ __launch_bounds__(64) void k_cdr(int32_t* __restrict__ offset, const float* __restrict__ x,
                                            size_t x_stride, int n, int sps) {
    extern __shared__ int sums_dyn[];
    const int ch = blockIdx.x;
    const int off = cdr_wave(x + (size_t)ch * x_stride, n, sps, sums_dyn);
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
                                                 size_t bits_stride) {
    extern __shared__ int sums_dyn[];
    __shared__ uint8_t symbols[SDR_MAX_SYMS];
    const int ch = blockIdx.x;
    const int lane = threadIdx.x;
    int32_t* d = dec + (size_t)ch * DEC_STATE;
    const int block_count = d[0];
    const float* xc = x + (size_t)ch * x_stride;
    const bool decode = (block_count > 5) && rds_on;
    if (!decode) {
        if (lane == 0) {
            if (offset_out) offset_out[ch] = d[4];
            if (nsym_out) nsym_out[ch] = 0;
            if (nbits_out) nbits_out[ch] = -1;
            d[0] = block_count + 1;
        }
        return;
    }
    const int off = cdr_wave(xc, n, sps, sums_dyn);
    int m = 0;
    if (off < n) m = (n - off + sps - 1) / sps;     // i with off + i*sps < n
    if (m > SDR_MAX_SYMS) m = SDR_MAX_SYMS;
    for (int i = lane; i < m; i += blockDim.x) symbols[i] = xc[off + i * sps] > 0;
    __syncthreads();
    if (lane == 0) {
        int half_symbol = d[1], start = d[2], last_bit = d[3];
        uint8_t bits[SDR_MAX_BITS];
        int nb = 0;
        if (start) bits[nb++] = (uint8_t)half_symbol;
        if (block_count == 0) {  // dead in the reference (decoding starts at block 6), kept for parity
            int score = 0;
            for (int i = 0; i < m - 1; i += 2) score += symbols[i] ^ symbols[i + 1];
            for (int j = 1; j < m - 1; j += 2) score -= symbols[j] ^ symbols[j + 1];
            start = score < 0;
        }
        for (int i = start; i < m - 1 && nb < SDR_MAX_BITS; i += 2) bits[nb++] = symbols[i];
        if (((m - start) & 0x01) == 1) {
            half_symbol = symbols[m - 1];
            start = 1;
        } else {
            start = 0;
        }
        uint8_t* bo = bits_out ? bits_out + (size_t)ch * bits_stride : nullptr;
        if (nb > 0) {
            uint8_t prevb = bits[0];
            const uint8_t first = (block_count == 0) ? bits[0] : (uint8_t)(bits[0] ^ (uint8_t)last_bit);
            if (bo) bo[0] = first;
            for (int i = 1; i < nb; i++) {
                if (bo) bo[i] = bits[i] ^ prevb;
                prevb = bits[i];
            }
            last_bit = bits[nb - 1];
        }
        if (sym_out) {
            uint8_t* so = sym_out + (size_t)ch * sym_stride;
            for (int i = 0; i < m; i++) so[i] = symbols[i];
        }
        d[1] = half_symbol;
        d[2] = start;
        d[3] = last_bit;
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

inline int cdiv(int a, int b) { return (a + b - 1) / b; }
inline size_t round_up(size_t a, size_t b) { return (a + b - 1) / b * b; }

size_t fir_lds_bytes(int ntaps, int nt, int tile, int D) {
    const int ntaps_pad = (ntaps + 3) & ~3;
    const int W = (tile - 1) * D + ntaps;
    return (size_t)(nt * ntaps_pad + W + 4) * sizeof(float);
}

size_t frontend_lds_bytes(int ntaps, int tile, int D) {
    const int ntaps_pad = (ntaps + 3) & ~3;
    const int W = tile * D + ntaps;                  // window incl. the extra output at n0-1
    return (size_t)ntaps_pad * 4 + (size_t)((W + 1) & ~1) * 8 + (size_t)(tile + 1) * 8 + 64;
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

// PLL + NCO output: k_pll (fast, default) or k_pll_libm (SDR_FLAG_PLL_LIBM / env SDR_PLL=libm)
bool pll_libm_env() {
    static const bool v = [] {
        const char* e = std::getenv("SDR_PLL");
        return e && std::strcmp(e, "libm") == 0;
    }();
    return v;
}

// SDR_PLL_TAB=0: per-lane trigArg offsets (A/B of the LDS table)
bool pll_notab_env() {
    static const bool v = [] {
        const char* e = std::getenv("SDR_PLL_TAB");
        return e && std::strcmp(e, "0") == 0;
    }();
    return v;
}

int launch_nco(const PllJobs& jobs, int njobs, int n, int nch, hipStream_t s) {
    if (n > 0) {
        hipLaunchKernelGGL(k_nco_out, dim3(cdiv(n, BLK), nch, njobs), dim3(BLK), 0, s, jobs, n);
        LAUNCH_CHECK();
    }
    return SDR_OK;
}

int launch_plls(bool libm, const PllJobs& jobs, int njobs, int n, int nch, hipStream_t s, bool with_nco = true) {
    const dim3 g(cdiv(nch, 64), njobs), b(64);
    bool vec = true;
    for (int k = 0; k < njobs; k++) {
        const PllJob& j = jobs.j[k];
        vec = vec && (reinterpret_cast<uintptr_t>(j.in) % 16 == 0) && (j.in_stride % 4 == 0) &&
              (reinterpret_cast<uintptr_t>(j.tbuf) % 16 == 0) && (j.t_stride % 4 == 0) &&
              (reinterpret_cast<uintptr_t>(j.rx) % 16 == 0) && (j.rx_stride % 2 == 0);
    }
    // LDS table of w * trigOffset (k_pll): n doubles, 16-byte rows
    const size_t tab_bytes = round_up((size_t)std::max(n, 1), 2) * sizeof(double);
    const int tab_ok = (tab_bytes <= 64 * 1024 && !pll_notab_env()) ? 1 : 0;
    const size_t lds = tab_ok ? tab_bytes : 0;
    if (libm || pll_libm_env()) {
        hipLaunchKernelGGL(k_pll_libm, g, b, 0, s, jobs, n, nch);
    } else if (vec) {
        hipLaunchKernelGGL(k_pll<true>, g, b, lds, s, jobs, n, nch, tab_ok);
    } else {
        hipLaunchKernelGGL(k_pll<false>, g, b, lds, s, jobs, n, nch, tab_ok);
    }
    LAUNCH_CHECK();
    return with_nco ? launch_nco(jobs, njobs, n, nch, s) : SDR_OK;
}

int launch_pll(bool libm, const float* in, size_t in_stride, int n, int nch, float freq, float Fs, float* tbuf,
               size_t t_stride, double* rxbuf, float* out, size_t out_stride, sdr_pll_state* st, float ncoScale,
               float phaseAdjust, float bw, hipStream_t s) {
    if (n > 0) {
        hipLaunchKernelGGL(k_pll_rx, dim3(cdiv(n, BLK), nch), dim3(BLK), 0, s, rxbuf, t_stride, in, in_stride, n);
        LAUNCH_CHECK();
    }
    PllJobs jobs{};
    jobs.j[0] = PllJob{in, in_stride, tbuf, t_stride, out, out_stride, st, freq, Fs, bw, ncoScale, phaseAdjust, nullptr,
                       rxbuf, t_stride};
    return launch_plls(libm, jobs, 1, n, nch, s);
}


}  // namespace

// ============================================================================================
// Context
// ============================================================================================
struct sdr_ctx {
    int device = 0, nch = 0, mode = 0, rds_on = 0, flags = 0;
    sdr_info info{};
    int ntaps = 101;
    // taps (device)
    float *rf_h = nullptr, *rf_hs = nullptr, *pilot_h = nullptr, *stereo_h = nullptr, *rds_h = nullptr, *rds_sq_h = nullptr,
          *rrc_h = nullptr;
    float *audio_pp = nullptr, *rdsbb_pp = nullptr;   // polyphase tables
    int *audio_cnt = nullptr, *rdsbb_cnt = nullptr;
    int audio_L = 0, rdsbb_L = 0;
    // extended streams [2][nch][HIST + len]; pointers below are the data bases of parity 0
    float *fm = nullptr, *sdc = nullptr, *rband = nullptr, *rdc = nullptr, *rfilt = nullptr;
    size_t fm_stride = 0, rf_stride = 0;               // per-channel strides (if, rds lengths)
    size_t fm_par = 0, rf_par = 0;                      // parity offsets in elements
    // plain per-block buffers
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
    int fe_grid = 0;                                    // front-end workgroups (0: one per tile)
    int fe_r = 8;                                       // front-end outputs per lane (4 or 8)
    uint32_t* pad80 = nullptr;                          // 64 words of u8 128 (the zero sample)
    void* fe_afrag = nullptr;                           // MFMA front end: tap digit fragments
    double fe_yscale = 0.0;                             // 2^-(F+7): fixed-point taps, x = (u-128)/128
    bool fe_mfma = false;                               // fast mode runs k_frontend_mfma
    int fe_nb = FT_NB_DEFAULT;                          // MFMA front end: 16-output blocks per tile
    int fe_wpe = 0;                                     // > 0: persistent register-prefetch MFMA front end
    int cus = 0;                                        // compute units of the device
    int parity = 1;                                     // parity of the current block
    long long block = -1;                               // index of the current block
    long long stereo_done = -1, rds_dsp_done = -1, rds_bits_done = -1, mono_done = -1;
    long long st_pre_done = -1, st_pll_done = -1, rds_pre_done = -1, rds_pll_done = -1;
    // persistent PLLs (sdr_plls_launch / _signal / _wait): device words [pre_flag, done_count,
    // err], per-block timestamps of the last launch, and the host's sequence bookkeeping
    uint32_t* pers_words = nullptr;
    unsigned long long *pers_t0 = nullptr, *pers_t1 = nullptr;
    int pers_tcap = 0, pers_last_n = 0;
    uint32_t pers_launched = 0, pers_signaled = 0, pers_waves = 0;
    long long pers_block = -1;                          // block of the last signal
    uint32_t pers_block_seq = 0;                        // its sequence number
    std::vector<void*> allocs;

    float* fm_cur() const { return fm + parity * fm_par; }
    float* fm_oth() const { return fm + (parity ^ 1) * fm_par; }
    float* ext(float* base, size_t par, int p) const { return base + p * par; }
    float* plain(float* base) const { return base + parity * plain_par; }
    float* pllbuf(float* base) const { return base + parity * pll_par; }
    double* rxbuf(double* base) const { return base + parity * plain_par; }
};

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
                  c->carrier + (c->parity ^ 1) * c->pll_par, c->rxbuf(c->rx_st), c->plain_stride};
}
PllJob rds_job(sdr_ctx* c) {      // rds.cpp:119: fmpll(gen_pilot, 114e3, if_Fs, ..., 0.5, 0, 0.001)
    const sdr_info& in = c->info;
    return PllJob{c->plain(c->gpilot), c->plain_stride, c->plain(c->t_rds), c->plain_stride, c->pllbuf(c->ipll),
                  c->pll_stride, c->rds_pll, 114e3f, (float)in.if_Fs, 0.001f, 0.5f, 0.0f,
                  c->ipll + (c->parity ^ 1) * c->pll_par, c->rxbuf(c->rx_rds), c->plain_stride};
}

}  // namespace

namespace {
// Scratch of the context-free PLL primitive (input reciprocals [nch][ts] f64 + phases [nch][ts]
// f32): one buffer per (device, stream), reused in that stream's order and grown on demand, so
// sdr_fmpll enqueues without synchronising. SDR_FMPLL_SCRATCH selects the older variants for the
// diagnosis in DESIGN.md (tools/diag_fmpll_scratch.py): "sync" (hipMalloc, synchronise, hipFree),
// "async" (two hipMallocAsync / hipFreeAsync pairs on the default pool).
struct StreamScratch {
    hipStream_t s;
    int dev;
    void* p;
    size_t bytes;
};
std::mutex g_scratch_mu;
std::vector<StreamScratch> g_scratch;

int stream_scratch(hipStream_t s, size_t bytes, void** out) {
    int dev = 0;
    HIP_TRY(hipGetDevice(&dev));
    std::lock_guard<std::mutex> lk(g_scratch_mu);
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

int fmpll_scratch_mode() {
    static const int v = [] {
        const char* e = std::getenv("SDR_FMPLL_SCRATCH");
        if (e && std::strcmp(e, "sync") == 0) return 1;
        if (e && std::strcmp(e, "async") == 0) return 2;
        if (e && std::strcmp(e, "async_leak") == 0) return 3;      // hipMallocAsync, never freed
        if (e && std::strcmp(e, "async_syncalloc") == 0) return 4; // hipMallocAsync + synchronise, then launch
        return 0;
    }();
    return v;
}

}  // namespace

extern "C" {

const char* sdr_last_error(void) { return g_err.c_str(); }
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
    std::vector<uint32_t> mask((ncu + 31) / 32, 0u);
    for (int cu = 0; cu < ncu; ++cu) {
        const bool in = cu >= first_cu && cu < first_cu + n_cu;
        if (in != (exclude != 0)) mask[cu / 32] |= 1u << (cu % 32);
    }
    hipStream_t s = nullptr;
    HIP_TRY(hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()));
    *stream = s;
    return SDR_OK;
}

int sdr_stream_destroy(void* stream) {
    if (!stream) return fail(SDR_E_INVALID, "sdr_stream_destroy: stream is NULL");
    const int rc = release_stream_scratch((hipStream_t)stream);
    if (rc != SDR_OK) return rc;
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

// Diagnosis builds only (-DSDR_PLL_COUNT=1): the PLL chunk counters [lane-chunks, failed lane-chunks,
// wave-chunks, redone wave-chunks], optionally reset; -1 in product builds. Not part of sdr_amd.h.
extern "C" int sdr_diag_pll_counts(unsigned long long* out, int reset) {
#if SDR_PLL_COUNT
    HIP_TRY(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_pll_counts), sizeof(unsigned long long) * 4));
    if (reset) {
        const unsigned long long z[4] = {0, 0, 0, 0};
        HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(g_pll_counts), z, sizeof z));
    }
    return SDR_OK;
#else
    (void)out;
    (void)reset;
    return -1;
#endif
}

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
        // One tile per workgroup by default: measured as fast as a persistent grid in isolation and
        // 2.5x faster while the other streams' kernels share the chip (the dispatcher balances).
        int cus = 0;
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device);
        c->cus = cus;
        if (const char* e = std::getenv("SDR_FE_MFMA_WPE")) {    // tuning knob: persistent MFMA, waves per SIMD
            const int k = std::atoi(e);
            if (k >= 2 && k <= 4) c->fe_wpe = k;
        }
        if (const char* e = std::getenv("SDR_FE_WG_PER_CU")) {   // tuning knob: persistent grid, k per CU
            const int k = std::atoi(e);
            if (k >= 0 && cus > 0) c->fe_grid = k * cus;
        }
        if (const char* e = std::getenv("SDR_FE_R")) {           // tuning knob: outputs per lane
            const int k = std::atoi(e);
            if (k == 4 || k == 8) c->fe_r = k;
        }
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
        // front-end v2 tap table: row S (input sample S of a thread window, R = 8 outputs) holds
        // h[r*D + 100 - S] / 128 (exact power-of-two scaling) or 0 where that tap does not exist
        const int R = c->fe_r, D = in.rf_decim, TWIN = (R - 1) * D + T;
        std::vector<float> tt((size_t)TWIN * R, 0.0f);
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
        c->fe_mfma = std::getenv("SDR_FE_FAST_VALU") == nullptr;   // A/B knob: packed-FMA VALU path
        if (const char* e = std::getenv("SDR_FE_NB")) c->fe_nb = std::atoi(e);   // tuning knob: 16, 24, 32
    }
    TRY(upload(c, &c->pilot_h, pilot));
    TRY(upload(c, &c->stereo_h, stereo));
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
    TRY(init_state(c, nullptr));
#undef TRY
    *out = c;
    return SDR_OK;
}

int sdr_ctx_destroy(sdr_ctx* c) {
    if (!c) return SDR_OK;
    (void)hipSetDevice(c->device);
    for (void* p : c->allocs) (void)hipFree(p);
    delete c;
    return SDR_OK;
}

int sdr_ctx_reset(sdr_ctx* c, void* stream) {
    if (!c) return fail(SDR_E_INVALID, "null context");
    HIP_TRY(hipSetDevice(c->device));
    return init_state(c, S(stream));
}

int sdr_ctx_info(const sdr_ctx* c, sdr_info* info) {
    if (!c || !info) return fail(SDR_E_INVALID, "null argument");
    *info = c->info;
    return SDR_OK;
}

int sdr_frontend(sdr_ctx* c, const uint8_t* iq, size_t iq_stride, void* stream) {
    if (!c || !iq) return fail(SDR_E_INVALID, "null argument");
    const sdr_info& in = c->info;
    if (iq_stride < (size_t)2 * in.block_iq || (iq_stride & 1) || (reinterpret_cast<uintptr_t>(iq) & 1))
        return fail(SDR_E_INVALID, "iq_stride %zu < 2*block_iq %d or misaligned", iq_stride, 2 * in.block_iq);
    const int p = c->parity ^ 1;
    const int hp = c->ntaps - 1;
    uint8_t* tail_in = c->tail + (size_t)(p ^ 1) * c->nch * 2 * hp;
    uint8_t* tail_out = c->tail + (size_t)p * c->nch * 2 * hp;
    const float2* prev_in = c->prev + (size_t)(p ^ 1) * c->nch;
    float2* prev_out = c->prev + (size_t)p * c->nch;
    const bool fast = (c->flags & SDR_FLAG_FAST_FRONTEND) != 0;
    float* fm_p = c->fm + p * c->fm_par;
    const float* fm_o = c->fm + (p ^ 1) * c->fm_par;
    const int R = c->fe_r;
    const int tiles_ch = cdiv(in.block_if + 1, 64 * R - 1);
    const int total = tiles_ch * c->nch;
    // fe_grid == 0: one tile per workgroup (the hardware dispatcher balances the load when other
    // streams share the chip); otherwise a persistent grid that prefetches its next tile
    const dim3 g2(c->fe_grid > 0 ? std::min(total, c->fe_grid) : total);
#define FE2P(RR, DD, FF, PP)                                                                                 \
    hipLaunchKernelGGL((k_frontend2<RR, DD, FF, PP>), g2, dim3(64), 0, S(stream), iq, iq_stride, tail_in,        \
                       tail_out, prev_in, prev_out, c->rf_hs, in.block_iq, in.block_if, fm_p, fm_o, c->fm_stride,  \
                       c->nch, tiles_ch, c->pad80)
#define FE2(RR, DD, FF) do { if (c->fe_grid > 0) FE2P(RR, DD, FF, true); else FE2P(RR, DD, FF, false); } while (0)
#define FE2R(DD)                                                                                             \
    do {                                                                                                     \
        if (R == 8) { if (fast) FE2(8, DD, true); else FE2(8, DD, false); }                                  \
        else { if (fast) FE2(4, DD, true); else FE2(4, DD, false); }                                         \
    } while (0)
    if (fast && c->fe_mfma) {
        const v4i* af = static_cast<const v4i*>(c->fe_afrag);
        // 16-byte I/Q group loads need 16-byte aligned rows (e.g. a row stride of 147008 for mode 0)
        const bool x4 = (iq_stride % 16 == 0) && (reinterpret_cast<uintptr_t>(iq) % 16 == 0);
#define FEMP(DD, NB, W)                                                                                      \
    hipLaunchKernelGGL((k_frontend_mfma_p<DD, (NB == 16 ? 16 : 32), W>), gp, dim3(64), 0, S(stream), iq, iq_stride, \
                       tail_in, tail_out, prev_in, prev_out, af, c->fe_yscale, in.block_iq, in.block_if, fm_p,     \
                       fm_o, c->fm_stride, tc, tc * c->nch, c->pad80)
#define FEM(DD, XX, NB)                                                                                      \
    do {                                                                                                     \
        const int tc = cdiv(in.block_if, ft_adv(DD, NB));                                                    \
        if (XX && c->fe_wpe > 0 && (NB == 16 || NB == 32)) {                                                 \
            const int g = c->fe_grid > 0 ? c->fe_grid : 4 * c->fe_wpe * c->cus;                              \
            const dim3 gp(std::min(tc * c->nch, g));                                                         \
            if (c->fe_wpe == 2) FEMP(DD, NB, 2); else if (c->fe_wpe == 4) FEMP(DD, NB, 4); else FEMP(DD, NB, 3); \
        } else if (XX && c->fe_grid > 0) {                                                                   \
            hipLaunchKernelGGL((k_frontend_mfma_q<DD, NB>), dim3(std::min(tc * c->nch, c->fe_grid)), dim3(64), \
                               0, S(stream), iq, iq_stride, tail_in, tail_out, prev_in, prev_out, af,        \
                               c->fe_yscale, in.block_iq, in.block_if, fm_p, fm_o, c->fm_stride, tc,          \
                               tc * c->nch, c->pad80);                                                       \
        } else {                                                                                             \
            hipLaunchKernelGGL((k_frontend_mfma<DD, XX, NB>), dim3(tc * c->nch), dim3(64), 0,                \
                               S(stream), iq, iq_stride,                                                     \
                               tail_in, tail_out, prev_in, prev_out, af, c->fe_yscale, in.block_iq, in.block_if, \
                               fm_p, fm_o, c->fm_stride, tc, c->pad80);                                      \
        }                                                                                                    \
    } while (0)
#define FEMN(DD, XX) do { if (c->fe_nb == 16) FEM(DD, XX, 16); else if (c->fe_nb == 24) FEM(DD, XX, 24); \
                             else if (c->fe_nb == 48) FEM(DD, XX, 48); else if (c->fe_nb == 64) FEM(DD, XX, 64); \
                             else FEM(DD, XX, 32); } while (0)
        if (in.rf_decim == 10) { if (x4) FEMN(10, true); else FEMN(10, false); }
        else if (in.rf_decim == 4) { if (x4) FEMN(4, true); else FEMN(4, false); }
        else { if (x4) FEMN(3, true); else FEMN(3, false); }
#undef FEMN
#undef FEM
#undef FEMP
    } else if (c->ntaps == 101 && in.rf_decim == 10) {
        FE2R(10);
    } else if (c->ntaps == 101 && in.rf_decim == 4) {
        FE2R(4);
    } else if (c->ntaps == 101 && in.rf_decim == 3) {
        FE2R(3);
    } else {
        const int tile = FIR_TILE;
        dim3 grid(cdiv(in.block_if, tile), c->nch);
        const size_t lds = frontend_lds_bytes(c->ntaps, tile, in.rf_decim);
        hipLaunchKernelGGL(k_frontend, grid, dim3(BLK), lds, S(stream), iq, iq_stride, tail_in, tail_out, prev_in,
                           prev_out, c->rf_h, c->ntaps, in.rf_decim, in.block_iq, in.block_if, tile, fm_p, fm_o,
                           c->fm_stride);
    }
#undef FE2R
#undef FE2
#undef FE2P
    LAUNCH_CHECK();
    c->parity = p;
    c->block++;
    return SDR_OK;
}

int sdr_get_fm_demod(sdr_ctx* c, float* fm, size_t fm_stride, void* stream) {
    if (!c || !fm) return fail(SDR_E_INVALID, "null argument");
    if (c->block < 0) return fail(SDR_E_INVALID, "no block processed yet");
    const sdr_info& in = c->info;
    HIP_TRY(hipMemcpy2DAsync(fm, fm_stride * sizeof(float), c->fm_cur(), c->fm_stride * sizeof(float),
                             in.block_if * sizeof(float), c->nch, hipMemcpyDeviceToDevice, S(stream)));
    return SDR_OK;
}

int sdr_mono(sdr_ctx* c, int16_t* audio, size_t audio_stride, void* stream) {
    if (!c || !audio) return fail(SDR_E_INVALID, "null argument");
    if (c->block < 0 || c->mono_done == c->block) return fail(SDR_E_INVALID, "mono: no new block");
    const sdr_info& in = c->info;
    const int tile = 512;
    dim3 grid(cdiv(in.n_audio, tile), c->nch);
    const size_t lds = resample_lds_bytes(c->audio_L, in.audio_upsample, in.audio_decim, tile, 1);
    const float* fm = c->fm_cur();
    auto km = c->audio_u1_101 ? k_resample<1, 101> : k_resample<1, 0>;
    hipLaunchKernelGGL(km, grid, dim3(BLK), lds, S(stream), fm, fm, c->fm_stride, c->fm_stride,
                       nullptr, nullptr, (size_t)0, (size_t)0, c->audio_pp, c->audio_cnt, c->audio_L,
                       in.audio_upsample, in.audio_decim, in.n_audio, tile, -HIST, (void*)audio, audio_stride);
    LAUNCH_CHECK();
    c->mono_done = c->block;
    return SDR_OK;
}

// The stereo and RDS loop bodies split at their PLL (pre: FIRs feeding the PLL; pll: the serial
// recurrence; post: everything after it), so a caller can run the PLL of block b on its own stream
// back to back with block b+1's while other streams do the rest. Intermediates that cross the
// split are kept per block parity. sdr_stereo / sdr_rds_dsp run the three parts on one stream.
int sdr_stereo_pre(sdr_ctx* c, void* stream) {
    if (!c) return fail(SDR_E_INVALID, "null context");
    if (c->block < 0 || c->st_pre_done == c->block) return fail(SDR_E_INVALID, "stereo_pre: no new block");
    const sdr_info& in = c->info;
    const int n = in.block_if, T = c->ntaps;
    const float* fm = c->fm_cur();
    // pilot BPF (stereo.cpp:74) + band BPF (:80) from one staged window of fm_demod
    if (T != FRB_T) return fail(SDR_E_INVALID, "stereo_pre: %d taps", T);
    dim3 gf(cdiv(n, FRB_TILE), c->nch);
    hipLaunchKernelGGL((k_fir_rb<2, false>), gf, dim3(BLK), 0, S(stream), fm, c->fm_stride, fm, c->fm_stride,
                       c->pilot_h, c->stereo_h, n, c->plain(c->pilot), c->plain(c->band), c->plain_stride,
                       c->rxbuf(c->rx_st), c->plain_stride);
    LAUNCH_CHECK();
    c->st_pre_done = c->block;
    return SDR_OK;
}

int sdr_stereo_pll(sdr_ctx* c, void* stream) {
    if (!c) return fail(SDR_E_INVALID, "null context");
    if (c->st_pre_done != c->block || c->st_pll_done == c->block)
        return fail(SDR_E_INVALID, "stereo_pll: run sdr_stereo_pre on a new block first");
    PllJobs jobs{};
    jobs.j[0] = stereo_job(c);   // PLL 19 kHz -> 38 kHz carrier (stereo.cpp:77); NCO output: stereo_post
    const int r = launch_plls(c->flags & SDR_FLAG_PLL_LIBM, jobs, 1, c->info.block_if, c->nch, S(stream), false);
    if (r) return r;
    c->st_pll_done = c->block;
    return SDR_OK;
}

int sdr_stereo_post(sdr_ctx* c, int16_t* lr, size_t lr_stride, void* stream) {
    if (!c || !lr) return fail(SDR_E_INVALID, "null argument");
    if (c->st_pll_done != c->block || c->stereo_done == c->block)
        return fail(SDR_E_INVALID, "stereo_post: run sdr_stereo_pll on a new block first");
    const sdr_info& in = c->info;
    hipStream_t s = S(stream);
    const int n = in.block_if;
    const float* fm = c->fm_cur();
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
    c->stereo_done = c->block;
    return SDR_OK;
}

int sdr_stereo(sdr_ctx* c, int16_t* lr, size_t lr_stride, void* stream) {
    if (!c || !lr) return fail(SDR_E_INVALID, "null argument");
    if (c->block < 0 || c->stereo_done == c->block) return fail(SDR_E_INVALID, "stereo: no new block");
    int r = sdr_stereo_pre(c, stream);
    if (!r) r = sdr_stereo_pll(c, stream);
    if (!r) r = sdr_stereo_post(c, lr, lr_stride, stream);
    return r;
}

int sdr_rds_pre(sdr_ctx* c, void* stream) {
    if (!c) return fail(SDR_E_INVALID, "null context");
    if (c->block < 0 || c->rds_pre_done == c->block) return fail(SDR_E_INVALID, "rds_pre: no new block");
    const sdr_info& in = c->info;
    hipStream_t s = S(stream);
    const int n = in.block_if, T = c->ntaps, p = c->parity;
    const float* fm = c->fm_cur();
    float* rband = c->rband + p * c->fm_par;
    if (T != FRB_T) return fail(SDR_E_INVALID, "rds_pre: %d taps", T);
    dim3 gf(cdiv(n, FRB_TILE), c->nch);
    // RDS band BPF (rds.cpp:105) into the extended rds_band stream
    hipLaunchKernelGGL(k_hist_copy, dim3(c->nch), dim3(HIST), 0, s, rband, c->rband + (p ^ 1) * c->fm_par,
                       c->fm_stride, n);
    LAUNCH_CHECK();
    hipLaunchKernelGGL((k_fir_rb<1, false>), gf, dim3(BLK), 0, s, fm, c->fm_stride, fm, c->fm_stride, c->rds_h,
                       nullptr, n, rband, nullptr, c->fm_stride, nullptr, 0);
    LAUNCH_CHECK();
    // squaring (:111-113) + 114 kHz BPF (:116)
    hipLaunchKernelGGL((k_fir_rb<1, true>), gf, dim3(BLK), 0, s, rband, c->fm_stride, rband, c->fm_stride,
                       c->rds_sq_h, nullptr, n, c->plain(c->gpilot), nullptr, c->plain_stride,
                       c->rxbuf(c->rx_rds), c->plain_stride);
    LAUNCH_CHECK();
    c->rds_pre_done = c->block;
    return SDR_OK;
}

int sdr_rds_pll(sdr_ctx* c, void* stream) {
    if (!c) return fail(SDR_E_INVALID, "null context");
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

int sdr_plls_launch(sdr_ctx* c, int nblocks, void* stream) {
    if (!c || nblocks <= 0) return fail(SDR_E_INVALID, "plls_launch: bad arguments");
    if (c->flags & SDR_FLAG_PLL_LIBM) return fail(SDR_E_INVALID, "plls_launch: not with SDR_FLAG_PLL_LIBM");
    if (c->pers_signaled != c->pers_launched)
        return fail(SDR_E_INVALID, "plls_launch: the previous launch still has %u blocks to signal",
                    c->pers_launched - c->pers_signaled);
    HIP_TRY(hipSetDevice(c->device));
    hipStream_t s = S(stream);
    if (!c->pers_words) {
        const int r = dalloc(c, &c->pers_words, 4);
        if (r) return r;
    }
    if (c->pers_tcap < nblocks) {   // grow the timestamp arrays (the previous launch finished first)
        HIP_TRY(hipStreamSynchronize(s));
        int r = dalloc(c, &c->pers_t0, (size_t)nblocks);
        if (!r) r = dalloc(c, &c->pers_t1, (size_t)nblocks);
        if (r) return r;
        c->pers_tcap = nblocks;
    }
    HIP_TRY(hipMemsetAsync(c->pers_t0, 0xFF, (size_t)nblocks * sizeof(unsigned long long), s));
    HIP_TRY(hipMemsetAsync(c->pers_t1, 0, (size_t)nblocks * sizeof(unsigned long long), s));
    const int n = c->info.block_if, nch = c->nch;
    PllJobs2 jobs{};
    const int first_parity = c->parity ^ 1;   // the parity the next sdr_frontend switches to: p[0]
    for (int k = 0; k < 2; k++) {
        const int saved = c->parity;
        c->parity = first_parity ^ k;
        jobs.p[k].j[0] = stereo_job(c);
        jobs.p[k].j[1] = rds_job(c);
        c->parity = saved;
    }
    bool vec = true;
    for (int k = 0; k < 2; k++)
        for (int q = 0; q < 2; q++) {
            const PllJob& j = jobs.p[k].j[q];
            vec = vec && (reinterpret_cast<uintptr_t>(j.in) % 16 == 0) && (j.in_stride % 4 == 0) &&
                  (reinterpret_cast<uintptr_t>(j.tbuf) % 16 == 0) && (j.t_stride % 4 == 0) &&
                  (reinterpret_cast<uintptr_t>(j.rx) % 16 == 0) && (j.rx_stride % 2 == 0);
        }
    const size_t tab_bytes = round_up((size_t)std::max(n, 1), 2) * sizeof(double);
    const int tab_ok = (tab_bytes <= 64 * 1024 && !pll_notab_env()) ? 1 : 0;
    const dim3 g(cdiv(nch, 64), 2), b(64);
    c->pers_waves = g.x * g.y;
    const char* acq = std::getenv("SDR_PLL_ACQUIRE");   // diagnosis: system-scope acquire
    const int sys_acq = (acq && std::strcmp(acq, "system") == 0) ? 1 : 0;
    uint32_t* w = c->pers_words;
    if (vec)
        hipLaunchKernelGGL(k_pll_multi<true>, g, b, tab_ok ? tab_bytes : 0, s, jobs, n, nch, tab_ok, nblocks,
                           w, c->pers_launched, w + 1, w + 2, c->pers_t0, c->pers_t1, sys_acq);
    else
        hipLaunchKernelGGL(k_pll_multi<false>, g, b, tab_ok ? tab_bytes : 0, s, jobs, n, nch, tab_ok, nblocks,
                           w, c->pers_launched, w + 1, w + 2, c->pers_t0, c->pers_t1, sys_acq);
    LAUNCH_CHECK();
    c->pers_launched += (uint32_t)nblocks;
    c->pers_last_n = nblocks;
    return SDR_OK;
}

int sdr_plls_signal(sdr_ctx* c, void* stream) {
    if (!c) return fail(SDR_E_INVALID, "null context");
    if (c->st_pre_done != c->block || c->rds_pre_done != c->block || c->st_pll_done == c->block ||
        c->rds_pll_done == c->block)
        return fail(SDR_E_INVALID, "plls_signal: run sdr_stereo_pre and sdr_rds_pre on a new block first");
    if (c->pers_signaled == c->pers_launched)
        return fail(SDR_E_INVALID, "plls_signal: no sdr_plls_launch covers this block");
    hipLaunchKernelGGL(k_flag_store, dim3(1), dim3(64), 0, S(stream), c->pers_words, c->pers_signaled + 1u);
    LAUNCH_CHECK();
    c->pers_block = c->block;
    c->pers_block_seq = c->pers_signaled;
    c->pers_signaled++;
    c->st_pll_done = c->rds_pll_done = c->block;
    return SDR_OK;
}

int sdr_plls_wait(sdr_ctx* c, void* stream) {
    if (!c) return fail(SDR_E_INVALID, "null context");
    if (c->pers_block != c->block) return fail(SDR_E_INVALID, "plls_wait: sdr_plls_signal this block first");
    const uint32_t want = c->pers_waves * (c->pers_block_seq + 1u);
    hipLaunchKernelGGL(k_flag_wait, dim3(1), dim3(64), 0, S(stream), c->pers_words + 1, want, c->pers_words + 2);
    LAUNCH_CHECK();
    return SDR_OK;
}

int sdr_plls_report(sdr_ctx* c, double* block_ms, int max_blocks, int* nblocks, void* stream) {
    if (!c || !c->pers_words) return fail(SDR_E_INVALID, "plls_report: no persistent launch");
    hipStream_t s = S(stream);
    const int n = std::min(c->pers_last_n, std::max(max_blocks, 0));
    std::vector<unsigned long long> t0((size_t)std::max(n, 1)), t1((size_t)std::max(n, 1));
    uint32_t words[4] = {0, 0, 0, 0};
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
    if (words[2])
        return fail(SDR_E_HIP, "plls_report: a persistent PLL wait timed out (outputs invalid): err %u, flag %u, "
                    "done %u, signalled %u, launched %u, waves %u", words[2], words[0], words[1], c->pers_signaled,
                    c->pers_launched, c->pers_waves);
    return SDR_OK;
}

int sdr_rds_post(sdr_ctx* c, float* rds_clean, size_t rds_stride, void* stream) {
    if (!c) return fail(SDR_E_INVALID, "null context");
    if (c->rds_pll_done != c->block || c->rds_dsp_done == c->block)
        return fail(SDR_E_INVALID, "rds_post: run sdr_rds_pll on a new block first");
    const sdr_info& in = c->info;
    hipStream_t s = S(stream);
    const int n = in.block_if, T = c->ntaps, p = c->parity;
    float* rband = c->rband + p * c->fm_par;
    float* rdc = c->rdc + p * c->fm_par;
    float* rfilt = c->rfilt + p * c->rf_par;
    {
        PllJobs jobs{};
        jobs.j[0] = rds_job(c);                       // NCO output of this block's PLL (rds.cpp:119)
        const int r = launch_nco(jobs, 1, n, c->nch, s);
        if (r) return r;
    }
    // delay (rds.cpp:122) + mixer (:125-127) into the extended rds_dc stream
    hipLaunchKernelGGL(k_mix<true>, dim3(cdiv(n, BLK), c->nch), dim3(BLK), 0, s, rband, c->fm_stride,
                       c->pllbuf(c->ipll), c->pll_stride, n, rdc, c->rdc + (p ^ 1) * c->fm_par, c->fm_stride, 50);
    LAUNCH_CHECK();
    // 247/640 resampler (:130) into the extended rds_filt stream
    hipLaunchKernelGGL(k_hist_copy, dim3(c->nch), dim3(HIST), 0, s, rfilt, c->rfilt + (p ^ 1) * c->rf_par,
                       c->rf_stride, in.n_rds);
    LAUNCH_CHECK();
    if (resample_lc_span(c->rdsbb_L, 247, 640) > 64 * RLC_XL || ((c->rdsbb_L + 3) & ~3) > 64 * RLC_HL)
        return fail(SDR_E_INVALID, "rds_post: resampler tile does not fit (L = %d)", c->rdsbb_L);
    dim3 gr(cdiv(in.n_rds, RLC_TN), cdiv(c->nch, 64));
    auto kr = c->rdsbb_all101 ? k_resample_lc<101> : k_resample_lc<0>;
    hipLaunchKernelGGL(kr, gr, dim3(BLK), resample_lc_lds_bytes(c->rdsbb_L, 247, 640), s, rdc,
                       c->fm_stride, -HIST, c->rdsbb_pp, c->rdsbb_cnt, c->rdsbb_L, c->rds_ptq, in.n_rds, c->nch,
                       rfilt, c->rf_stride);
    LAUNCH_CHECK();
    // RRC (:133)
    dim3 gc(cdiv(in.n_rds, FRB_TILE), c->nch);
    float* dst = rds_clean ? rds_clean : c->rds_clean;
    const size_t dst_stride = rds_clean ? rds_stride : c->clean_stride;
    if (T != FRB_T) return fail(SDR_E_INVALID, "rds_post: %d taps", T);
    hipLaunchKernelGGL((k_fir_rb<1, false>), gc, dim3(BLK), 0, s, rfilt, c->rf_stride, rfilt, c->rf_stride,
                       c->rrc_h, nullptr, in.n_rds, dst, nullptr, dst_stride, nullptr, 0);
    LAUNCH_CHECK();
    if (rds_clean) {
        HIP_TRY(hipMemcpy2DAsync(c->rds_clean, c->clean_stride * sizeof(float), rds_clean, rds_stride * sizeof(float),
                                 in.n_rds * sizeof(float), c->nch, hipMemcpyDeviceToDevice, s));
    }
    c->rds_dsp_done = c->block;
    return SDR_OK;
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
    if (c->rds_dsp_done != c->block || c->rds_bits_done == c->block)
        return fail(SDR_E_INVALID, "rds_bits: run sdr_rds_dsp on a new block first");
    const sdr_info& in = c->info;
    hipLaunchKernelGGL(k_rds_bits, dim3(c->nch), dim3(64), 64 * sizeof(int), S(stream), c->rds_clean,
                       c->clean_stride, in.n_rds, in.symbol_Fs, c->rds_on, c->dec, offset, nsym, symbols,
                       sym_stride, nbits, bits, bits_stride);
    LAUNCH_CHECK();
    c->rds_bits_done = c->block;
    return SDR_OK;
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
    const size_t rx_bytes = ts * nch * sizeof(double), t_bytes = ts * nch * sizeof(float);
    const int mode = fmpll_scratch_mode();
    hipStream_t s = S(stream);
    if (mode >= 2) {
        void *rxp = nullptr, *tp = nullptr;
        HIP_TRY(hipMallocAsync(&rxp, rx_bytes, s));
        HIP_TRY(hipMallocAsync(&tp, t_bytes, s));
        if (mode == 4) HIP_TRY(hipStreamSynchronize(s));
        const int r = launch_pll(false, in, in_stride, n, nch, freq, Fs, static_cast<float*>(tp), ts,
                                 static_cast<double*>(rxp), out, out_stride, state, ncoScale, phaseAdjust,
                                 normBandwidth, s);
        if (mode != 3) {
            HIP_TRY(hipFreeAsync(rxp, s));
            HIP_TRY(hipFreeAsync(tp, s));
        }
        return r;
    }
    void* scratch = nullptr;
    if (mode == 1) {
        HIP_TRY(hipMalloc(&scratch, rx_bytes + t_bytes));
    } else {
        const int rc = stream_scratch(s, rx_bytes + t_bytes, &scratch);
        if (rc != SDR_OK) return rc;
    }
    double* rxbuf = static_cast<double*>(scratch);
    float* tbuf = reinterpret_cast<float*>(rxbuf + ts * nch);
    const int r = launch_pll(false, in, in_stride, n, nch, freq, Fs, tbuf, ts, rxbuf, out, out_stride, state, ncoScale,
                             phaseAdjust, normBandwidth, s);
    if (mode == 1) {
        HIP_TRY(hipStreamSynchronize(s));
        HIP_TRY(hipFree(scratch));
    }
    return r;
}

int sdr_cdr(int32_t* offset, const float* x, size_t x_stride, int nch, int n, int sps, void* stream) {
    if (!offset || !x || nch <= 0 || n < 0 || sps <= 0 || sps > 64) return fail(SDR_E_INVALID, "cdr: bad arguments");
    hipLaunchKernelGGL(k_cdr, dim3(nch), dim3(64), 64 * sizeof(int), S(stream), offset, x, x_stride, n, sps);
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
    const sdr_info& in = c->info;
    const int p = c->parity ^ 1;
    float* dst = c->fm + p * c->fm_par;
    HIP_TRY(hipMemcpy2DAsync(dst, c->fm_stride * sizeof(float), fm, fm_stride * sizeof(float),
                             in.block_if * sizeof(float), c->nch, hipMemcpyDeviceToDevice, S(stream)));
    hipLaunchKernelGGL(k_hist_copy, dim3(c->nch), dim3(HIST), 0, S(stream), dst, c->fm + (p ^ 1) * c->fm_par,
                       c->fm_stride, in.block_if);
    LAUNCH_CHECK();
    c->parity = p;
    c->block++;
    return SDR_OK;
}

}  // extern "C"

