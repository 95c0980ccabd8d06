// sdr_frontend.hip -- RF front end of the FM/RDS hot path on MI355X (gfx950):
//   u8 I/Q -> 101-tap FIR /D on I and Q -> FM discriminator       rffrontend.cpp:58-71,
//   filter.cpp:106-121 (convolveFIR), demod.cpp:3-24 (fmDemodNoArctan)
// Exact mode (k_frontend2): the reference's f32 products and sums in tap order, f64 discriminator
// division. Fast mode (k_frontend_mfma): the FIR as an int8 Toeplitz GEMM on the matrix cores.
#include "sdr_internal.h"

#include <algorithm>
#include <cstdlib>

#pragma clang fp contract(off)

namespace sdrk {
namespace {
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
// SDR_FE_VTAP=1: the exact front end keeps all 101 taps (h/128, 51 VGPR pairs) in registers instead
// of streaming per-sample tap rows through SGPRs. Scalar loads return out of order, so every use of a
// prefetched SGPR row waits for ALL scalar loads in flight (lgkmcnt(0), which the LDS window reads
// share): the SGPR ring exposes the scalar-cache latency every few samples.
// Not adopted: the 102 tap VGPRs leave 2 waves per SIMD and the kernel runs 8 % slower
// (profiles/r03/ab_fe_vtap.txt).
#ifndef SDR_FE_VTAP
#define SDR_FE_VTAP 0
#endif

// {h, h} * m with h one half (HI) of an SGPR pair: v_pk_mul_f32 with a scalar operand whose half
// is broadcast to both lanes by op_sel / op_sel_hi (no VGPR copy of the tap)
// the same with the tap pair in VGPRs (SDR_FE_VTAP: all taps resident in registers)
__device__ __forceinline__ f32x2 fe_mul_vv(double hpair, int hi, f32x2 m) {
    f32x2 r;
    if (hi) asm volatile("v_pk_mul_f32 %0, %1, %2 op_sel:[1,0] op_sel_hi:[1,1]" : "=v"(r) : "v"(hpair), "v"(m));
    else asm volatile("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[0,1]" : "=v"(r) : "v"(hpair), "v"(m));
    return r;
}
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
// NB = 16-output blocks per wave tile (NB/8 C tiles of 8 blocks). Tile j computes outputs
// c0 .. c0 + 16*NB - 1 with c0 = j*ADV - CARRY and writes the ADV outputs from c0 + CARRY on (the
// CARRY >= 1 before them feed the discriminator). (ADV, CARRY) per D make the first staged sample
// m0 = c0*D - 100 a multiple of 8 (16-byte I/Q groups) on every tile.
constexpr int ft_adv(int D, int NB) { return D == 3 ? 16 * NB - 8 : 16 * NB - 4; }
constexpr int ft_carry(int D) { return D == 10 ? 2 : D == 4 ? 1 : 4; }
constexpr int ft_win(int D, int NB) { return 16 * D * (NB - 1) + 256; }
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
    const float* __restrict__ hs, const float* __restrict__ hv, int block_iq, int block_if,
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
#if SDR_FE_VTAP
    double tv[(NT + 1) / 2];          // tv[j] = {h[2j], h[2j+1]} / 128, uniform, held in VGPRs
    auto load_taps = [&]() {
#pragma unroll
        for (int j = 0; j < (NT + 1) / 2; j++) {
            double x = reinterpret_cast<const double*>(hv)[j];
            asm volatile("" : "+v"(x));
            tv[j] = x;
        }
    };
    // VTAP 1: before the window staging (tap and window registers overlap); 2: after it
    if (SDR_FE_VTAP == 1) load_taps();
#endif
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
#if SDR_FE_VTAP
        if (SDR_FE_VTAP == 2) load_taps();
#endif
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
#if SDR_FE_VTAP
                    if (k >= 0 && k < NT) prod[r] = fe_mul_vv(tv[k >> 1], k & 1, m);
#else
                    if (k >= 0 && k < NT) prod[r] = fe_mul_v(ring[slot][r >> 1], r & 1, m);
#endif
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
// Front end v3 (exact): lanes are SEGMENTS of R consecutive decimated outputs, each streaming its
// own window of TWIN = (R-1)*D + 101 u8 I/Q pairs straight from HBM/L2 into registers (16-byte
// loads a few chunks ahead of the sweep; no LDS, so occupancy is set by VGPRs alone). The window
// is swept in DESCENDING sample order as in k_frontend2, so every output accumulates its taps in
// ascending k (filter.cpp:110-116) with the reference's f32 product and sum roundings; the taps
// come from the same per-sample SGPR rows. Segments are phase-aligned (first output c with
// 2*(D*c - 100) a multiple of 16), so any 64 of them share one instruction stream: a wave takes 63
// consecutive segments of the flattened (channel, segment) order, lane 0 recomputing the
// previous wave's last one for the discriminator's carry (demod.cpp:16) and writing nothing.
// Segment i of a channel computes outputs [C0 + R*i, C0 + R*(i+1)); the last one is pulled back
// to end at block_if (its overlap with the one before is written twice with identical values),
// so no lane reads past its channel's block. The HEAD outputs [0, C0], whose windows reach into
// the previous block (the u8 tail), are computed by the first waves of the grid (lane = channel,
// same sweep from an 8-byte-granular tail/row window), which also copy the tail and the f32
// history of the next block.
// ------------------------------------------------------------------------------------------
constexpr int fe3_c0(int D) {
    int c = (100 + D - 1) / D;
    while ((D * c - 100) % 8) c++;
    return c;
}
constexpr int fe3_m(int D) { return D % 8 == 0 ? 1 : D % 4 == 0 ? 2 : D % 2 == 0 ? 4 : 8; }
#ifndef SDR_FE3_PD
#define SDR_FE3_PD 4
#endif
constexpr int FE3_PD = SDR_FE3_PD;   // 16-byte window chunks loaded ahead of the one being swept

// discriminator of one output (demod.cpp:8-19): f32 numerator, f64 denominator and division
__device__ __forceinline__ float fe_disc(f32x2 cur, f32x2 pv) {
    if ((cur.x == 0) & (cur.y == 0)) return 0.0f;
    const float num = cur.x * (cur.y - pv.y) - cur.y * (cur.x - pv.x);
    const double den = (double)cur.x * (double)cur.x + (double)cur.y * (double)cur.y;
    return (float)((double)num / den);
}

// The register-blocked sweep of one lane window: acc[r] = (I, Q) of the lane's output r. load(q)
// returns 16-byte chunk q of the window (samples 8q .. 8q+7), called in descending q.
template <int R, int D, typename Load>
__device__ __forceinline__ void fe3_sweep(const float* __restrict__ hs, Load load, f32x2 (&acc)[R]) {
    constexpr int NT = 101, HP = NT - 1;
    constexpr int TWIN = (R - 1) * D + NT;
    constexpr int NCH = (2 * TWIN + 15) / 16;
    uint4 chunk[NCH];
#pragma unroll
    for (int q = NCH - 1; q >= 0 && q >= NCH - 1 - FE3_PD; q--) chunk[q] = load(q);
#pragma unroll
    for (int r = 0; r < R; r++) acc[r] = f32x2{0.0f, 0.0f};
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
    auto sample = [&](int S) -> f32x2 {
        const uint4 c4 = chunk[S >> 3];
        const int dw = (S & 7) >> 1;
        const uint32_t w = (dw == 0 ? c4.x : dw == 1 ? c4.y : dw == 2 ? c4.z : c4.w) ^ 0x80808080u;
        return (S & 1) ? fe_cvt_v<1>(w) : fe_cvt_v<0>(w);
    };
    f32x2 m_next = sample(TWIN - 1);
#pragma unroll
    for (int S = TWIN - 1; S >= 0; S--) {
        const int slot = S % FE_PF;
        // entering chunk S>>3: the chunk FE3_PD + 1 below it goes in flight
        if (((S & 7) == 7 || S == TWIN - 1) && (S >> 3) - FE3_PD - 1 >= 0) {
            const int q = (S >> 3) - FE3_PD - 1;
            chunk[q] = load(q);
        }
        const f32x2 m = m_next;
        f32x2 prod[R];
#pragma unroll
        for (int r = 0; r < R; r++) {
            const int k = r * D + HP - S;
            if (k >= 0 && k < NT) prod[r] = fe_mul_v(ring[slot][r >> 1], r & 1, m);
        }
        if (S > 0) m_next = sample(S - 1);
#pragma unroll
        for (int r = 0; r < R; r++) {
            const int k = r * D + HP - S;
            if (k >= 0 && k < NT) acc[r] = fe_add_v(acc[r], prod[r]);
        }
        if (S - FE_PF >= 0) {
#pragma unroll
            for (int q = 0; q < R / 2; q++) ring[slot][q] = hsd[(S - FE_PF) * (R / 2) + q];
        }
        __builtin_amdgcn_sched_barrier(0);
    }
}

template <int R, int D, bool X4>
__global__ __launch_bounds__(64) void k_frontend3(
    const uint8_t* __restrict__ iq, size_t iq_stride, const uint8_t* __restrict__ tail_in,
    uint8_t* __restrict__ tail_out, const float2* __restrict__ prev_in, float2* __restrict__ prev_out,
    const float* __restrict__ hs, int block_iq, int block_if, float* __restrict__ fm,
    const float* __restrict__ fm_other, size_t fm_stride, int nch, int segs_ch, int head_waves) {
    constexpr int NT = 101, HP = NT - 1;
    constexpr int C0 = fe3_c0(D), M = fe3_m(D), A = C0 % M;
    static_assert(R % M == 0 && A == 2 && M == 4, "store layout below assumes D == 10 alignment");
    static_assert(C0 + 1 <= R, "the head lane computes outputs 0 .. C0 in one sweep");
    const int t = threadIdx.x;
    f32x2 acc[R];
    if ((int)blockIdx.x < head_waves) {
        // ---- head: lane = channel, outputs 0 .. C0 from samples [-HP, D*(R-1)] ----
        const int ch = min((int)blockIdx.x * 64 + t, nch - 1);
        const uint2* tl = reinterpret_cast<const uint2*>(tail_in + (size_t)ch * 2 * HP);   // samples -HP..-1
        const uint2* rw = reinterpret_cast<const uint2*>(iq + (size_t)ch * iq_stride);      // samples 0..
        // window byte b <-> sample -HP + b/2; 8-byte piece p: tail piece p (p < 25), row piece p - 25
        auto piece = [&](int p) -> uint2 { return p < HP / 4 ? tl[p] : rw[p - HP / 4]; };
        fe3_sweep<R, D>(hs, [&](int q) -> uint4 {
            const uint2 lo = piece(2 * q), hi = piece(2 * q + 1);
            return make_uint4(lo.x, lo.y, hi.x, hi.y);
        }, acc);
        if ((int)blockIdx.x * 64 + t < nch) {
            float* out = fm + (size_t)ch * fm_stride;
            const float2 p = prev_in[ch];
            f32x2 pv = f32x2{p.x, p.y};
#pragma unroll
            for (int r = 0; r <= C0; r++) {
                out[r] = fe_disc(acc[r], pv);
                pv = acc[r];
            }
        }
        // this block's u8 tail and the f32 history in front of this parity's stream, a channel
        // per iteration with the wave's lanes along it (coalesced)
        for (int cc = 0; cc < 64; cc++) {
            const int c = (int)blockIdx.x * 64 + cc;
            if (c >= nch) break;
            const uint16_t* last = reinterpret_cast<const uint16_t*>(iq + (size_t)c * iq_stride) + (block_iq - HP);
            uint16_t* tout = reinterpret_cast<uint16_t*>(tail_out + (size_t)c * 2 * HP);
            for (int i = t; i < HP; i += 64) tout[i] = last[i];
            float* out = fm + (size_t)c * fm_stride;
            const float* o = fm_other + (size_t)c * fm_stride;
            for (int i = t; i < HIST; i += 64) out[i - HIST] = o[block_if - HIST + i];
        }
        return;
    }
    // ---- segments: lane t takes flattened segment gb + t - 1 ----
    const int gb = ((int)blockIdx.x - head_waves) * 63;          // wave-uniform
    const int ch0 = gb / segs_ch, i0 = gb - ch0 * segs_ch;       // scalar division
    int ch = ch0, i = i0 + t - 1;
    if (i < 0) { ch -= 1; i += segs_ch; }
    if (i >= segs_ch) { ch += 1; i -= segs_ch; }
    bool writer = t > 0 && ch < nch;
    if (ch < 0) { ch = 0; i = 0; }
    if (ch >= nch) { ch = nch - 1; i = segs_ch - 1; }
    const int c_last = A + M * ((block_if - R - A) / M);
    const int cu = C0 + R * i;
    const int cl = min(cu, c_last);
    const bool write_first = writer && i > 0 && cu <= c_last;
    const uint8_t* src = iq + (size_t)ch * iq_stride + 2 * (D * cl - HP);
    if (X4) {   // 16-byte aligned rows: one load per chunk
        fe3_sweep<R, D>(hs, [&](int q) -> uint4 { return reinterpret_cast<const uint4*>(src)[q]; }, acc);
    } else {    // 8-byte aligned rows (e.g. a row stride of 147000 bytes): two
        fe3_sweep<R, D>(hs, [&](int q) -> uint4 {
            const uint2 lo = reinterpret_cast<const uint2*>(src)[2 * q], hi = reinterpret_cast<const uint2*>(src)[2 * q + 1];
            return make_uint4(lo.x, lo.y, hi.x, hi.y);
        }, acc);
    }
    // ---- discriminator: the previous output of lane t's first is lane t-1's last ----
    const f32x2 left = f32x2{__shfl_up(acc[R - 1].x, 1), __shfl_up(acc[R - 1].y, 1)};
    float v[R];
#pragma unroll
    for (int r = 0; r < R; r++) v[r] = fe_disc(acc[r], r > 0 ? acc[r > 0 ? r - 1 : 0] : left);
    if (writer) {
        float* out = fm + (size_t)ch * fm_stride + cl;             // cl == 2 (mod 4): out + 2 is 16-byte aligned
        if (write_first) out[0] = v[0];
        out[1] = v[1];
#pragma unroll
        for (int r = 2; r + 4 <= R; r += 4)
            *reinterpret_cast<float4*>(out + r) = make_float4(v[r], v[r + 1], v[r + 2], v[r + 3]);
        *reinterpret_cast<float2*>(out + R - 2) = make_float2(v[R - 2], v[R - 1]);
        if (cl + R == block_if) prev_out[ch] = make_float2(acc[R - 1].x, acc[R - 1].y);
    }
}

size_t frontend_lds_bytes(int ntaps, int tile, int D) {
    const int ntaps_pad = (ntaps + 3) & ~3;
    const int W = tile * D + ntaps;                  // window incl. the extra output at n0-1
    return (size_t)ntaps_pad * 4 + (size_t)((W + 1) & ~1) * 8 + (size_t)(tile + 1) * 8 + 64;
}

// k_frontend3's layout assumptions, checked per launch (otherwise k_frontend2 runs): 8-byte
// aligned input rows (16-byte aligned: one load per window chunk), 16-byte aligned fm_demod rows, the last segment ending exactly at block_if, segments
// per channel >= 64 (a wave spans at most two channels), no window chunk past the block.
bool fe3_ok(const FrontendArgs& a) {
    constexpr int R = FE3_R, D = 10, TWIN = (R - 1) * D + 101, NCH = (2 * TWIN + 15) / 16;
    constexpr int C0 = fe3_c0(D), M = fe3_m(D), A = C0 % M;
    if (!std::getenv("SDR_FE_V3") || std::atoi(std::getenv("SDR_FE_V3")) != 1) return false;   // A/B knob, off
    if (reinterpret_cast<uintptr_t>(a.iq) % 8 || a.iq_stride % 8) return false;
    if (reinterpret_cast<uintptr_t>(a.fm) % 16 || a.fm_stride % 4) return false;
    if (reinterpret_cast<uintptr_t>(a.tail_in) % 8) return false;
    if ((a.block_if - R - A) % M != 0) return false;
    if (cdiv(a.block_if - C0, R) < 64) return false;
    if (2 * (D * (a.block_if - R) - 100) + 16 * NCH > 2 * a.block_iq) return false;
    if (2 * (D * (R - 1) + 1) > 2 * a.block_iq) return false;
    return true;
}

}  // namespace

// One block of every channel (the RF_frontend loop body): picks the kernel for the context's
// numerics, decimation and tuning knobs.
int frontend_launch(const FrontendArgs& a, hipStream_t s) {
    const uint8_t* iq = a.iq;
    const size_t iq_stride = a.iq_stride;
    const uint8_t* tail_in = a.tail_in;
    uint8_t* tail_out = a.tail_out;
    const float2* prev_in = a.prev_in;
    float2* prev_out = a.prev_out;
    float* fm_p = a.fm;
    const float* fm_o = a.fm_other;
    const bool fast = a.fast;
    const int R = a.fe_r;
    const int tiles_ch = cdiv(a.block_if + 1, 64 * R - 1);
    const int total = tiles_ch * a.nch;
    // fe_grid == 0: one tile per workgroup (the hardware dispatcher balances the load when other
    // streams share the chip); otherwise a persistent grid that prefetches its next tile
    const dim3 g2(a.fe_grid > 0 ? std::min(total, a.fe_grid) : total);
#define FE2P(RR, DD, FF, PP)                                                                                 \
    hipLaunchKernelGGL((k_frontend2<RR, DD, FF, PP>), g2, dim3(64), 0, s, iq, iq_stride, tail_in,                \
                       tail_out, prev_in, prev_out, a.hs, a.hv, a.block_iq, a.block_if, fm_p, fm_o, a.fm_stride,  \
                       a.nch, tiles_ch, a.pad80)
#define FE2(RR, DD, FF) do { if (a.fe_grid > 0) FE2P(RR, DD, FF, true); else FE2P(RR, DD, FF, false); } while (0)
#define FE2R(DD)                                                                                             \
    do {                                                                                                     \
        if (R == 8) { if (fast) FE2(8, DD, true); else FE2(8, DD, false); }                                  \
        else { if (fast) FE2(4, DD, true); else FE2(4, DD, false); }                                         \
    } while (0)
    if (fast && a.mfma) {
        const v4i* af = static_cast<const v4i*>(a.afrag);
        // 16-byte I/Q group loads need 16-byte aligned rows (e.g. a row stride of 147008 for mode 0)
        const bool x4 = (iq_stride % 16 == 0) && (reinterpret_cast<uintptr_t>(iq) % 16 == 0);
#define FEMP(DD, NB, W)                                                                                      \
    hipLaunchKernelGGL((k_frontend_mfma_p<DD, (NB == 16 ? 16 : 32), W>), gp, dim3(64), 0, s, iq, iq_stride,       \
                       tail_in, tail_out, prev_in, prev_out, af, a.yscale, a.block_iq, a.block_if, fm_p,          \
                       fm_o, a.fm_stride, tc, tc * a.nch, a.pad80)
#define FEM(DD, XX, NB)                                                                                      \
    do {                                                                                                     \
        const int tc = cdiv(a.block_if, ft_adv(DD, NB));                                                     \
        if (XX && a.fe_wpe > 0 && (NB == 16 || NB == 32)) {                                                  \
            const int g = a.fe_grid > 0 ? a.fe_grid : 4 * a.fe_wpe * a.cus;                                  \
            const dim3 gp(std::min(tc * a.nch, g));                                                          \
            if (a.fe_wpe == 2) FEMP(DD, NB, 2); else if (a.fe_wpe == 4) FEMP(DD, NB, 4); else FEMP(DD, NB, 3); \
        } else if (XX && a.fe_grid > 0) {                                                                    \
            hipLaunchKernelGGL((k_frontend_mfma_q<DD, NB>), dim3(std::min(tc * a.nch, a.fe_grid)), dim3(64), \
                               0, s, iq, iq_stride, tail_in, tail_out, prev_in, prev_out, af,               \
                               a.yscale, a.block_iq, a.block_if, fm_p, fm_o, a.fm_stride, tc,                \
                               tc * a.nch, a.pad80);                                                         \
        } else {                                                                                             \
            hipLaunchKernelGGL((k_frontend_mfma<DD, XX, NB>), dim3(tc * a.nch), dim3(64), 0, s, iq,          \
                               iq_stride, tail_in, tail_out, prev_in, prev_out, af, a.yscale, a.block_iq,    \
                               a.block_if, fm_p, fm_o, a.fm_stride, tc, a.pad80);                            \
        }                                                                                                    \
    } while (0)
#define FEMN(DD, XX) do { if (a.fe_nb == 16) FEM(DD, XX, 16); else if (a.fe_nb == 24) FEM(DD, XX, 24); \
                             else if (a.fe_nb == 48) FEM(DD, XX, 48); else if (a.fe_nb == 64) FEM(DD, XX, 64); \
                             else FEM(DD, XX, 32); } while (0)
        if (a.D == 10) { if (x4) FEMN(10, true); else FEMN(10, false); }
        else if (a.D == 4) { if (x4) FEMN(4, true); else FEMN(4, false); }
        else { if (x4) FEMN(3, true); else FEMN(3, false); }
#undef FEMN
#undef FEM
#undef FEMP
    } else if (!fast && a.hs3 && a.ntaps == 101 && a.D == 10 && fe3_ok(a)) {
        constexpr int R3 = FE3_R;
        const int C0 = fe3_c0(10);
        const int segs = cdiv(a.block_if - C0, R3);
        const int head = cdiv(a.nch, 64);
        const dim3 g3(head + cdiv(a.nch * segs, 63));
        const bool x4 = (iq_stride % 16 == 0) && (reinterpret_cast<uintptr_t>(iq) % 16 == 0);
#define FE3(XX) hipLaunchKernelGGL((k_frontend3<R3, 10, XX>), g3, dim3(64), 0, s, iq, iq_stride, tail_in, tail_out, \
                                   prev_in, prev_out, a.hs3, a.block_iq, a.block_if, fm_p, fm_o, a.fm_stride, a.nch, segs, head)
        if (x4) FE3(true); else FE3(false);
#undef FE3
    } else if (a.ntaps == 101 && a.D == 10) {
        FE2R(10);
    } else if (a.ntaps == 101 && a.D == 4) {
        FE2R(4);
    } else if (a.ntaps == 101 && a.D == 3) {
        FE2R(3);
    } else {
        const int tile = FIR_TILE;
        dim3 grid(cdiv(a.block_if, tile), a.nch);
        const size_t lds = frontend_lds_bytes(a.ntaps, tile, a.D);
        hipLaunchKernelGGL(k_frontend, grid, dim3(BLK), lds, s, iq, iq_stride, tail_in, tail_out, prev_in,
                           prev_out, a.h, a.ntaps, a.D, a.block_iq, a.block_if, tile, fm_p, fm_o, a.fm_stride);
    }
#undef FE2R
#undef FE2
#undef FE2P
    LAUNCH_CHECK();
    return SDR_OK;
}

}  // namespace sdrk
