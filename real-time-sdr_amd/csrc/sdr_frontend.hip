// sdr_frontend.hip -- RF front end of the FM/RDS hot path on MI355X (gfx950):
//   u8 I/Q -> 101-tap FIR /D on I and Q -> FM discriminator       rffrontend.cpp:58-71,
//   filter.cpp:106-121 (convolveFIR), demod.cpp:3-24 (fmDemodNoArctan)
// Exact mode (k_frontend2): the reference's f32 products and sums in tap order, f64 discriminator
// division. Fast mode (k_frontend_mfma): the FIR as an int8 Toeplitz GEMM on the matrix cores.
#include "sdr_internal.h"

#include <hip/hip_ext.h>

#include <algorithm>
#include <cstdlib>

#pragma clang fp contract(off)

// Diagnosis builds only (timing, wrong outputs; tools/build_variant.sh FEFLAGS=-DSDR_FE_DIAG=n):
// bit 0 -- k_frontend2 multiplies the raw window words instead of converted samples (no
// conversion), bit 1 -- no discriminator division, bit 2 -- every workgroup stages the same
// L2-resident window. The product build is SDR_FE_DIAG = 0.
#ifndef SDR_FE_DIAG
#define SDR_FE_DIAG 0
#endif

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
constexpr int FE_PF = 5;           // tap rows prefetched this many samples ahead (rotating SGPR ring;
                                   // 2-8 and hand-issued batches measured, profiles/r02/fe_exact_ab.txt)
// exact front end: outputs per lane (16 halves the occupancy: 1.54x slower, profiles/r04/ab_fe_r16.txt;
// 12 or 16 with the next tile's window prefetched in registers: slower too, profiles/r04/ab_fe_v4.txt)
#ifndef SDR_FE_R
#define SDR_FE_R 8
#endif
constexpr int FE_R = SDR_FE_R;
// exact discriminator: 1 = reciprocal + Newton step with a tie proof (IEEE division as the fallback),
// 0 = the IEEE f64 division on every output
#ifndef SDR_FE_DISC
#define SDR_FE_DISC 1
#endif
constexpr uint32_t FE_TIE_ULPS = 2048;   // > the fast quotient's 550-ulp error bound, with margin
// {h, h} * m with h one half (HI) of an SGPR pair: v_pk_mul_f32 with a scalar operand whose half
// is broadcast to both lanes by op_sel / op_sel_hi (no VGPR copy of the tap)
__device__ __forceinline__ f32x2 fe_mul_v(double hpair, int hi, f32x2 m) {
    f32x2 r;
    if (hi) asm volatile("v_pk_mul_f32 %0, %1, %2 op_sel:[1,0] op_sel_hi:[1,1]" : "=v"(r) : "s"(hpair), "v"(m));
    else asm volatile("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[0,1]" : "=v"(r) : "s"(hpair), "v"(m));
    return r;
}
// (I, Q) of one sample, sign-extended from the bytes of a dword that holds two samples
// (u8 ^ 0x80 == u8 - 128 as int8), converted in program order (volatile asm; the plain C++ form
// saves hazard waits but is no faster, profiles/r02/ab_fe_exact_asm.txt, profiles/r04/ab_fe_v4.txt)
template <int HALF>
__device__ __forceinline__ f32x2 fe_cvt_v(uint32_t w) {
    f32x2 r;
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
__device__ __forceinline__ f32x2 fe_add_v(f32x2 a, f32x2 b) {
    f32x2 r;
    asm volatile("v_pk_add_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
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

// One wave tile of the MFMA front end, I and Q of a block in ONE lane (NB a multiple of 16): a
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
#pragma unroll 1
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
template <int D, bool X4, int NB>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(4, 8))) void k_frontend_mfma(
    const uint8_t* __restrict__ iq, size_t iq_stride, const uint8_t* __restrict__ tail_in,
    uint8_t* __restrict__ tail_out, const float2* __restrict__ prev_in, float2* __restrict__ prev_out,
    const v4i* __restrict__ afrag, double yscale, int block_iq, int block_if,
    float* __restrict__ fm, const float* __restrict__ fm_other, size_t fm_stride, int tiles_ch,
    const uint32_t* __restrict__ pad, unsigned long long* __restrict__ stamps) {
    static_assert(15 * D + 101 <= 256, "one block's window must fit K = 256");
    // sdr_frontend_timing: this workgroup's start and end on the 100 MHz clock (as k_frontend2)
    if (stamps && threadIdx.x == 0) stamps[2 * blockIdx.x] = __builtin_amdgcn_s_memrealtime();
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
#pragma unroll
        for (int f = 0; f < FT_AFRAGS; f++) A[f] = afrag[f * 64 + t];
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
    ft_tile_iq<D, NB>(plane[0], A, yscale, c0, ch, prev_in[ch], prev_out, block_if, out);
    if (j == 0) {
        const uint16_t* last = reinterpret_cast<const uint16_t*>(src) + (block_iq - HP);
        uint16_t* tout = reinterpret_cast<uint16_t*>(tail_out + (size_t)ch * 2 * HP);
        for (int i = t; i < HP; i += 64) tout[i] = last[i];
        const float* o = fm_other + (size_t)ch * fm_stride;
        for (int i = t; i < HIST; i += 64) out[i - HIST] = o[block_if - HIST + i];
    }
    if (stamps) {   // the end: after this wave's stores have completed
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (threadIdx.x == 0) stamps[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
    }
}

// The FIR sweep of one tile: lane t's R outputs from its TWIN-sample window of sign-flipped bytes at
// sw + 2 t R D; 16-byte chunks are read from LDS two ahead of their use.
template <int R, int D>
__device__ __forceinline__ void fe_fir(const uint8_t* __restrict__ sw, const float* __restrict__ hs, f32x2 (&acc)[R]) {
    constexpr int NT = 101, HP = NT - 1;
    constexpr int TWIN = (R - 1) * D + NT;            // samples one thread reads
    constexpr int TCH = (2 * TWIN + 15) / 16;         // 16-byte LDS chunks per thread window
    const int t = threadIdx.x;
    uint4 chunk[TCH];
    const uint4* tw = reinterpret_cast<const uint4*>(sw + 2 * t * R * D);
    chunk[TCH - 1] = tw[TCH - 1];
    if (TCH >= 2) chunk[TCH - 2] = tw[TCH - 2];
#pragma unroll
    for (int r = 0; r < R; r++) acc[r] = f32x2{0.0f, 0.0f};
    // Taps live in SGPRs: row S of the table holds the R taps sample S meets (uniform across the
    // wave), fetched with scalar loads FE_PF samples ahead into a rotating ring and fed to the packed
    // multiplies as scalar operands (op_sel picks the half of the SGPR pair), so the VALU gets its
    // taps without LDS or VGPR traffic. The tap pointer is made opaque (otherwise every tap load is
    // hoisted and the TWIN*R taps overflow the SGPR file), then declared uniform again with
    // readfirstlane so the loads stay scalar.
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
        const uint32_t w = dw == 0 ? c4.x : dw == 1 ? c4.y : dw == 2 ? c4.z : c4.w;   // signed bytes (staging)
#if SDR_FE_DIAG & 1
        return f32x2{__builtin_bit_cast(float, w & 0x3F3F3F3Fu), __builtin_bit_cast(float, w & 0x3E3E3E3Eu)};
#else
        return (S & 1) ? fe_cvt_v<1>(w) : fe_cvt_v<0>(w);
#endif
    };
    // one sample of look-ahead: sample S-1 is converted while sample S's MACs issue
    f32x2 m_next = sample(TWIN - 1);
#pragma unroll
    for (int S = TWIN - 1; S >= 0; S--) {
        const int slot = S % FE_PF;
        if (((S & 7) == 7 || S == TWIN - 1) && (S >> 3) >= 2) chunk[(S >> 3) - 2] = tw[(S >> 3) - 2];
        const f32x2 m = m_next;
        // all products of the sample first, then the adds, in program order (volatile asm): no add
        // waits on the product issued just before it (filter.cpp:115: multiply, then add)
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

// The discriminator (demod.cpp:8-19) of lane t's R outputs c0 + t R + r and their stores into out
// (fm_demod of the channel; c0 is the tile's carry output, never written); the block's last (I, Q)
// goes to prev_out.
template <int R>
__device__ __forceinline__ void fe_disc_store(const f32x2 (&acc)[R], int c0, int ch, const float2* __restrict__ prev_in,
                                              float2* __restrict__ prev_out, float* __restrict__ out, int block_if) {
    // ---- discriminator (demod.cpp:8-19); the previous output of lane t's first comes from t-1
    const f32x2 left = f32x2{__shfl_up(acc[R - 1].x, 1), __shfl_up(acc[R - 1].y, 1)};
    const int t = threadIdx.x;
    const int cbase = c0 + t * R;
    float v[R];
#if SDR_FE_DIAG & 2
#pragma unroll
    for (int r = 0; r < R; r++) v[r] = acc[r].x + ((r > 0) ? acc[r > 0 ? r - 1 : 0] : left).y;
#else
    // the previous sample of output r; output 0 of the block (its previous sample is the last block's
    // carry, prev_in) can only be output 1 of lane 0 of tile 0 (c0 = j*ADV - 1 >= -1)
    auto prev = [&](int r) -> f32x2 {
        f32x2 pv = (r > 0) ? acc[r > 0 ? r - 1 : 0] : left;
        if (r == 1 && cbase == -1) {
            const float2 p = prev_in[ch];
            pv = f32x2{p.x, p.y};
        }
        return pv;
    };
#if SDR_FE_DISC
    // The reference's value is RN32(RN64(num / den)), den = RN64(I^2 + Q^2) (pow(x, 2.0) is exact
    // in f64, so den is one fma). Instead of the IEEE f64 division: q = RN64(num * r1), r1 = 1/den
    // from v_rcp_f64 (~2^-23 relative) refined by one Newton step, so |q / (num/den) - 1| < 2^-43.9,
    // i.e. < 550 ulps of q. RN32(q) equals the reference's value unless q lies within FE_TIE_ULPS
    // ulps of an f32 rounding tie (the tie key) or rounds to an f32 subnormal: a lane with any such
    // output recomputes its outputs by the division (a branch taken by ~1e-5 of the lanes).
    uint32_t kmin = 0xFFFFFFFFu;
    bool sub = false;
#pragma unroll
    for (int r = 0; r < R; r++) {
        const f32x2 cur = acc[r], pv = prev(r);
        const float num = cur.x * (cur.y - pv.y) - cur.y * (cur.x - pv.x);
        const double dI = (double)cur.x, dQ = (double)cur.y;
        const double den = __builtin_fma(dI, dI, dQ * dQ);
        const double r0 = __builtin_amdgcn_rcp(den);
        const double r1 = __builtin_fma(r0, __builtin_fma(-den, r0, 1.0), r0);
        const double q = (double)num * r1;
        const float vq = (float)q;
        const uint32_t key = ((uint32_t)__builtin_bit_cast(uint64_t, q) << 3) + (0x80000000u + 8u * FE_TIE_ULPS);
        kmin = key < kmin ? key : kmin;
        sub |= __builtin_amdgcn_classf(vq, 0x90);   // negative or positive f32 subnormal
        v[r] = den == 0.0 ? 0.0f : vq;              // (I, Q) = (0, 0): demod.cpp:15-16
    }
    if (kmin <= 16u * FE_TIE_ULPS || sub) {
#else
    {
#endif
#pragma unroll
        for (int r = 0; r < R; r++) {
            const f32x2 cur = acc[r], pv = prev(r);
            if ((cur.x == 0) & (cur.y == 0)) {
                v[r] = 0.0f;
            } else {
                const float num = cur.x * (cur.y - pv.y) - cur.y * (cur.x - pv.x);
                const double den = (double)cur.x * (double)cur.x + (double)cur.y * (double)cur.y;
                v[r] = (float)((double)num / den);
            }
        }
    }
#endif
    if (t > 0 && cbase + R < block_if) {             // all R outputs written, none the block's last
        if ((reinterpret_cast<uintptr_t>(out + cbase) & 7) == 0) {
#pragma unroll
            for (int r = 0; r < R; r += 2) *reinterpret_cast<float2*>(out + cbase + r) = make_float2(v[r], v[r + 1]);
        } else {
#pragma unroll
            for (int r = 0; r < R; r++) out[cbase + r] = v[r];
        }
    } else {
#pragma unroll
        for (int r = 0; r < R; r++) {
            const int c = cbase + r;
            if (c > c0 && c >= 0 && c < block_if) out[c] = v[r];
            if (c == block_if - 1) prev_out[ch] = make_float2(acc[r].x, acc[r].y);
        }
    }
}

// Exact front end, one tile per workgroup (64 lanes): a tile = 64*R decimated outputs starting one
// before the first fm_demod sample it writes (the discriminator's carry, demod.cpp:16); tiles
// advance by 64*R-1. The tile's u8 window goes HBM -> registers (coalesced dwords) -> LDS, then every
// lane sweeps its R outputs' window. Boundary tiles (the first reads the previous block's tail, the
// last runs into the padding, u8 128 = 0.0f) stage per dword from the block, the tail or the pad.
// Tiles j0 .. j0+jn-1 of every channel (blockIdx.x = ch*jn + j - j0): the whole block (j0 = 0, jn =
// tiles per channel) or one part of it (sdr_frontend_pre_parts, the pipeline fill).
template <int R, int D>
__global__ __launch_bounds__(64) void k_frontend2(
    const uint8_t* __restrict__ iq, size_t iq_stride, const uint8_t* __restrict__ tail_in,
    uint8_t* __restrict__ tail_out, const float2* __restrict__ prev_in, float2* __restrict__ prev_out,
    const float* __restrict__ hs, int block_iq, int block_if,
    float* __restrict__ fm, const float* __restrict__ fm_other, size_t fm_stride, int j0, int jn,
    const uint32_t* __restrict__ pad, unsigned long long* __restrict__ stamps) {
    constexpr int NT = 101, HP = NT - 1, NTH = 64;
    // sdr_frontend_timing: this workgroup's start and end on the 100 MHz clock (the launch's span is
    // the earliest start to the latest end, computed on the host)
    if (stamps && threadIdx.x == 0) stamps[2 * blockIdx.x] = __builtin_amdgcn_s_memrealtime();
    constexpr int TILE = NTH * R;
    constexpr int ADV = TILE - 1;
    constexpr int WIN = (TILE - 1) * D + NT;          // staged samples (u8 I/Q pairs)
    constexpr int NG = (2 * WIN + 3) / 4;             // dwords of one tile window
    constexpr int PER = (NG + NTH - 1) / NTH;         // dwords per lane
    constexpr int LDS_BYTES = ((2 * WIN + 15) / 16) * 16 + 32;
    __shared__ __attribute__((aligned(16))) uint8_t sw[LDS_BYTES];
    const int t = threadIdx.x;
    const int ch = (int)blockIdx.x / jn, j = j0 + (int)blockIdx.x - ch * jn;
    const int c0 = j * ADV - 1;                       // first decimated output (the carry)
    const int m0 = c0 * D - HP;                       // first staged sample
    const uint8_t* src = iq + (size_t)ch * iq_stride;
#if SDR_FE_DIAG & 4
    // diagnosis: every workgroup stages channel 0's second tile (L2-resident input, staging latency
    // without HBM misses)
    const int m0s = ADV * D - D - HP;
    const uint8_t* srcs = iq;
#else
    const int m0s = m0;
    const uint8_t* srcs = src;
#endif
    {
        // window -> LDS (lane t holds dwords t, t+64, ...). Every I/Q sample is one u16; samples
        // before the block come from the previous block's tail, samples past its end are u8 128.
        // With D even the window starts on an even sample, so each dword is wholly in the block, in
        // the tail or in the padding: one load (or constant) per dword.
        uint32_t* sd = reinterpret_cast<uint32_t*>(sw);
        const uint8_t* tin = tail_in + (size_t)ch * 2 * HP;
        if (D % 2 == 0) {
            if (m0s >= 0 && m0s + WIN <= block_iq) {
                const uint32_t* g = reinterpret_cast<const uint32_t*>(srcs + 2 * m0s);
                uint32_t pf[PER];
#pragma unroll
                for (int k = 0; k < PER; k++) {
                    const int i = t + NTH * k;
                    pf[k] = (k < PER - 1 || i < NG) ? __builtin_nontemporal_load(g + i) : 0u;
                }
#pragma unroll
                for (int k = 0; k < PER; k++) {
                    const int i = t + NTH * k;
                    if (k < PER - 1 || i < NG) sd[i] = pf[k] ^ 0x80808080u;
                }
            } else {
                const uint32_t* gs = reinterpret_cast<const uint32_t*>(src);
                const uint32_t* gt = reinterpret_cast<const uint32_t*>(tin);
                for (int i = t; i < NG; i += NTH) {
                    const int mm = m0 + 2 * i;
                    const uint32_t* pa = mm >= 0 ? (mm < block_iq ? gs + (mm >> 1) : pad)
                                                 : (mm >= -HP ? gt + ((HP + mm) >> 1) : pad);
                    sd[i] = *pa ^ 0x80808080u;
                }
            }
        } else {
            const uint16_t* s16 = reinterpret_cast<const uint16_t*>(src);
            const uint16_t* t16 = reinterpret_cast<const uint16_t*>(tin);
            for (int i = t; i < NG; i += NTH) {
                uint32_t v = 0;
#pragma unroll
                for (int h = 0; h < 2; h++) {
                    const int m = m0 + 2 * i + h;
                    const uint16_t* pa = m >= 0 ? s16 + m : t16 + (HP + m);
                    if (m < -HP || m >= block_iq) pa = reinterpret_cast<const uint16_t*>(pad);
                    v |= (uint32_t)*pa << (16 * h);
                }
                sd[i] = v ^ 0x80808080u;
            }
        }
    }
    __syncthreads();
    f32x2 acc[R];
    fe_fir<R, D>(sw, hs, acc);
    fe_disc_store<R>(acc, c0, ch, prev_in, prev_out, fm + (size_t)ch * fm_stride, block_if);
    float* out = fm + (size_t)ch * fm_stride;
    if (j == 0) {
        const uint16_t* last = reinterpret_cast<const uint16_t*>(src) + (block_iq - HP);
        uint16_t* tout = reinterpret_cast<uint16_t*>(tail_out + (size_t)ch * 2 * HP);
        for (int i = t; i < HP; i += NTH) tout[i] = last[i];
        const float* o = fm_other + (size_t)ch * fm_stride;
        for (int i = t; i < HIST; i += NTH) out[i - HIST] = o[block_if - HIST + i];
    }
    if (stamps) {   // the end: after this wave's stores have completed
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (threadIdx.x == 0) stamps[2 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
    }
}

size_t frontend_lds_bytes(int ntaps, int tile, int D) {
    const int ntaps_pad = (ntaps + 3) & ~3;
    const int W = tile * D + ntaps;                  // window incl. the extra output at n0-1
    return (size_t)ntaps_pad * 4 + (size_t)((W + 1) & ~1) * 8 + (size_t)(tile + 1) * 8 + 64;
}

}  // namespace

// One block of every channel (the RF_frontend loop body), or tiles [j0, j0 + jn) of it (a part of
// the pipeline fill, sdr_frontend_pre_parts): picks the kernel for the context's numerics and
// decimation.
int frontend_tiles(int block_if) { return cdiv(block_if + 1, 64 * FE_R - 1); }
int frontend_tab_r() { return FE_R; }

int frontend_launch(const FrontendArgs& a, hipStream_t s, int j0, int jn) {
    const uint8_t* iq = a.iq;
    const size_t iq_stride = a.iq_stride;
    const uint8_t* tail_in = a.tail_in;
    uint8_t* tail_out = a.tail_out;
    const float2* prev_in = a.prev_in;
    float2* prev_out = a.prev_out;
    float* fm_p = a.fm;
    const float* fm_o = a.fm_other;
    const int tiles_ch = frontend_tiles(a.block_if);
    if (jn <= 0) { j0 = 0; jn = tiles_ch; }
    if (j0 < 0 || j0 + jn > tiles_ch) return fail(SDR_E_INVALID, "frontend: tiles [%d, %d) of %d", j0, j0 + jn, tiles_ch);
    const dim3 g2(jn * a.nch);
    // sdr_frontend_timing: k_frontend2 and k_frontend_mfma stamp each workgroup's start and end
    // (a.stamps); the generic kernel records HIP events with the launch (hipExtLaunchKernelGGL: the
    // start event is a marker ahead of the dispatch, so its span exceeds the kernel's by the marker's
    // latency, ~9 us)
#define FE2(DD)                                                                                               \
    hipExtLaunchKernelGGL((k_frontend2<FE_R, DD>), g2, dim3(64), 0, s, a.ev0, a.ev1, 0, iq, iq_stride, tail_in, \
                          tail_out, prev_in, prev_out, a.hs, a.block_iq, a.block_if, fm_p, fm_o, a.fm_stride, j0, jn, \
                          a.pad80, a.stamps)
    if (a.fast) {
        if (j0 != 0 || jn != tiles_ch) return fail(SDR_E_INVALID, "frontend: parts need the exact front end");
        const v4i* af = static_cast<const v4i*>(a.afrag);
        // 16-byte I/Q group loads need 16-byte aligned rows (e.g. a row stride of 147008 for mode 0)
        const bool x4 = (iq_stride % 16 == 0) && (reinterpret_cast<uintptr_t>(iq) % 16 == 0);
        constexpr int NB = FT_NB;
#define FEM(DD, XX)                                                                                          \
        hipExtLaunchKernelGGL((k_frontend_mfma<DD, XX, NB>), dim3(cdiv(a.block_if, ft_adv(DD, NB)) * a.nch),   \
                              dim3(64), 0, s, a.ev0, a.ev1, 0, iq, iq_stride, tail_in, tail_out, prev_in, prev_out, af, \
                              a.yscale, a.block_iq, a.block_if, fm_p, fm_o, a.fm_stride,                            \
                              cdiv(a.block_if, ft_adv(DD, NB)), a.pad80, a.stamps)
        if (a.D == 10) { if (x4) FEM(10, true); else FEM(10, false); }
        else if (a.D == 4) { if (x4) FEM(4, true); else FEM(4, false); }
        else { if (x4) FEM(3, true); else FEM(3, false); }
#undef FEM
    } else if (a.ntaps == 101 && a.D == 10) {
        FE2(10);
    } else if (a.ntaps == 101 && a.D == 4) {
        FE2(4);
    } else if (a.ntaps == 101 && a.D == 3) {
        FE2(3);
    } else {
        if (j0 != 0 || jn != tiles_ch) return fail(SDR_E_INVALID, "frontend: parts need 101 taps");
        const int tile = FIR_TILE;
        dim3 grid(cdiv(a.block_if, tile), a.nch);
        const size_t lds = frontend_lds_bytes(a.ntaps, tile, a.D);
        hipExtLaunchKernelGGL(k_frontend, grid, dim3(BLK), (uint32_t)lds, s, a.ev0, a.ev1, 0, iq, iq_stride, tail_in,
                              tail_out, prev_in, prev_out, a.h, a.ntaps, a.D, a.block_iq, a.block_if, tile, fm_p, fm_o,
                              a.fm_stride);
    }
#undef FE2
    LAUNCH_CHECK();
    return SDR_OK;
}

int frontend_stamp_wgs(int block_if, int nch, int ntaps, int D, bool fast) {
    if (D != 10 && D != 4 && D != 3) return 0;
    if (fast) return cdiv(block_if, ft_adv(D, FT_NB)) * nch;
    return ntaps == 101 ? frontend_tiles(block_if) * nch : 0;
}

}  // namespace sdrk
