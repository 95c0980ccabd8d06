// Dependent-chain latency and single-wave issue cost of the VALU instructions on the PLL's
// critical path (one wave on an idle chip, s_memtime shader cycles per instruction).
//   hipcc --offload-arch=gfx950 -O3 -o valu_latency valu_latency.hip
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int N = 256;

#define CHAIN(NAME, TY, ASM, ...)                                                                  \
    __global__ void NAME(TY* out, long long* cyc, TY a, TY b) {                                     \
        TY x = a, y = b, z = a, w = b;                                                             \
        (void)y; (void)z; (void)w;                                                                 \
        long long t0 = 0, t1 = 0;                                                                  \
        for (int rep = 0; rep < 2; rep++) {                                                        \
            t0 = __builtin_amdgcn_s_memtime();                                                     \
            _Pragma("unroll") for (int i = 0; i < N; i++) { asm volatile(ASM : __VA_ARGS__); }            \
            t1 = __builtin_amdgcn_s_memtime();                                                     \
        }                                                                                          \
        out[threadIdx.x] = x + y + z + w;                                                          \
        if (threadIdx.x == 0) cyc[0] = t1 - t0;                                                    \
    }

// dependent: every instruction reads the previous result
CHAIN(d_fma_f64, double, "v_fma_f64 %0, %0, %1, %2", "+v"(x) : "v"(a), "v"(b))
CHAIN(d_mul_f64, double, "v_mul_f64 %0, %0, %1", "+v"(x) : "v"(a))
CHAIN(d_add_f64, double, "v_add_f64 %0, %0, %1", "+v"(x) : "v"(a))
CHAIN(d_rcp_f64, double, "v_rcp_f64 %0, %0", "+v"(x))
CHAIN(d_rndne_f64, double, "v_rndne_f64 %0, %0", "+v"(x))
CHAIN(d_fma_f32, float, "v_fma_f32 %0, %0, %1, %2", "+v"(x) : "v"(a), "v"(b))
CHAIN(d_mul_f32, float, "v_mul_f32 %0, %0, %1", "+v"(x) : "v"(a))
CHAIN(d_rcp_f32, float, "v_rcp_f32 %0, %0", "+v"(x))
CHAIN(d_xor_b32, float, "v_xor_b32 %0, %0, %1", "+v"(x) : "v"(a))
// independent: four interleaved chains
CHAIN(i_fma_f64, double, "v_fma_f64 %0, %0, %4, %5\n v_fma_f64 %1, %1, %4, %5\n v_fma_f64 %2, %2, %4, %5\n v_fma_f64 %3, %3, %4, %5",
      "+v"(x), "+v"(y), "+v"(z), "+v"(w) : "v"(a), "v"(b))
CHAIN(i_fma_f32, float, "v_fma_f32 %0, %0, %4, %5\n v_fma_f32 %1, %1, %4, %5\n v_fma_f32 %2, %2, %4, %5\n v_fma_f32 %3, %3, %4, %5",
      "+v"(x), "+v"(y), "+v"(z), "+v"(w) : "v"(a), "v"(b))
CHAIN(i_mul_f64, double, "v_mul_f64 %0, %0, %4\n v_mul_f64 %1, %1, %4\n v_mul_f64 %2, %2, %4\n v_mul_f64 %3, %3, %4",
      "+v"(x), "+v"(y), "+v"(z), "+v"(w) : "v"(a))

CHAIN(i_add_f64, double, "v_add_f64 %0, %0, %4\n v_add_f64 %1, %1, %4\n v_add_f64 %2, %2, %4\n v_add_f64 %3, %3, %4",
      "+v"(x), "+v"(y), "+v"(z), "+v"(w) : "v"(a))
CHAIN(i_rcp_f64, double, "v_rcp_f64 %0, %0\n v_rcp_f64 %1, %1\n v_rcp_f64 %2, %2\n v_rcp_f64 %3, %3",
      "+v"(x), "+v"(y), "+v"(z), "+v"(w))
CHAIN(i_rndne_f64, double, "v_rndne_f64 %0, %0\n v_rndne_f64 %1, %1\n v_rndne_f64 %2, %2\n v_rndne_f64 %3, %3",
      "+v"(x), "+v"(y), "+v"(z), "+v"(w))
CHAIN(i_xor_b32, float, "v_xor_b32 %0, %0, %4\n v_xor_b32 %1, %1, %4\n v_xor_b32 %2, %2, %4\n v_xor_b32 %3, %3, %4",
      "+v"(x), "+v"(y), "+v"(z), "+v"(w) : "v"(a))
CHAIN(i_cvt_f64_f32, double, "v_cvt_f64_f32 %0, %4\n v_cvt_f64_f32 %1, %4\n v_cvt_f64_f32 %2, %4\n v_cvt_f64_f32 %3, %4",
      "=v"(x), "=v"(y), "=v"(z), "=v"(w) : "v"((float)a))
CHAIN(i_cvt_f32_f64, float, "v_cvt_f32_f64 %0, %4\n v_cvt_f32_f64 %1, %4\n v_cvt_f32_f64 %2, %4\n v_cvt_f32_f64 %3, %4",
      "=v"(x), "=v"(y), "=v"(z), "=v"(w) : "v"((double)a))
CHAIN(i_pk_mul_f32, double, "v_pk_mul_f32 %0, %0, %4\n v_pk_mul_f32 %1, %1, %4\n v_pk_mul_f32 %2, %2, %4\n v_pk_mul_f32 %3, %3, %4",
      "+v"(x), "+v"(y), "+v"(z), "+v"(w) : "v"(a))
CHAIN(i_mix_f64_f32, double, "v_fma_f64 %0, %0, %4, %4\n v_xor_b32 %5, %5, %5\n v_fma_f64 %1, %1, %4, %4\n v_xor_b32 %6, %6, %6",
      "+v"(x), "+v"(y), "+v"(z), "+v"(w) : "v"(a), "v"(0), "v"(1))
CHAIN(i_mov_dpp, float, "v_mov_b32_dpp %0, %4 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n v_mov_b32_dpp %1, %4 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n v_mov_b32_dpp %2, %4 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n v_mov_b32_dpp %3, %4 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf",
      "=v"(x), "=v"(y), "=v"(z), "=v"(w) : "v"(a))
// the DPP exchange on the lane-pair PLL's chain: a DPP read of a VGPR written by the previous VALU
// instruction needs 2 wait states (s_nop 1 here, as the compiler inserts)
CHAIN(d_mov_dpp, float, "s_nop 1\n v_mov_b32_dpp %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf", "+v"(x))
CHAIN(d_mul_dpp, float, "s_nop 1\n v_mul_f32_dpp %0, %0, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf bound_ctrl:1",
      "+v"(x) : "v"(a))
CHAIN(d_nop_mul, float, "s_nop 1\n v_mul_f32 %0, %0, %1", "+v"(x) : "v"(a))
CHAIN(d_pk_mul, double, "v_pk_mul_f32 %0, %0, %1", "+v"(x) : "v"(a))
CHAIN(d_cvt_f64_f32, float, "v_cvt_f64_f32 v[40:41], %0\n v_cvt_f32_f64 %0, v[40:41]", "+v"(x) : : "v40", "v41")
CHAIN(d_cvt_rt, float, "v_cvt_f64_f32 v[40:41], %0\n v_cvt_f32_f64 %0, v[40:41]", "+v"(x) : : "v40", "v41")

template <typename TY>
void run(void (*k)(TY*, long long*, TY, TY), const char* name, int per_iter) {
    TY* o;
    long long* c;
    hipMalloc(&o, 64 * sizeof(TY));
    hipMalloc(&c, sizeof(long long));
    long long best = 1LL << 60;
    for (int it = 0; it < 5; it++) {
        hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, o, c, (TY)1.0000001, (TY)1e-9);
        hipDeviceSynchronize();
        long long h;
        hipMemcpy(&h, c, sizeof h, hipMemcpyDeviceToHost);
        if (h < best) best = h;
    }
    printf("%-14s %6.2f cycles per instruction\n", name, (double)best / (N * per_iter));
    hipFree(o);
    hipFree(c);
}

int main() {
    run(d_fma_f64, "dep fma_f64", 1);
    run(d_mul_f64, "dep mul_f64", 1);
    run(d_add_f64, "dep add_f64", 1);
    run(d_rcp_f64, "dep rcp_f64", 1);
    run(d_rndne_f64, "dep rndne_f64", 1);
    run(d_fma_f32, "dep fma_f32", 1);
    run(d_mul_f32, "dep mul_f32", 1);
    run(d_rcp_f32, "dep rcp_f32", 1);
    run(d_xor_b32, "dep xor_b32", 1);
    run(i_fma_f64, "ind fma_f64", 4);
    run(i_fma_f32, "ind fma_f32", 4);
    run(i_mul_f64, "ind mul_f64", 4);
    run(i_add_f64, "ind add_f64", 4);
    run(i_rcp_f64, "ind rcp_f64", 4);
    run(i_rndne_f64, "ind rndne_f64", 4);
    run(i_xor_b32, "ind xor_b32", 4);
    run(i_cvt_f64_f32, "ind cvt64_32", 4);
    run(i_cvt_f32_f64, "ind cvt32_64", 4);
    run(i_pk_mul_f32, "ind pk_mul", 4);
    run(i_mix_f64_f32, "ind fma64+xor", 4);
    run(i_mov_dpp, "ind mov_dpp", 4);
    run(d_cvt_rt, "dep cvt 64<-32->", 2);
    run(d_mov_dpp, "dep nop1+mov_dpp", 1);
    run(d_mul_dpp, "dep nop1+mul_dpp", 1);
    run(d_nop_mul, "dep nop1+mul_f32", 1);
    run(d_pk_mul, "dep pk_mul", 1);
    return 0;
}
