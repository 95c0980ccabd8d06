// Microbenchmark: wave64 issue cost of packed vs scalar f32 VALU instructions on gfx950, with many
// waves per SIMD (throughput) and one (lone-wave issue). Each kernel runs ITERS x 16 independent
// instances of one instruction (16 accumulators) through inline asm, so the compiler cannot change
// the instruction; the time per instruction per SIMD is derived from the kernel time.
//   hipcc --offload-arch=gfx950 -O3 -o tools/microbench/bin/pk_rate tools/microbench/pk_rate.hip
#include <hip/hip_runtime.h>
#include <cstdio>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)
typedef float f2 __attribute__((ext_vector_type(2)));

constexpr int ITERS = 2048;

#define BODY16(STMT) STMT(0) STMT(1) STMT(2) STMT(3) STMT(4) STMT(5) STMT(6) STMT(7) \
                     STMT(8) STMT(9) STMT(10) STMT(11) STMT(12) STMT(13) STMT(14) STMT(15)

template <int OP>
__global__ void __launch_bounds__(64) k_rate(float* out, float a, float b) {
    f2 acc[16];
    const float x = threadIdx.x * 1e-3f;
#pragma unroll
    for (int i = 0; i < 16; i++) acc[i] = f2{x + i, x - i};
    const double sab = __builtin_bit_cast(double, f2{a, b});
    // per-lane copies (VGPR operands)
    float va = a + threadIdx.x * 0.0f;
    f2 vab = f2{a, b} + f2{threadIdx.x * 0.0f, 0.0f};
    double vd = (double)a + threadIdx.x * 0.0;
    double dacc[16];
#pragma unroll
    for (int i = 0; i < 16; i++) dacc[i] = x + i;
    const unsigned long long c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < ITERS; it++) {
#define S_PKMUL(i) asm volatile("v_pk_mul_f32 %0, %1, %0 op_sel_hi:[0,1]" : "+v"(acc[i]) : "s"(sab));
#define S_PKADD(i) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(acc[i]) : "v"(acc[(i + 8) & 15]));
#define S_PKFMA(i) asm volatile("v_pk_fma_f32 %0, %1, %0, %0 op_sel_hi:[0,1,1]" : "+v"(acc[i]) : "s"(sab));
#define S_MUL(i) asm volatile("v_mul_f32 %0, %1, %0" : "+v"(acc[i].x) : "s"(a));
#define S_ADD(i) asm volatile("v_add_f32 %0, %0, %1" : "+v"(acc[i].x) : "v"(acc[(i + 8) & 15].x));
#define S_FMA(i) asm volatile("v_fmac_f32 %0, %1, %0" : "+v"(acc[i].x) : "s"(a));
#define S_MUL2(i) asm volatile("v_mul_f32 %0, %2, %0\n\tv_mul_f32 %1, %2, %1" : "+v"(acc[i].x), "+v"(acc[i].y) : "s"(a));
#define S_MULV(i) asm volatile("v_mul_f32 %0, %1, %0" : "+v"(acc[i].x) : "v"(va));
#define S_PKMULV(i) asm volatile("v_pk_mul_f32 %0, %1, %0 op_sel_hi:[0,1]" : "+v"(acc[i]) : "v"(vab));
#define S_FMA64S(i) asm volatile("v_fma_f64 %0, %1, %0, %0" : "+v"(dacc[i]) : "s"(sab));
#define S_FMA64V(i) asm volatile("v_fma_f64 %0, %1, %0, %0" : "+v"(dacc[i]) : "v"(vd));
#define S_ADD64S(i) asm volatile("v_add_f64 %0, %0, %1" : "+v"(dacc[i]) : "s"(sab));
#define S_ADD64V(i) asm volatile("v_add_f64 %0, %0, %1" : "+v"(dacc[i]) : "v"(vd));
#define S_CVT(i) asm volatile("v_cvt_f32_i32_sdwa %0, sext(%1) dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1" : "=v"(acc[i].x) : "v"(acc[(i + 8) & 15].y));
        if (OP == 0) { BODY16(S_PKMUL) }
        if (OP == 1) { BODY16(S_PKADD) }
        if (OP == 2) { BODY16(S_PKFMA) }
        if (OP == 3) { BODY16(S_MUL) }
        if (OP == 4) { BODY16(S_ADD) }
        if (OP == 5) { BODY16(S_FMA) }
        if (OP == 6) { BODY16(S_MUL2) }
        if (OP == 7) { BODY16(S_MULV) }
        if (OP == 8) { BODY16(S_PKMULV) }
        if (OP == 9) { BODY16(S_FMA64S) }
        if (OP == 10) { BODY16(S_FMA64V) }
        if (OP == 11) { BODY16(S_ADD64S) }
        if (OP == 12) { BODY16(S_ADD64V) }
        if (OP == 13) { BODY16(S_CVT) }
    }
    float s = 0.0f;
#pragma unroll
    for (int i = 0; i < 16; i++) s += acc[i].x + acc[i].y + (float)dacc[i];
    out[blockIdx.x * 64 + threadIdx.x] = s;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        // shader clock over the wave's loop: s_memtime (core clock) over s_memrealtime (100 MHz)
        const unsigned long long c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
        out[0] = (float)((double)(c1 - c0) / (double)(r1 - r0) * 100.0);   // MHz
    }
}

int main() {
    hipDeviceProp_t p;
    CHECK(hipGetDeviceProperties(&p, 0));
    const int cus = p.multiProcessorCount;
    const double mhz = p.clockRate / 1e3;
    float* d;
    CHECK(hipMalloc(&d, sizeof(float) * 64 * cus * 4 * 16));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    const char* names[] = {"v_pk_mul_f32 (s op)", "v_pk_add_f32", "v_pk_fma_f32 (s op)", "v_mul_f32 (s op)",
                           "v_add_f32", "v_fmac_f32 (s op)", "2x v_mul_f32 (I, Q)", "v_mul_f32 (v op)",
                           "v_pk_mul_f32 (v op)", "v_fma_f64 (s op)", "v_fma_f64 (v op)", "v_add_f64 (s op)",
                           "v_add_f64 (v op)", "v_cvt_f32_i32_sdwa"};
    void (*ks[])(float*, float, float) = {k_rate<0>, k_rate<1>, k_rate<2>, k_rate<3>, k_rate<4>, k_rate<5>, k_rate<6>,
                                          k_rate<7>, k_rate<8>, k_rate<9>, k_rate<10>, k_rate<11>, k_rate<12>, k_rate<13>};
    const int instr_per_iter[] = {16, 16, 16, 16, 16, 16, 32, 16, 16, 16, 16, 16, 16, 16};
    printf("%d CUs, max clock %.0f MHz; cycles per wave instruction per SIMD at that clock\n", cus, mhz);
    float mhz_meas = 0.0f;
    for (int op = 0; op < 14; op++) {
        for (int wps : {1, 2, 4, 8}) {
            const int grid = cus * 4 * wps;
            hipLaunchKernelGGL(ks[op], dim3(grid), dim3(64), 0, 0, d, 0.999f, 1.001f);
            CHECK(hipEventRecord(e0));
            hipLaunchKernelGGL(ks[op], dim3(grid), dim3(64), 0, 0, d, 0.999f, 1.001f);
            CHECK(hipEventRecord(e1));
            CHECK(hipEventSynchronize(e1));
            float ms = 0.0f;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            const double instr_per_simd = (double)wps * ITERS * instr_per_iter[op];
            const double cyc = ms * 1e-3 * mhz * 1e6 / instr_per_simd;
            CHECK(hipMemcpy(&mhz_meas, d, sizeof(float), hipMemcpyDeviceToHost));
            printf("%-22s waves/SIMD %d: %.3f ms, %.2f cycles per instruction per SIMD (%.2f at the measured %.0f MHz)\n",
                   names[op], wps, ms, cyc, cyc * mhz_meas / mhz, mhz_meas);
        }
    }
    CHECK(hipFree(d));
    return 0;
}
