// ifetch.hip -- is instruction fetch the resource four lone waves per CU share? (DESIGN.md 4a,
// profiles/r05/). Kernels with the same dynamic instruction count per wave -- 8 independent chains,
// NI instructions per wave in total -- differ in code size and instruction width:
//   straight: 2048 instructions unrolled (re-fetched every outer iteration)
//   tight:    64 instructions unrolled
// op: v_fma_f64 (8-byte VOP3), v_add_f32_e32 (4-byte VOP2), v_fma_f32 (8-byte VOP3) -- the two f32
// forms issue at the same rate, so a gap between them at 4 waves per CU is instruction bytes.
// Each wave stamps its shader cycles (s_memtime) around its loop; the host reports cycles per
// instruction for 1, 2 and 4 waves per CU: one workgroup per CU (96 KiB of dynamic LDS each) of 64,
// 128 or 256 threads, whose waves the dispatcher puts on distinct SIMDs.
//   hipcc --offload-arch=gfx950 -O3 tools/microbench/ifetch.hip -o tools/microbench/bin/ifetch
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#define CHECK(x)                                                                        \
    do {                                                                                \
        hipError_t e_ = (x);                                                            \
        if (e_ != hipSuccess) {                                                         \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));               \
            return 1;                                                                   \
        }                                                                               \
    } while (0)

template <int UNROLL, int OP, int PRIO = 0>
__global__ __launch_bounds__(256) void k_fma(double* out, unsigned long long* cyc, int outer, double b, double c) {
    if (PRIO) __builtin_amdgcn_s_setprio(3);   // as the PLL kernels
    double a[8];
    float f[8];
    const float fb = (float)b, fc = (float)c;
    unsigned sreg = 0;
    double lv = 0.0;
#pragma unroll
    for (int k = 0; k < 8; k++) { a[k] = threadIdx.x + k; f[k] = (float)a[k]; }
    extern __shared__ double lds[];              // 96 KiB: one workgroup per CU
    lds[threadIdx.x] = out[threadIdx.x];
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int o = 0; o < outer; o++) {
#pragma unroll
        for (int u = 0; u < UNROLL / 8; u++) {
#pragma unroll
            for (int k = 0; k < 8; k++) {
                if (OP == 0) a[k] = __builtin_fma(a[k], b, c);
                else if (OP == 1) asm volatile("v_add_f32_e32 %0, %1, %0" : "+v"(f[k]) : "v"(fc));
                else if (OP == 2) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(f[k]) : "v"(fb), "v"(fc));
                else if (OP == 3) {   // f32 <-> f64 conversions, two per step of the chain
                    asm volatile("v_cvt_f64_f32_e32 %0, %1" : "=v"(a[k]) : "v"(f[k]));
                    asm volatile("v_cvt_f32_f64_e32 %0, %1" : "=v"(f[k]) : "v"(a[k]));
                } else if (OP == 4) { // DPP moves (quad_perm [1,0,3,2], the PLL's lane-pair exchange)
                    asm volatile("v_mov_b32_dpp %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "+v"(f[k]));
                } else if (OP == 5) { // f64 add / mul
                    asm volatile("v_add_f64 %0, %0, %1" : "+v"(a[k]) : "v"(b));
                } else if (OP == 6) { // v_mul_f32 with a DPP source
                    asm volatile("v_mul_f32_dpp %0, %0, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "+v"(f[k]) : "v"(fb));
                } else if (OP == 7) { // v_fma_f64 with one SGPR-pair operand (the PLL's scalar constants)
                    asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(a[k]) : "s"(b), "v"(c));
                } else if (OP == 8) { // v_fma_f64 with two SGPR-pair operands (the same pair)
                    asm volatile("v_fma_f64 %0, %1, %0, %1" : "+v"(a[k]) : "s"(b));
                } else if (OP == 9) { // ONE dependent chain of v_fma_f64 (the latency, not the issue rate)
                    asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(a[0]) : "v"(b), "v"(c));
                } else if (OP == 10) {// one dependent chain of v_add_f32
                    asm volatile("v_add_f32_e32 %0, %1, %0" : "+v"(f[0]) : "v"(fc));
                } else if (OP >= 12) {
                    a[k] = __builtin_fma(a[k], b, c);
                    if (k == 0 && OP == 12 && (u % 4) == 0) {   // one 16-byte load per 32 fmas, a chunk ahead
                        const double2 v = reinterpret_cast<const double2*>(out)[(threadIdx.x + 64 * u) & 1023];
                        a[7] += v.x * 1e-300;
                    }
                    if (OP == 13) asm volatile("s_add_u32 %0, %0, 1" : "+s"(sreg) :: "scc");
                    if (OP == 14 && k == 0) { lv = lds[(threadIdx.x * 3 + u) & 4095]; a[6] += lv * 1e-300; }
                    if (OP == 15 && k == 7) {              // a wave-uniform branch per 8 fmas
                        if (__builtin_amdgcn_readfirstlane(__builtin_bit_cast(int2, a[0]).x) == 7) a[1] = 0.0;
                    }
                } else {              // one chain alternating f64 fma and f32<->f64 conversions
                    asm volatile("v_cvt_f32_f64_e32 %0, %1" : "=v"(f[0]) : "v"(a[0]));
                    asm volatile("v_cvt_f64_f32_e32 %0, %1" : "=v"(a[0]) : "v"(f[0]));
                    asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(a[0]) : "v"(b), "v"(c));
                }
            }
        }
        asm volatile("" : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]),
                     "+v"(a[7]));
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < 8; k++) s += a[k] + f[k];
    s += lds[(threadIdx.x + 1) & 255];
    if (s == 12345.678 || sreg == 77u) out[threadIdx.x] = s;   // keeps the work
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 4 + (threadIdx.x >> 6)] = t1 - t0;
}

template <int UNROLL, int OP, int PRIO = 0>
int run(const char* name, int per_cu, int ncu, double* out, unsigned long long* cyc) {
    const long NI = 1 << 21;   // fmas per wave
    const int outer = (int)(NI / UNROLL);
    const int grid = ncu;
    const size_t lds = 96 * 1024;
    CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(k_fma<UNROLL, OP, PRIO>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    CHECK(hipMemset(cyc, 0, 4 * 1024 * sizeof(unsigned long long)));
    hipLaunchKernelGGL((k_fma<UNROLL, OP, PRIO>), dim3(grid), dim3(64 * per_cu), lds, 0, out, cyc, outer, 1.0000001, 1e-9);
    CHECK(hipDeviceSynchronize());
    hipLaunchKernelGGL((k_fma<UNROLL, OP, PRIO>), dim3(grid), dim3(64 * per_cu), lds, 0, out, cyc, outer, 1.0000001, 1e-9);
    CHECK(hipDeviceSynchronize());
    std::vector<unsigned long long> h(4 * grid);
    CHECK(hipMemcpy(h.data(), cyc, 4 * grid * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    double sum = 0.0;
    for (int g = 0; g < grid; g++)
        for (int w = 0; w < per_cu; w++) sum += (double)h[4 * g + w];
    sum /= per_cu;
    const char* ops[16] = {"v_fma_f64 (8 B)", "v_add_f32_e32 (4 B)", "v_fma_f32 (8 B)",
                          "v_cvt_f64_f32 + v_cvt_f32_f64 (pairs)", "v_mov_b32_dpp", "v_add_f64", "v_mul_f32_dpp",
                          "v_fma_f64, one SGPR-pair operand", "v_fma_f64, two SGPR-pair operands",
                          "v_fma_f64, one dependent chain", "v_add_f32, one dependent chain",
                          "cvt f32, cvt f64, fma f64: one dependent chain",
                          "v_fma_f64 + a 16-byte global load per 32", "v_fma_f64 + s_add_u32 per fma",
                          "v_fma_f64 + an LDS read per 8", "v_fma_f64 + a uniform branch per 8"};
    const double per = OP == 3 ? 2.0 : OP == 11 ? 3.0 : 1.0;   // instructions per chain step
    std::printf("{\"kernel\": \"%s\", \"op\": \"%s\", \"unrolled\": %d, \"waves_per_cu\": %d, "
                "\"cycles_per_instruction\": %.3f}\n", name, ops[OP], UNROLL, per_cu, sum / grid / (double)NI / per);
    return 0;
}

int main() {
    int ncu = 0;
    CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    double* out = nullptr;
    unsigned long long* cyc = nullptr;
    CHECK(hipMalloc(&out, 4096 * sizeof(double)));
    CHECK(hipMemset(out, 0, 4096 * sizeof(double)));
    CHECK(hipMalloc(&cyc, 4 * 1024 * sizeof(unsigned long long)));
    for (int per_cu : {1, 4}) {
        if (run<2048, 0>("straight", per_cu, ncu, out, cyc)) return 1;
        if (run<64, 0>("tight", per_cu, ncu, out, cyc)) return 1;
        if (run<2048, 1>("straight", per_cu, ncu, out, cyc)) return 1;
        if (run<2048, 2>("straight", per_cu, ncu, out, cyc)) return 1;
        if (run<64, 2>("tight", per_cu, ncu, out, cyc)) return 1;
        if (run<1024, 3>("straight", per_cu, ncu, out, cyc)) return 1;
        if (run<2048, 4>("straight", per_cu, ncu, out, cyc)) return 1;
        if (run<2048, 5>("straight", per_cu, ncu, out, cyc)) return 1;
        if (run<2048, 6>("straight", per_cu, ncu, out, cyc)) return 1;
        if (run<2048, 7>("straight", per_cu, ncu, out, cyc)) return 1;
        if (run<2048, 8>("straight", per_cu, ncu, out, cyc)) return 1;
        if (run<256, 9>("dependent", per_cu, ncu, out, cyc)) return 1;
        if (run<256, 10>("dependent", per_cu, ncu, out, cyc)) return 1;
        if (run<128, 11>("dependent", per_cu, ncu, out, cyc)) return 1;
        if (run<2048, 12>("mixed", per_cu, ncu, out, cyc)) return 1;
        if (run<2048, 13>("mixed", per_cu, ncu, out, cyc)) return 1;
        if (run<2048, 14>("mixed", per_cu, ncu, out, cyc)) return 1;
        if (run<2048, 15>("mixed", per_cu, ncu, out, cyc)) return 1;
        if (run<2048, 0, 1>("straight, s_setprio 3", per_cu, ncu, out, cyc)) return 1;
        if (run<256, 9, 1>("dependent, s_setprio 3", per_cu, ncu, out, cyc)) return 1;
        if (run<128, 11, 1>("dependent, s_setprio 3", per_cu, ncu, out, cyc)) return 1;
    }
    return 0;
}
