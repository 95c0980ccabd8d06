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
//   tools/microbench/bin/ifetch wg1    (one-wave workgroups with the PLL's register footprint, k_fma1)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <string>
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

// One-wave workgroups, per_cu of them per CU (grid = per_cu * ncu), with the PLL's register
// footprint (v255 and AGPRs in use: one wave per SIMD, as k_pll's 256 VGPRs + 18 AGPRs): the k_pll
// launch shape of DESIGN.md 5's four-waves-per-CU case, on independent f64 fma chains. Each wave
// records its HW_ID and XCC_ID beside its cycles, so placement and slowdown can be put side by side.
template <int OP>
__global__ __launch_bounds__(64) void k_fma1(double* out, unsigned long long* rec, int outer, double b, double c) {
    asm volatile("" ::: "v255", "a31");
    double a[8];
#pragma unroll
    for (int k = 0; k < 8; k++) a[k] = threadIdx.x + k;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int o = 0; o < outer; o++) {
#pragma unroll
        for (int u = 0; u < 256; u++) {
            if (OP == 0) a[u & 7] = __builtin_fma(a[u & 7], b, c);
            else asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(a[0]) : "v"(b), "v"(c));
        }
        asm volatile("" : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]),
                     "+v"(a[7]));
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    uint32_t hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < 8; k++) s += a[k];
    if (s == 12345.678) out[threadIdx.x] = s;
    if (threadIdx.x == 0) {
        rec[3 * blockIdx.x] = t1 - t0;
        rec[3 * blockIdx.x + 1] = hw;
        rec[3 * blockIdx.x + 2] = xcc;
    }
}

template <int OP>
int run1(int per_cu, int ncu, double* out, unsigned long long* rec) {
    const long NI = 1 << 21;
    const int outer = (int)(NI / 256);
    const int grid = per_cu * ncu;
    for (int rep = 0; rep < 2; rep++) {
        hipLaunchKernelGGL(k_fma1<OP>, dim3(grid), dim3(64), 0, 0, out, rec, outer, 1.0000001, 1e-9);
        CHECK(hipDeviceSynchronize());
    }
    std::vector<unsigned long long> h(3 * grid);
    CHECK(hipMemcpy(h.data(), rec, 3 * grid * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    // waves per (xcc, se, sh, cu) and per SIMD; cycles per instruction by how many waves shared the SIMD
    std::vector<int> cu_n(16 * 8 * 2 * 16, 0), simd_n(16 * 8 * 2 * 16 * 4, 0);
    auto cu_key = [&](int g) {
        const unsigned hw = (unsigned)h[3 * g + 1], x = (unsigned)h[3 * g + 2] & 15u;
        return (int)(((x * 8 + ((hw >> 13) & 7)) * 2 + ((hw >> 12) & 1)) * 16 + ((hw >> 8) & 15));
    };
    for (int g = 0; g < grid; g++) {
        cu_n[cu_key(g)]++;
        simd_n[cu_key(g) * 4 + (((unsigned)h[3 * g + 1] >> 4) & 3)]++;
    }
    double sum[5] = {}, cnt[5] = {};
    int cus = 0, shared_simds = 0, maxcu = 0;
    for (int v : cu_n) { cus += v > 0; maxcu = v > maxcu ? v : maxcu; }
    for (int v : simd_n) shared_simds += v > 1;
    for (int g = 0; g < grid; g++) {
        const int k = std::min(simd_n[cu_key(g) * 4 + (((unsigned)h[3 * g + 1] >> 4) & 3)], 4);
        sum[k] += (double)h[3 * g];
        cnt[k] += 1.0;
    }
    std::printf("{\"kernel\": \"one-wave workgroups, 1 wave/SIMD footprint\", \"op\": \"%s\", \"waves_per_cu\": %d, "
                "\"cus_used\": %d, \"max_waves_on_a_cu\": %d, \"simds_with_2plus_waves\": %d",
                OP == 0 ? "v_fma_f64, 8 chains" : "v_fma_f64, one dependent chain", per_cu, cus, maxcu, shared_simds);
    for (int k = 1; k <= 4; k++)
        if (cnt[k] > 0)
            std::printf(", \"cpi_waves_on_simd_%d\": %.3f", k, sum[k] / cnt[k] / (double)NI);
    std::printf("}\n");
    return 0;
}

int main(int argc, char** argv) {
    int ncu = 0;
    CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    double* out = nullptr;
    unsigned long long* cyc = nullptr;
    CHECK(hipMalloc(&out, 4096 * sizeof(double)));
    CHECK(hipMemset(out, 0, 4096 * sizeof(double)));
    CHECK(hipMalloc(&cyc, 4 * 1024 * sizeof(unsigned long long)));
    if (argc > 1 && std::string(argv[1]) == "wg1") {   // one-wave workgroups (k_fma1)
        unsigned long long* rec = nullptr;
        CHECK(hipMalloc(&rec, 3 * 8 * (size_t)ncu * sizeof(unsigned long long)));
        for (int per_cu : {1, 2, 4, 5, 8}) {
            if (run1<0>(per_cu, ncu, out, rec)) return 1;
            if (run1<1>(per_cu, ncu, out, rec)) return 1;
        }
        return 0;
    }
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
