// vbank.hip -- VGPR bank conflicts on gfx950: the same stream of independent f64 adds / fmas with
// operand registers chosen in the same bank (register index mod 4) or in different banks, one wave
// alone on its SIMD; cycles per instruction from s_memtime.
//   hipcc --offload-arch=gfx950 -O3 tools/microbench/vbank.hip -o tools/microbench/bin/vbank
#include <hip/hip_runtime.h>
#include <cstdio>

#define R8(x) x x x x x x x x
// 8 independent accumulators v[40:41] .. v[54:55] (banks 0,1 / 2,3 alternate), operand registers fixed
#define ADD_CONF "v_add_f64 v[40:41], v[40:41], v[60:61]\n v_add_f64 v[42:43], v[42:43], v[62:63]\n v_add_f64 v[44:45], v[44:45], v[60:61]\n v_add_f64 v[46:47], v[46:47], v[62:63]\n v_add_f64 v[48:49], v[48:49], v[60:61]\n v_add_f64 v[50:51], v[50:51], v[62:63]\n v_add_f64 v[52:53], v[52:53], v[60:61]\n v_add_f64 v[54:55], v[54:55], v[62:63]\n"
#define ADD_FREE "v_add_f64 v[40:41], v[40:41], v[62:63]\n v_add_f64 v[42:43], v[42:43], v[60:61]\n v_add_f64 v[44:45], v[44:45], v[62:63]\n v_add_f64 v[46:47], v[46:47], v[60:61]\n v_add_f64 v[48:49], v[48:49], v[62:63]\n v_add_f64 v[50:51], v[50:51], v[60:61]\n v_add_f64 v[52:53], v[52:53], v[62:63]\n v_add_f64 v[54:55], v[54:55], v[60:61]\n"
#define FMA_A "v_fma_f64 v[40:41], v[40:41], v[62:63], v[64:65]\n v_fma_f64 v[42:43], v[42:43], v[60:61], v[66:67]\n v_fma_f64 v[44:45], v[44:45], v[62:63], v[64:65]\n v_fma_f64 v[46:47], v[46:47], v[60:61], v[66:67]\n v_fma_f64 v[48:49], v[48:49], v[62:63], v[64:65]\n v_fma_f64 v[50:51], v[50:51], v[60:61], v[66:67]\n v_fma_f64 v[52:53], v[52:53], v[62:63], v[64:65]\n v_fma_f64 v[54:55], v[54:55], v[60:61], v[66:67]\n"
#define FMA_B "v_fma_f64 v[40:41], v[40:41], v[60:61], v[64:65]\n v_fma_f64 v[42:43], v[42:43], v[62:63], v[66:67]\n v_fma_f64 v[44:45], v[44:45], v[60:61], v[64:65]\n v_fma_f64 v[46:47], v[46:47], v[62:63], v[66:67]\n v_fma_f64 v[48:49], v[48:49], v[60:61], v[64:65]\n v_fma_f64 v[50:51], v[50:51], v[62:63], v[66:67]\n v_fma_f64 v[52:53], v[52:53], v[60:61], v[64:65]\n v_fma_f64 v[54:55], v[54:55], v[62:63], v[66:67]\n"
#define CLOB "v40","v41","v42","v43","v44","v45","v46","v47","v48","v49","v50","v51","v52","v53","v54","v55","v60","v61","v62","v63","v64","v65","v66","v67"

template <int K>
__global__ __launch_bounds__(64) void k_bank(unsigned long long* cyc, int outer) {
    asm volatile("v_mov_b32 v60, 0\n v_mov_b32 v61, 0x3ff00000\n v_mov_b32 v62, 0\n v_mov_b32 v63, 0x3ff00000\n"
                 "v_mov_b32 v64, 0\n v_mov_b32 v65, 0\n v_mov_b32 v66, 0\n v_mov_b32 v67, 0\n" ::: CLOB);
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int o = 0; o < outer; o++) {
        if (K == 0) asm volatile(R8(ADD_CONF) ::: CLOB);
        if (K == 1) asm volatile(R8(ADD_FREE) ::: CLOB);
        if (K == 2) asm volatile(R8(FMA_A) ::: CLOB);
        if (K == 3) asm volatile(R8(FMA_B) ::: CLOB);
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int K>
void run(const char* name, unsigned long long* cyc) {
    const int outer = 4096;
    hipLaunchKernelGGL(k_bank<K>, dim3(256), dim3(64), 0, 0, cyc, outer);
    hipDeviceSynchronize();
    hipLaunchKernelGGL(k_bank<K>, dim3(256), dim3(64), 0, 0, cyc, outer);
    hipDeviceSynchronize();
    unsigned long long h[256];
    hipMemcpy(h, cyc, sizeof h, hipMemcpyDeviceToHost);
    double s = 0;
    for (auto v : h) s += (double)v;
    std::printf("{\"case\": \"%s\", \"cycles_per_instruction\": %.3f}\n", name, s / 256 / (outer * 64.0));
}

int main() {
    unsigned long long* cyc = nullptr;
    hipMalloc(&cyc, 256 * sizeof(unsigned long long));
    run<0>("v_add_f64 acc + const, const in the accumulator's bank (0/1 with 0/1)", cyc);
    run<1>("v_add_f64 acc + const, const in the other bank pair", cyc);
    run<2>("v_fma_f64 acc*c1+c2: src0/src1/src2 banks all different pairs where possible (A)", cyc);
    run<3>("v_fma_f64 acc*c1+c2: src0 and src1 in the same pair (B)", cyc);
    return 0;
}
