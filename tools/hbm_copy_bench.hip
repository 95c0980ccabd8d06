// HBM copy microbenchmark: which plain streaming copy reaches the best rate on this device
// (load/store cache policy, grid size, loads in flight per lane). Calibrates sdr_hbm_copy.
//   hipcc --offload-arch=gfx950 -O3 -o tools/hbm_copy_bench tools/hbm_copy_bench.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int U, bool NT>
__global__ __launch_bounds__(256) void copy_k(u32x4* __restrict__ dst, const u32x4* __restrict__ src, size_t n) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + (U - 1) * stride < n; i += U * stride) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; u++) v[u] = NT ? __builtin_nontemporal_load(src + i + u * stride) : src[i + u * stride];
#pragma unroll
        for (int u = 0; u < U; u++) {
            if (NT) __builtin_nontemporal_store(v[u], dst + i + u * stride);
            else dst[i + u * stride] = v[u];
        }
    }
    for (; i < n; i += stride) dst[i] = src[i];
}

// one element per thread, no loop (the classic float4 copy)
__global__ __launch_bounds__(256) void copy_flat(u32x4* __restrict__ dst, const u32x4* __restrict__ src, size_t n) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) dst[i] = src[i];
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("%s: %s\n", #x, hipGetErrorString(e_)); std::exit(1); } } while (0)

template <typename F>
static double time_ms(F f, int reps) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    f();
    f();
    CK(hipEventRecord(a));
    for (int r = 0; r < reps; r++) f();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    CK(hipEventDestroy(a));
    CK(hipEventDestroy(b));
    return ms / reps;
}

int main(int argc, char** argv) {
    const size_t bytes = (argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 1024ull) << 20;
    const size_t n = bytes / 16;
    void *s, *d;
    CK(hipMalloc(&s, bytes));
    CK(hipMalloc(&d, bytes));
    CK(hipMemset(s, 1, bytes));
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    auto S = static_cast<const u32x4*>(s);
    auto D = static_cast<u32x4*>(d);
    auto report = [&](const char* name, double ms) {
        std::printf("{\"variant\": \"%s\", \"MiB\": %zu, \"ms\": %.4f, \"GBps\": %.1f}\n", name, bytes >> 20, ms,
                    2.0 * bytes / (ms * 1e-3) / 1e9);
    };
    const int reps = 20;
    report("flat", time_ms([&] { hipLaunchKernelGGL(copy_flat, dim3((n + 255) / 256), dim3(256), 0, 0, D, S, n); }, reps));
    report("hipMemcpyDtoD", time_ms([&] { CK(hipMemcpyAsync(d, s, bytes, hipMemcpyDeviceToDevice, 0)); }, reps));
    for (int wpc : {4, 8, 16, 32}) {
        char nm[64];
        const int g = cus * wpc;
        std::snprintf(nm, sizeof nm, "u4_nt_g%d", wpc);
        report(nm, time_ms([&] { hipLaunchKernelGGL((copy_k<4, true>), dim3(g), dim3(256), 0, 0, D, S, n); }, reps));
        std::snprintf(nm, sizeof nm, "u4_g%d", wpc);
        report(nm, time_ms([&] { hipLaunchKernelGGL((copy_k<4, false>), dim3(g), dim3(256), 0, 0, D, S, n); }, reps));
        std::snprintf(nm, sizeof nm, "u1_g%d", wpc);
        report(nm, time_ms([&] { hipLaunchKernelGGL((copy_k<1, false>), dim3(g), dim3(256), 0, 0, D, S, n); }, reps));
        std::snprintf(nm, sizeof nm, "u8_g%d", wpc);
        report(nm, time_ms([&] { hipLaunchKernelGGL((copy_k<8, false>), dim3(g), dim3(256), 0, 0, D, S, n); }, reps));
    }
    CK(hipFree(s));
    CK(hipFree(d));
    return 0;
}
