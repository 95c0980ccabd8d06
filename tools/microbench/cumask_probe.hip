// Microbenchmark: how a HIP CU mask (hipExtStreamCreateWithCUMask) maps to (XCC, SE, CU) on MI355X,
// and how many one-wave workgroups of a launch a masked stream actually runs at once.
//   hipcc --offload-arch=gfx950 -O3 -o tools/microbench/bin/cumask_probe tools/microbench/cumask_probe.hip
// Part A ("bit"): one stream per mask bit, one wave each; the wave records HW_ID and XCC_ID.
// Part B ("cap"): masks [0, n) for several n; a launch of n * per_cu one-wave workgroups whose LDS
// allows per_cu of them per CU (the persistent PLL's residency claim). Every wave stamps its start,
// holds ~HOLD_US, stamps its end and exits (bounded: nothing waits on anything). The waves that start
// after the earliest end were not resident together with the rest: the claim "n * per_cu fit" is true
// only when that count is 0.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <vector>

#define CHECK(x)                                                                              \
    do {                                                                                      \
        hipError_t e_ = (x);                                                                  \
        if (e_ != hipSuccess) {                                                               \
            std::fprintf(stderr, "HIP error %s at line %d\n", hipGetErrorString(e_), __LINE__); \
            std::exit(1);                                                                     \
        }                                                                                     \
    } while (0)

constexpr int HOLD_US = 300;

__global__ __launch_bounds__(64) void k_where(unsigned long long* rec) {
    uint32_t hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    if (threadIdx.x == 0) {
        rec[2 * blockIdx.x] = hw;
        rec[2 * blockIdx.x + 1] = xcc;
    }
}

// LDS_BYTES sets how many workgroups fit one CU (160 KiB of LDS per CU)
template <int LDS_BYTES>
__global__ __launch_bounds__(64) void k_hold(unsigned long long* rec) {
    __shared__ uint32_t pad[LDS_BYTES / 4];
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    pad[threadIdx.x] = (uint32_t)t0;
    unsigned long long t = t0;
    while (t - t0 < (unsigned long long)HOLD_US * 100ull) {   // 100 MHz clock, bounded
        __builtin_amdgcn_s_sleep(8);
        t = __builtin_amdgcn_s_memrealtime();
    }
    uint32_t hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    __syncthreads();
    if (threadIdx.x == 0) {
        rec[4 * blockIdx.x] = t0;
        rec[4 * blockIdx.x + 1] = t;
        rec[4 * blockIdx.x + 2] = hw;
        rec[4 * blockIdx.x + 3] = xcc | ((unsigned long long)pad[5] << 32);   // keeps the LDS allocated
    }
}

static hipStream_t masked(int ncu, int first, int n) {
    std::vector<uint32_t> m((ncu + 31) / 32, 0u);
    for (int c = first; c < first + n; c++) m[c / 32] |= 1u << (c % 32);
    hipStream_t s;
    CHECK(hipExtStreamCreateWithCUMask(&s, (uint32_t)m.size(), m.data()));
    return s;
}

static void part_bits(int ncu, unsigned long long* d) {
    std::printf("{\"part\": \"bit\", \"map\": [");
    for (int b = 0; b < ncu; b++) {
        hipStream_t s = masked(ncu, b, 1);
        hipLaunchKernelGGL(k_where, dim3(1), dim3(64), 0, s, d);
        CHECK(hipStreamSynchronize(s));
        unsigned long long h[2];
        CHECK(hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost));
        CHECK(hipStreamDestroy(s));
        const unsigned hw = (unsigned)h[0];
        std::printf("%s[%d, %u, %u, %u, %u]", b ? ", " : "", b, (unsigned)h[1] & 15u, (hw >> 13) & 7u, (hw >> 12) & 1u,
                    (hw >> 8) & 15u);
    }
    std::printf("], \"fields\": [\"bit\", \"xcc\", \"se\", \"sh\", \"cu\"]}\n");
}

template <int LDS_BYTES>
static void part_cap(int ncu, unsigned long long* d, int per_cu, const std::vector<int>& ns) {
    for (int n : ns) {
        hipStream_t s = masked(ncu, 0, n);
        const int grid = n * per_cu;
        hipLaunchKernelGGL(k_hold<LDS_BYTES>, dim3(grid), dim3(64), 0, s, d);
        CHECK(hipStreamSynchronize(s));
        std::vector<unsigned long long> h(4 * (size_t)grid);
        CHECK(hipMemcpy(h.data(), d, h.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
        CHECK(hipStreamDestroy(s));
        unsigned long long first_end = ~0ull, t_min = ~0ull, t_max = 0;
        for (int g = 0; g < grid; g++) {
            first_end = std::min(first_end, h[4 * g + 1]);
            t_min = std::min(t_min, h[4 * g]);
            t_max = std::max(t_max, h[4 * g + 1]);
        }
        int late = 0;
        std::map<int, int> per_se_first, per_cu_first;   // (xcc, se) -> waves started before the first end
        for (int g = 0; g < grid; g++) {
            const unsigned hw = (unsigned)h[4 * g + 2];
            const int key = (int)(((unsigned)h[4 * g + 3] & 15u) * 8 + ((hw >> 13) & 7u));
            const int ckey = key * 32 + (int)(((hw >> 12) & 1u) * 16 + ((hw >> 8) & 15u));
            if (h[4 * g] >= first_end) late++;
            else {
                per_se_first[key]++;
                per_cu_first[ckey]++;
            }
        }
        std::map<int, int> se_hist;
        for (auto& kv : per_se_first) se_hist[kv.second]++;
        int cus_used = (int)per_cu_first.size(), max_on_cu = 0;
        for (auto& kv : per_cu_first) max_on_cu = std::max(max_on_cu, kv.second);
        std::printf("{\"part\": \"cap\", \"mask_cus\": %d, \"per_cu_lds\": %d, \"waves\": %d, \"late_waves\": %d, "
                    "\"span_us\": %.1f, \"ses_used\": %d, \"cus_used\": %d, \"max_waves_on_a_cu\": %d, "
                    "\"first_round_waves_per_se_hist\": {",
                    n, per_cu, grid, late, (t_max - t_min) / 100.0, (int)per_se_first.size(), cus_used, max_on_cu);
        bool first = true;
        for (auto& kv : se_hist) {
            std::printf("%s\"%d\": %d", first ? "" : ", ", kv.first, kv.second);
            first = false;
        }
        std::printf("}}\n");
        std::fflush(stdout);
    }
}

int main() {
    hipDeviceProp_t p;
    CHECK(hipGetDeviceProperties(&p, 0));
    const int ncu = p.multiProcessorCount;
    unsigned long long* d;
    CHECK(hipMalloc(&d, sizeof(unsigned long long) * 4 * 4096));
    part_bits(ncu, d);
    const std::vector<int> ns = {8, 16, 24, 32, 40, 48, 56, 64, 80, 96, 128, 192};
    part_cap<72 * 1024>(ncu, d, 2, ns);   // two per CU (72 KiB each)
    part_cap<100 * 1024>(ncu, d, 1, ns);  // one per CU
    part_cap<36 * 1024>(ncu, d, 4, ns);   // four per CU
    CHECK(hipFree(d));
    return 0;
}
