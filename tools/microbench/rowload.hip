// rowload.hip -- the PLL's memory access pattern at 1, 2 and 4 waves per CU (four waves
// per CU). Each lane pair of k_pll reads its own rows: per 16-step chunk 4 float4 loads of x (a row per
// lane), 8 double2 loads of rx (a row per pair) and 4 float4 stores of t (a row per pair), one chunk
// ahead, between ~690 VALU. A wave instruction of that pattern touches 32-64 distinct 128-B lines.
// This kernel replays it on independent f64 fma chains (8 chains, 43 fmas per step) with the PLL's
// register footprint (one wave per SIMD, one-wave workgroups, per_cu of them per CU) in two layouts:
//   rows:  the PLL's (row stride 7352 elements, as the library pads)
//   tiled: the same bytes with a 16-byte piece of each lane side by side ([piece][lane]): one wave
//          instruction reads 1 KiB contiguous
// and reports shader cycles per step of one wave, and the same with the loads and stores left out.
//   hipcc --offload-arch=gfx950 -O3 tools/microbench/rowload.hip -o tools/microbench/bin/rowload
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

constexpr int C = 16, NSTEP = 7328, STRIDE = 7352, FMAS = 43;

// MODE 0: rows, 1: tiled, 2: no memory traffic
template <int MODE>
__global__ __launch_bounds__(64) void k_row(const float* __restrict__ x, const double* __restrict__ rx,
                                            float* __restrict__ t, unsigned long long* rec, double b, double c) {
    asm volatile("" ::: "v255", "a31");
    const int lane = threadIdx.x, wave = blockIdx.x;
    const long lg = (long)wave * 64 + lane;           // this lane's x row
    const long pg = lg >> 1;                          // this pair's rx and t rows
    double a[8];
#pragma unroll
    for (int k = 0; k < 8; k++) a[k] = lane + k;
    float xb[2][C];
    double rb[2][C];
    auto xaddr = [&](int i) -> const float4* {        // the float4 holding x[i..i+3] of this lane
        if (MODE == 0) return reinterpret_cast<const float4*>(x + lg * STRIDE + i);
        return reinterpret_cast<const float4*>(x) + ((long)(i / 4) * gridDim.x + wave) * 64 + lane;
    };
    auto raddr = [&](int i) -> const double2* {       // rx[i..i+1] of this pair
        if (MODE == 0) return reinterpret_cast<const double2*>(rx + pg * STRIDE + i);
        return reinterpret_cast<const double2*>(rx) + ((long)(i / 2) * gridDim.x + wave) * 32 + (lane >> 1);
    };
    auto taddr = [&](int i) -> float4* {
        if (MODE == 0) return reinterpret_cast<float4*>(t + pg * STRIDE + i);
        return reinterpret_cast<float4*>(t) + ((long)(i / 4) * gridDim.x + wave) * 32 + (lane >> 1);
    };
    auto load = [&](int u, int i0) {
        if (MODE == 2) {
#pragma unroll
            for (int k = 0; k < C; k++) { xb[u][k] = (float)k; rb[u][k] = k; }
            return;
        }
#pragma unroll
        for (int k = 0; k < C / 4; k++) {
            const float4 v = *xaddr(i0 + 4 * k);
            xb[u][4 * k] = v.x; xb[u][4 * k + 1] = v.y; xb[u][4 * k + 2] = v.z; xb[u][4 * k + 3] = v.w;
        }
#pragma unroll
        for (int k = 0; k < C / 2; k++) {
            const double2 v = *raddr(i0 + 2 * k);
            rb[u][2 * k] = v.x; rb[u][2 * k + 1] = v.y;
        }
    };
    load(0, 0);
    load(1, C);
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int c0 = 0; c0 < NSTEP / C; c0 += 2) {
#pragma unroll
        for (int u = 0; u < 2; u++) {
            float tv[C];
#pragma unroll
            for (int j = 0; j < C; j++) {
                a[j & 7] += (double)xb[u][j] * rb[u][j] * 1e-300;
#pragma unroll
                for (int f = 0; f < FMAS - 1; f++) a[(j + f) & 7] = __builtin_fma(a[(j + f) & 7], b, c);
                tv[j] = (float)a[j & 7];
            }
            const int i0 = (c0 + u) * C;
            if (MODE != 2) {   // both lanes of a pair, as the PLL
#pragma unroll
                for (int k = 0; k < C / 4; k++) *taddr(i0 + 4 * k) = make_float4(tv[4 * k], tv[4 * k + 1], tv[4 * k + 2], tv[4 * k + 3]);
            } else if (MODE == 2 && tv[0] == 1234.5f) {
                a[0] = 0.0;
            }
            const int nx = min(c0 + u + 2, NSTEP / C - 1) * C;
            load(u, nx);
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < 8; k++) s += a[k];
    if (s == 12345.678) t[lane] = (float)s;
    if (lane == 0) rec[wave] = t1 - t0;
}

template <int MODE>
int run(const char* name, int per_cu, int ncu, const float* x, const double* rx, float* t, unsigned long long* rec) {
    const int grid = per_cu * ncu;
    for (int rep = 0; rep < 2; rep++) {
        hipLaunchKernelGGL(k_row<MODE>, dim3(grid), dim3(64), 0, 0, x, rx, t, rec, 1.0000001, 1e-9);
        CHECK(hipDeviceSynchronize());
    }
    std::vector<unsigned long long> h(grid);
    CHECK(hipMemcpy(h.data(), rec, grid * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    double sum = 0.0, mx = 0.0;
    for (unsigned long long v : h) { sum += (double)v; mx = mx > (double)v ? mx : (double)v; }
    std::printf("{\"layout\": \"%s\", \"waves_per_cu\": %d, \"cycles_per_step\": %.1f, \"max\": %.1f}\n", name, per_cu,
                sum / grid / NSTEP, mx / NSTEP);
    return 0;
}

int main() {
    int ncu = 0;
    CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    const size_t lanes = 4 * (size_t)ncu * 64;        // at 4 waves per CU
    float *x = nullptr, *t = nullptr;
    double* rx = nullptr;
    unsigned long long* rec = nullptr;
    CHECK(hipMalloc(&x, lanes * STRIDE * sizeof(float)));
    CHECK(hipMalloc(&rx, lanes / 2 * STRIDE * sizeof(double)));
    CHECK(hipMalloc(&t, lanes / 2 * STRIDE * sizeof(float)));
    CHECK(hipMalloc(&rec, 4 * (size_t)ncu * sizeof(unsigned long long)));
    CHECK(hipMemset(x, 0, lanes * STRIDE * sizeof(float)));
    CHECK(hipMemset(rx, 0, lanes / 2 * STRIDE * sizeof(double)));
    for (int per_cu : {1, 2, 4}) {
        if (run<0>("rows (the PLL's)", per_cu, ncu, x, rx, t, rec)) return 1;
        if (run<1>("tiled (16-byte pieces side by side)", per_cu, ncu, x, rx, t, rec)) return 1;
        if (run<2>("no loads or stores", per_cu, ncu, x, rx, t, rec)) return 1;
    }
    CHECK(hipFree(x));
    CHECK(hipFree(rx));
    CHECK(hipFree(t));
    CHECK(hipFree(rec));
    return 0;
}
