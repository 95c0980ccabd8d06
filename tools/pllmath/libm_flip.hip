// libm_flip.hip -- does the device libm (OCML) agree with glibc (the reference's libm) on the f64
// calls of the PLL (pll.cpp:39 atan2, :49-50 sin/cos on f32 arguments)? k_pll falls back to OCML
// only when its proven fast path cannot decide an f32 rounding, i.e. on inputs near a rounding
// boundary, where any f64 disagreement between the two libms can flip the f32 result.
// This counts, on N random PLL-like inputs, how often OCML and glibc differ in the f64 result at
// all, by how many ulps, and how often that changes the f32 rounding -- and the same for the
// double-double fallbacks that replace OCML in the kernels (pll_math.h: correctly rounded f64, so
// they differ from glibc only where glibc itself misrounds, by 1 ulp).
//   hipcc --offload-arch=gfx950 -O2 -std=c++17 -ffp-contract=off -I real-time-sdr_amd/csrc \
//         tools/pllmath/libm_flip.hip \
//         -o tools/pllmath/libm_flip && ./tools/pllmath/libm_flip [N]
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "pll_math.h"

#define CHECK(x)                                                                      \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            std::printf("HIP error %s at line %d\n", hipGetErrorString(e_), __LINE__); \
            return 1;                                                                 \
        }                                                                             \
    } while (0)

// DD: the double-double fallbacks of pll_math.h (what k_pll and k_nco_out use) instead of OCML
template <bool DD>
__global__ void k_libm(const float* t, const float* eq, const float* ei, int n, double* c, double* s, double* a) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    double sv, cv;
    if (DD)
        pllm::dd_sincos((double)t[i], &sv, &cv);
    else
        sincos((double)t[i], &sv, &cv);
    c[i] = cv;
    s[i] = sv;
    const double th = atan2((double)eq[i], (double)ei[i]);
    a[i] = DD ? pllm::dd_atan2_f32(eq[i], ei[i], th) : th;
}

static int64_t ulps(double a, double b) {
    int64_t ia, ib;
    std::memcpy(&ia, &a, 8);
    std::memcpy(&ib, &b, 8);
    return ia > ib ? ia - ib : ib - ia;
}

int main(int argc, char** argv) {
    const int N = argc > 1 ? std::atoi(argv[1]) : 4000000;
    std::mt19937_64 rng(2024);
    std::uniform_real_distribution<double> U(0.0, 1.0);
    std::vector<float> t(N), eq(N), ei(N);
    for (int i = 0; i < N; i++) {
        // trigArgs of runs from seconds to hours (|t| up to 2^26) and detector inputs x*(cos, -sin)
        t[i] = (float)(U(rng) * std::exp2(26.0 * U(rng)) * (U(rng) < 0.5 ? -1 : 1));
        const float x = (float)((U(rng) - 0.5) * 0.2);
        const float tt = (float)(U(rng) * std::exp2(22.0 * U(rng)));
        ei[i] = x * (float)std::cos((double)tt);
        eq[i] = x * (-(float)std::sin((double)tt));
    }
    float *dt, *deq, *dei;
    double *dc, *ds, *da;
    CHECK(hipMalloc(&dt, N * sizeof(float)));
    CHECK(hipMalloc(&deq, N * sizeof(float)));
    CHECK(hipMalloc(&dei, N * sizeof(float)));
    CHECK(hipMalloc(&dc, N * sizeof(double)));
    CHECK(hipMalloc(&ds, N * sizeof(double)));
    CHECK(hipMalloc(&da, N * sizeof(double)));
    CHECK(hipMemcpy(dt, t.data(), N * sizeof(float), hipMemcpyHostToDevice));
    CHECK(hipMemcpy(deq, eq.data(), N * sizeof(float), hipMemcpyHostToDevice));
    CHECK(hipMemcpy(dei, ei.data(), N * sizeof(float), hipMemcpyHostToDevice));
    std::printf("{");
    for (int dd = 0; dd < 2; dd++) {
        if (dd)
            hipLaunchKernelGGL(k_libm<true>, dim3((N + 255) / 256), dim3(256), 0, 0, dt, deq, dei, N, dc, ds, da);
        else
            hipLaunchKernelGGL(k_libm<false>, dim3((N + 255) / 256), dim3(256), 0, 0, dt, deq, dei, N, dc, ds, da);
        CHECK(hipGetLastError());
        std::vector<double> c(N), s(N), a(N);
        CHECK(hipMemcpy(c.data(), dc, N * sizeof(double), hipMemcpyDeviceToHost));
        CHECK(hipMemcpy(s.data(), ds, N * sizeof(double), hipMemcpyDeviceToHost));
        CHECK(hipMemcpy(a.data(), da, N * sizeof(double), hipMemcpyDeviceToHost));
        long d64[3] = {0, 0, 0}, d32[3] = {0, 0, 0};
        int64_t umax[3] = {0, 0, 0};
        for (int i = 0; i < N; i++) {
            const double ref[3] = {std::cos((double)t[i]), std::sin((double)t[i]),
                                   std::atan2((double)eq[i], (double)ei[i])};
            const double got[3] = {c[i], s[i], a[i]};
            for (int k = 0; k < 3; k++) {
                if (got[k] != ref[k]) {
                    d64[k]++;
                    const int64_t u = ulps(got[k], ref[k]);
                    if (u > umax[k]) umax[k] = u;
                    if ((float)got[k] != (float)ref[k]) d32[k]++;
                }
            }
        }
        std::printf("%s\"%s\": {\"n\": %d, \"cos\": {\"f64_differ\": %ld, \"max_ulp\": %lld, \"f32_differ\": %ld}, "
                    "\"sin\": {\"f64_differ\": %ld, \"max_ulp\": %lld, \"f32_differ\": %ld}, "
                    "\"atan2\": {\"f64_differ\": %ld, \"max_ulp\": %lld, \"f32_differ\": %ld}}",
                    dd ? ", " : "", dd ? "double_double" : "ocml", N, d64[0], (long long)umax[0], d32[0], d64[1],
                    (long long)umax[1], d32[1], d64[2], (long long)umax[2], d32[2]);
    }
    std::printf("}\n");
    return 0;
}
