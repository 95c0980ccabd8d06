// Microbenchmark: can the f32 matrix cores supply the exact front end's tap products?
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o tools/microbench/bin/mfma_products tools/microbench/mfma_products.hip
// The reference's FIR (filter.cpp:115) rounds every product fl(h*x) and then every sum. An f32 MFMA
// with C = 0 and K = 1 computes D = RN(a*b + 0) = fl(a*b) if it rounds to nearest even like the VALU;
// the adds then stay on the VALU, in tap order, and the products run on the matrix pipe beside them.
// Part 1 ("exact"): v_mfma_f32_{4x4x1_16b, 16x16x1_4b, 32x32x1_2b}_f32 on random operands (full-range
// f32 and the front end's shape: taps/128 times int8 samples); the host finds each output's (A lane, B
// lane) pair on the first wave (the layout) and then checks every output bit for bit against fl(a*b).
// Part 2 ("rate"): cycles per wave instruction per SIMD, MFMA alone, VALU adds alone, and the FIR-shaped
// mix (4 MFMA 4x4x1 + 16 v_add_f32 per sample) from one and several waves per SIMD.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CHECK(x)                                                                              \
    do {                                                                                      \
        hipError_t e_ = (x);                                                                  \
        if (e_ != hipSuccess) {                                                               \
            std::fprintf(stderr, "HIP error %s at line %d\n", hipGetErrorString(e_), __LINE__); \
            std::exit(1);                                                                     \
        }                                                                                     \
    } while (0)

typedef float v4f __attribute__((ext_vector_type(4)));
typedef float v16f __attribute__((ext_vector_type(16)));
typedef float v32f __attribute__((ext_vector_type(32)));

// ---- part 1: products ---------------------------------------------------------------------------
template <int SHAPE>   // 0: 4x4x1_16b (4 outputs per lane), 1: 16x16x1_4b (16), 2: 32x32x1_2b (32)
__global__ __launch_bounds__(64) void k_prod(const float* a, const float* b, float* d) {
    const int l = threadIdx.x;
    const float av = a[blockIdx.x * 64 + l], bv = b[blockIdx.x * 64 + l];
    if (SHAPE == 0) {
        const v4f r = __builtin_amdgcn_mfma_f32_4x4x1f32(av, bv, v4f{0, 0, 0, 0}, 0, 0, 0);
        for (int i = 0; i < 4; i++) d[(blockIdx.x * 64 + l) * 4 + i] = r[i];
    } else if (SHAPE == 1) {
        v16f z = {};
        const v16f r = __builtin_amdgcn_mfma_f32_16x16x1f32(av, bv, z, 0, 0, 0);
        for (int i = 0; i < 16; i++) d[(blockIdx.x * 64 + l) * 16 + i] = r[i];
    } else {
        v32f z = {};
        const v32f r = __builtin_amdgcn_mfma_f32_32x32x1f32(av, bv, z, 0, 0, 0);
        for (int i = 0; i < 32; i++) d[(blockIdx.x * 64 + l) * 32 + i] = r[i];
    }
}

static uint64_t g_rng = 0x9E3779B97F4A7C15ull;
static uint32_t rnd() {
    g_rng ^= g_rng << 13;
    g_rng ^= g_rng >> 7;
    g_rng ^= g_rng << 17;
    return (uint32_t)(g_rng >> 11);
}
static float bits(uint32_t u) {
    float f;
    std::memcpy(&f, &u, 4);
    return f;
}
static uint32_t ubits(float f) {
    uint32_t u;
    std::memcpy(&u, &f, 4);
    return u;
}

static void part_exact(int shape, int kind) {
    const int per = shape == 0 ? 4 : shape == 1 ? 16 : 32;
    const int waves = 2048;
    const size_t n = (size_t)waves * 64;
    std::vector<float> ha(n), hb(n), hd(n * per);
    for (size_t i = 0; i < n; i++) {
        if (kind == 0) {   // full-range normal f32 operands whose product stays normal
            ha[i] = bits((rnd() & 0x807FFFFFu) | ((uint32_t)(100 + rnd() % 55) << 23));
            hb[i] = bits((rnd() & 0x807FFFFFu) | ((uint32_t)(100 + rnd() % 55) << 23));
        } else {           // the front end: tap/128 (random 24-bit mantissa, |h| in [2^-14, 2^-3]) x int8
            ha[i] = bits((rnd() & 0x807FFFFFu) | ((uint32_t)(113 + rnd() % 11) << 23));
            hb[i] = (float)((int)(rnd() % 256) - 128);
        }
    }
    float *da, *db, *dd;
    CHECK(hipMalloc(&da, n * 4));
    CHECK(hipMalloc(&db, n * 4));
    CHECK(hipMalloc(&dd, n * per * 4));
    CHECK(hipMemcpy(da, ha.data(), n * 4, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(db, hb.data(), n * 4, hipMemcpyHostToDevice));
    if (shape == 0) hipLaunchKernelGGL(k_prod<0>, dim3(waves), dim3(64), 0, 0, da, db, dd);
    if (shape == 1) hipLaunchKernelGGL(k_prod<1>, dim3(waves), dim3(64), 0, 0, da, db, dd);
    if (shape == 2) hipLaunchKernelGGL(k_prod<2>, dim3(waves), dim3(64), 0, 0, da, db, dd);
    CHECK(hipDeviceSynchronize());
    CHECK(hipMemcpy(hd.data(), dd, n * per * 4, hipMemcpyDeviceToHost));
    CHECK(hipFree(da));
    CHECK(hipFree(db));
    CHECK(hipFree(dd));
    // layout from wave 0: for every (lane, reg) the unique (A lane, B lane) whose exact product matches
    std::vector<int> la(64 * per, -1), lb(64 * per, -1);
    int unresolved = 0;
    for (int l = 0; l < 64; l++)
        for (int r = 0; r < per; r++) {
            const float v = hd[(size_t)l * per + r];
            int hits = 0;
            for (int x = 0; x < 64; x++)
                for (int y = 0; y < 64; y++) {
                    volatile float p = ha[x] * hb[y];
                    if (ubits(p) == ubits(v) && v != 0.0f) {
                        if (!hits) {
                            la[l * per + r] = x;
                            lb[l * per + r] = y;
                        }
                        hits++;
                    }
                }
            if (hits != 1) unresolved++;
        }
    // every wave checked with wave 0's layout
    long long mism = 0, total = 0, ulp1 = 0;
    for (int w = 0; w < waves; w++)
        for (int l = 0; l < 64; l++)
            for (int r = 0; r < per; r++) {
                const int x = la[l * per + r], y = lb[l * per + r];
                if (x < 0) continue;
                volatile float p = ha[(size_t)w * 64 + x] * hb[(size_t)w * 64 + y];
                const float v = hd[((size_t)w * 64 + l) * per + r];
                total++;
                if (ubits(p) != ubits(v)) {
                    mism++;
                    if (std::llabs((long long)ubits(p) - (long long)ubits(v)) == 1) ulp1++;
                }
            }
    std::printf("{\"part\": \"exact\", \"shape\": \"%s\", \"operands\": \"%s\", \"layout_unresolved\": %d, "
                "\"layout_lane0\": [",
                shape == 0 ? "4x4x1_16b" : shape == 1 ? "16x16x1_4b" : "32x32x1_2b",
                kind == 0 ? "random f32" : "tap/128 x int8", unresolved);
    for (int r = 0; r < per; r++) std::printf("%s[%d, %d]", r ? ", " : "", la[r], lb[r]);
    std::printf("], \"layout_lane5\": [");
    for (int r = 0; r < per; r++) std::printf("%s[%d, %d]", r ? ", " : "", la[5 * per + r], lb[5 * per + r]);
    std::printf("], \"products\": %lld, \"mismatches\": %lld, \"off_by_1ulp\": %lld}\n", total, mism, ulp1);
    std::fflush(stdout);
}

// ---- part 2: rates ------------------------------------------------------------------------------
constexpr int ITERS = 1024;

template <int MODE>
__global__ __launch_bounds__(64) void k_rate(float* out, float a, float b) {
    const float x = threadIdx.x * 1e-3f;
    v4f m[8];
    v16f m16[2];
    v32f m32;
#pragma unroll
    for (int i = 0; i < 8; i++) m[i] = v4f{x, x + 1, x + 2, x + i};
#pragma unroll
    for (int i = 0; i < 2; i++)
#pragma unroll
        for (int k = 0; k < 16; k++) m16[i][k] = x + k + i;
#pragma unroll
    for (int k = 0; k < 32; k++) m32[k] = x + k;
    float s[16];
#pragma unroll
    for (int i = 0; i < 16; i++) s[i] = x + i;
    const float av = a + x, bv = b - x;
    const unsigned long long c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < ITERS; it++) {
        if (MODE == 0 || MODE == 2) {   // 8 independent 4x4x1_16b (C = the chain's previous D)
#pragma unroll
            for (int i = 0; i < (MODE == 0 ? 8 : 4); i++) m[i] = __builtin_amdgcn_mfma_f32_4x4x1f32(av, bv, m[i], 0, 0, 0);
        }
        if (MODE == 1 || MODE == 2) {   // 16 independent v_add_f32, VGPR operands
#pragma unroll
            for (int i = 0; i < 16; i++) asm volatile("v_add_f32 %0, %0, %1" : "+v"(s[i]) : "v"(s[(i + 8) & 15]));
        }
        if (MODE == 3) {
#pragma unroll
            for (int i = 0; i < 2; i++) m16[i] = __builtin_amdgcn_mfma_f32_16x16x1f32(av, bv, m16[i], 0, 0, 0);
        }
        if (MODE == 4) m32 = __builtin_amdgcn_mfma_f32_32x32x1f32(av, bv, m32, 0, 0, 0);
        if (MODE == 5) {   // the current exact FIR's pair: 8 v_pk_mul_f32 + 8 v_pk_add_f32 per sample
            typedef float f2 __attribute__((ext_vector_type(2)));
#pragma unroll
            for (int i = 0; i < 8; i++) {
                f2 p = f2{s[i], s[i + 8]};
                asm volatile("v_pk_mul_f32 %0, %1, %0" : "+v"(p) : "v"(f2{av, bv}));
                asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(p) : "v"(f2{bv, av}));
                s[i] = p.x;
                s[i + 8] = p.y;
            }
        }
        if (MODE == 6) {   // FIR-shaped: 4 MFMA (products) and 16 adds of the previous sample's products
#pragma unroll
            for (int i = 0; i < 4; i++) m[4 + i] = m[i];
#pragma unroll
            for (int i = 0; i < 4; i++) m[i] = __builtin_amdgcn_mfma_f32_4x4x1f32(av, s[i], v4f{0, 0, 0, 0}, 0, 0, 0);
#pragma unroll
            for (int i = 0; i < 16; i++) asm volatile("v_add_f32 %0, %0, %1" : "+v"(s[i]) : "v"(m[4 + (i >> 2)][i & 3]));
        }
    }
    float t = 0.0f;
#pragma unroll
    for (int i = 0; i < 8; i++) t += m[i][0] + m[i][3];
#pragma unroll
    for (int i = 0; i < 16; i++) t += s[i] + m16[i & 1][i] + m32[i] + m32[i + 16];
    out[blockIdx.x * 64 + threadIdx.x] = t;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        const unsigned long long c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
        out[0] = (float)((double)(c1 - c0) / (double)(r1 - r0) * 100.0);   // MHz
    }
}

int main(int argc, char** argv) {
    const bool only_rate = argc > 1 && std::strcmp(argv[1], "rate") == 0;
    if (!only_rate) {
        for (int shape = 0; shape < 3; shape++)
            for (int kind = 0; kind < 2; kind++) part_exact(shape, kind);
    }
    hipDeviceProp_t p;
    CHECK(hipGetDeviceProperties(&p, 0));
    const int cus = p.multiProcessorCount;
    float* d;
    CHECK(hipMalloc(&d, sizeof(float) * 64 * cus * 4 * 8));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    const char* names[] = {"8x mfma 4x4x1_16b", "16x v_add_f32", "4x mfma 4x4x1 + 16x v_add_f32",
                           "2x mfma 16x16x1_4b", "1x mfma 32x32x1_2b", "8x (v_pk_mul_f32 + v_pk_add_f32)",
                           "FIR-shaped: 4x mfma 4x4x1 (C=0) + 16x v_add_f32 of their products"};
    void (*ks[])(float*, float, float) = {k_rate<0>, k_rate<1>, k_rate<2>, k_rate<3>, k_rate<4>, k_rate<5>, k_rate<6>};
    for (int op = 0; op < 7; op++)
        for (int wps : {1, 2, 4, 8}) {
            const int grid = cus * 4 * wps;
            hipLaunchKernelGGL(ks[op], dim3(grid), dim3(64), 0, 0, d, 0.999f, 1.001f);
            CHECK(hipEventRecord(e0));
            hipLaunchKernelGGL(ks[op], dim3(grid), dim3(64), 0, 0, d, 0.999f, 1.001f);
            CHECK(hipEventRecord(e1));
            CHECK(hipEventSynchronize(e1));
            float ms = 0.0f, mhz = 0.0f;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            CHECK(hipMemcpy(&mhz, d, sizeof(float), hipMemcpyDeviceToHost));
            const double cyc_per_iter = ms * 1e-3 * mhz * 1e6 / ((double)wps * ITERS);
            std::printf("{\"part\": \"rate\", \"body\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.4f, \"mhz\": %.0f, "
                        "\"cycles_per_iteration_per_simd\": %.2f}\n",
                        names[op], wps, ms, mhz, cyc_per_iter);
            std::fflush(stdout);
        }
    CHECK(hipFree(d));
    return 0;
}
