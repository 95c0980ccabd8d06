// validate_dd.cpp -- the double-double fallbacks of pll_math.h against glibc, on the host:
// dd_sincos(t) vs glibc cos/sin and dd_atan2_f32(y, x, th0) vs glibc atan2, compared as f64 bit
// patterns (glibc returns RN64 of the exact value on all but a vanishing fraction of inputs, so any
// mismatch is either a dd error or a glibc misrounding; the f32 roundings are what the PLL uses).
// th0 is glibc's value perturbed by up to +-4 ulps, standing in for the device libm's.
//   g++ -O2 -std=c++17 -ffp-contract=off -I real-time-sdr_amd/csrc tools/pllmath/validate_dd.cpp \
//       -o /tmp/validate_dd && /tmp/validate_dd [N]
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>

#include "pll_math.h"

static double nudge(double v, int64_t u) {
    int64_t i;
    std::memcpy(&i, &v, 8);
    i += u;
    std::memcpy(&v, &i, 8);
    return v;
}

int main(int argc, char** argv) {
    const long N = argc > 1 ? std::atol(argv[1]) : 4000000;
    std::mt19937_64 rng(7);
    std::uniform_real_distribution<double> U(0.0, 1.0);
    long bad64[3] = {0, 0, 0}, bad32[3] = {0, 0, 0}, hard[3] = {0, 0, 0};
    for (long i = 0; i < N; i++) {
        const float t = (float)(U(rng) * std::exp2(30.0 * U(rng) - 2.0) * (U(rng) < 0.5 ? -1 : 1));
        double s, c;
        pllm::dd_sincos((double)t, &s, &c);
        const double gc = std::cos((double)t), gs = std::sin((double)t);
        const double got[2] = {c, s}, ref[2] = {gc, gs};
        for (int k = 0; k < 2; k++) {
            if (!pllm::f32_rounding_safe_rel64(ref[k])) hard[k]++;
            if (got[k] != ref[k]) bad64[k]++;
            if ((float)got[k] != (float)ref[k]) bad32[k]++;
        }
        const float x = (float)((U(rng) - 0.5) * std::exp2(-20.0 * U(rng)));
        const float y = (float)((U(rng) - 0.5) * std::exp2(-20.0 * U(rng)));
        const double ga = std::atan2((double)y, (double)x);
        const double a = pllm::dd_atan2_f32(y, x, nudge(ga, (int64_t)(rng() % 9) - 4));
        if (a != ga) bad64[2]++;
        if ((float)a != (float)ga) bad32[2]++;
    }
    // the inputs that matter: t whose glibc cos/sin lie within 64 f64 ulps of an f32 midpoint
    long nh = 0, hb64 = 0, hb32 = 0;
    for (long i = 0; nh < N / 8 && i < 64 * N; i++) {
        const float t = (float)(U(rng) * std::exp2(30.0 * U(rng) - 2.0));
        const double gc = std::cos((double)t);
        if (pllm::tie_distance64(gc) > 64u) continue;
        nh++;
        double s, c;
        pllm::dd_sincos((double)t, &s, &c);
        if (c != gc) hb64++;
        if ((float)c != (float)gc) hb32++;
    }
    // large arguments (|t| >= 2^30, Payne-Hanek): PLL-like 2^30..2^36 and the whole f32 range
    long nl = 0, lb64 = 0, lb32 = 0;
    for (long i = 0; i < N / 4; i++) {
        const double ex = (i & 1) ? 30.0 + 6.0 * U(rng) : 30.0 + 98.0 * U(rng);
        const float t = (float)(std::exp2(ex) * (U(rng) < 0.5 ? -1 : 1));
        double s, c;
        pllm::dd_sincos_f32(t, &s, &c);
        const double gc = std::cos((double)t), gs = std::sin((double)t);
        nl++;
        lb64 += (c != gc) + (s != gs);
        lb32 += ((float)c != (float)gc) + ((float)s != (float)gs);
    }
    std::printf("{\"large\": {\"n\": %ld, \"f64_mismatch\": %ld, \"f32_mismatch\": %ld}, ", nl, lb64, lb32);
    std::printf("\"n\": %ld, \"cos\": {\"f64_mismatch\": %ld, \"f32_mismatch\": %ld}, "
                "\"sin\": {\"f64_mismatch\": %ld, \"f32_mismatch\": %ld}, "
                "\"atan2\": {\"f64_mismatch\": %ld, \"f32_mismatch\": %ld}, "
                "\"cos_near_f32_midpoint\": {\"n\": %ld, \"f64_mismatch\": %ld, \"f32_mismatch\": %ld}}\n",
                N, bad64[0], bad32[0], bad64[1], bad32[1], bad64[2], bad32[2], nh, hb64, hb32);
    return (bad32[0] | bad32[1] | bad32[2] | hb32 | lb32) ? 1 : 0;
}
