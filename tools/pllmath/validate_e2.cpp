// validate_e2.cpp -- measured absolute error of the v2 phase detector's e (pll_math.h sincos2_f32 +
// base_angle + phase_detect2, the c and s of the sine/cosine kernels, not exact ones) against
// atan2l(eQ, eI) in 64-bit-mantissa long double, and of glibc's f64 atan2 (the reference's value,
// src/pll.cpp) against the same: the two terms of the e bracket EPS_ABS_E2.
//   g++ -O2 -std=c++17 -ffp-contract=off -I real-time-sdr_amd/csrc tools/pllmath/validate_e2.cpp -o /tmp/validate_e2
//   /tmp/validate_e2 [N]
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>

#include "pll_math.h"

int main(int argc, char** argv) {
    const long N = argc > 1 ? std::atol(argv[1]) : 20000000;
    std::mt19937_64 rng(2045);
    std::uniform_real_distribution<double> U(0.0, 1.0);
    long used = 0;
    long double emax = 0.0L, gmax = 0.0L, smax = 0.0L;
    for (long i = 0; i < N; i++) {
        const float t = (float)((U(rng) - 0.5) * std::exp2(1.0 + 28.0 * U(rng)));
        const pllm::SinCos2 r = pllm::sincos2_f32(t);
        // the reference's own cos/sin of t, rounded to f32, make (eI, eQ) (pll.cpp)
        const float fbI = (float)std::cos((double)t), fbQ = (float)std::sin((double)t);
        const float x = (float)((U(rng) - 0.5) * std::exp2(-40.0 * U(rng) * U(rng)));
        if (!(std::fabs(x) >= 0x1p-60f)) continue;
        const float eI = x * fbI, eQ = x * (-fbQ);
        const double rx = pllm::pll_rx(x);
        const double base = pllm::base_angle(pllm::lo_word(rx), r.q, r.b, r.mr);
        const pllm::Phase2 p = pllm::phase_detect2(eI, eQ, r.c, r.s, rx, base);
        if (!(std::fabs(p.e) < pllm::PI - 0x1p-30)) continue;
        used++;
        const long double ex = atan2l((long double)eQ, (long double)eI);
        const long double err = std::fabs((long double)p.e - ex);
        const long double gerr = std::fabs((long double)std::atan2((double)eQ, (double)eI) - ex);
        if (err > emax) emax = err;
        if (gerr > gmax) gmax = gerr;
        // the kernels' own part: c, s against cos, sin of t (absolute, |c|, |s| <= 1)
        const long double sc = std::fmax(std::fabs((long double)r.c - cosl((long double)t)),
                                         std::fabs((long double)r.s - sinl((long double)t)));
        if (sc > smax) smax = sc;
    }
    std::printf("{\"n\": %ld, \"log2_e_err\": %.3f, \"log2_glibc_err\": %.3f, \"log2_cs_err\": %.3f, "
                "\"log2_sum\": %.3f, \"log2_eps\": %.1f}\n",
                used, (double)std::log2(emax), (double)std::log2(gmax), (double)std::log2(smax),
                (double)std::log2(emax + gmax), std::log2(pllm::EPS_ABS_E2));
    return 0;
}
