// validate_e3.cpp -- the e bracket (pll_math.h EPS_ABS_E2) on the phase detector the kernels ship:
// the lane-pair step of sdr_pll.hip pll_step_split, evaluated here operation for operation on the
// host. Per sample (t, x): the previous step's sincos_rn(t) gives cos r, sin r, the quadrant and
// the reduced argument; lane A forms g = RN32(-x RN32(sin r)) (= eQ0) and q = g cos r, lane B
// g = RN32(x RN32(cos r)) (= eI0) and q = g sin r; Y = qA + qB, e = fma(Y, RN(1/x)', base_angle_n).
// Reference (src/pll.cpp:36-39): eI = RN32(x RN32(cos t)), eQ = RN32(x * -RN32(sin t)) with glibc's
// cos / sin, and e_ref = glibc atan2(eQ, eI). Reports the largest |e - atan2l| and |e_ref - atan2l|
// (64-bit mantissa), their sum against EPS_ABS_E2, and the samples whose bracket test passes
// (RN32(e - eps) == RN32(e) == RN32(e + eps)) but whose RN32(e) differs from RN32(e_ref): must be 0.
// Samples whose own cos/sin roundings the kernel would not accept (tie key) are skipped, as the
// kernel redoes those steps.
//   g++ -O2 -std=c++17 -ffp-contract=off -I real-time-sdr_amd/csrc tools/pllmath/validate_e3.cpp -o /tmp/validate_e3
//   /tmp/validate_e3 [N]
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>

#include "pll_math.h"

int main(int argc, char** argv) {
    const long N = argc > 1 ? std::atol(argv[1]) : 20000000;
    std::mt19937_64 rng(2046);
    std::uniform_real_distribution<double> U(0.0, 1.0);
    long used = 0, accepted = 0, wrong = 0;
    long double emax = 0.0L, gmax = 0.0L, dmax = 0.0L;
    for (long i = 0; i < N; i++) {
        const float t = (float)((U(rng) - 0.5) * std::exp2(1.0 + 28.0 * U(rng)));
        const float x = (float)((U(rng) - 0.5) * std::exp2(-40.0 * U(rng) * U(rng)));
        if (!(std::fabs(x) >= 0x1p-60f)) continue;
        const pllm::SinCosRN sc = pllm::sincos_rn(t);
        if (!(sc.tie > pllm::TIE_MIN)) continue;                 // the kernel redoes this step
        const float fbA = (float)sc.cr, fbB = (float)sc.sr;       // lane A: RN(cos r), lane B: RN(sin r)
        const float gA = -x * fbB, gB = x * fbA;                  // xs * partner's fb
        const double qA = (double)gA * sc.cr, qB = (double)gB * sc.sr;
        const double Y = qA + qB;
        const double rx = pllm::pll_rx(x);
        const double base = pllm::base_angle_n(pllm::lo_word(rx), sc.nq1, sc.b, -sc.r);
        const double ed = pllm::fma_(Y, rx, base);
        if (!(std::fabs(ed) < pllm::PI - 0x1p-30)) continue;      // the kernel's e range test
        used++;
        const float fbI = (float)std::cos((double)t), fbQ = (float)std::sin((double)t);
        const float eI = x * fbI, eQ = x * (-fbQ);
        const double eref = std::atan2((double)eQ, (double)eI);
        const long double ex = atan2l((long double)eQ, (long double)eI);
        const long double err = std::fabs((long double)ed - ex), gerr = std::fabs((long double)eref - ex);
        const long double d = std::fabs((long double)ed - (long double)eref);
        if (err > emax) emax = err;
        if (gerr > gmax) gmax = gerr;
        if (d > dmax) dmax = d;
        const float e = (float)ed;
        const bool ok = (float)(ed - pllm::EPS_ABS_E2) == e && (float)(ed + pllm::EPS_ABS_E2) == e;
        if (ok) {
            accepted++;
            if (e != (float)eref) wrong++;
        }
    }
    std::printf("{\"n\": %ld, \"accepted\": %ld, \"wrong\": %ld, \"log2_e_err\": %.3f, \"log2_glibc_err\": %.3f, "
                "\"log2_sum\": %.3f, \"log2_e_minus_ref\": %.3f, \"log2_eps\": %.1f}\n",
                used, accepted, wrong, (double)std::log2(emax), (double)std::log2(gmax),
                (double)std::log2(emax + gmax), (double)std::log2(dmax), std::log2(pllm::EPS_ABS_E2));
    return wrong == 0 ? 0 : 1;
}
