// validate.cpp -- CPU validation of real-time-sdr_amd/csrc/pll_math.h against glibc libm.
// Checks that whenever the fast path reports ok, its f32 results equal RN_f32(glibc f64) -- the
// reference's values (src/pll.cpp:39,49-50) -- and measures how often the fallback is needed.
//   g++ -O2 -std=c++17 -ffp-contract=off -I real-time-sdr_amd/csrc tools/pllmath/validate.cpp -o /tmp/validate
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>

#include "pll_math.h"

static float ref_cos(float t) { return (float)std::cos((double)t); }
static float ref_sin(float t) { return (float)std::sin((double)t); }

int main(int argc, char** argv) {
    const long N = argc > 1 ? std::atol(argv[1]) : 20000000;
    std::mt19937_64 rng(12345);
    std::uniform_real_distribution<double> U(0.0, 1.0);
    long sc_ok = 0, sc_bad = 0, sc_mis = 0;
    // 1) sin/cos on f32 arguments across magnitudes 2^-30 .. 2^30 (log-uniform) and near k*pi/2
    for (long i = 0; i < N; i++) {
        float t;
        if (i % 4 == 3) {
            const double k = std::floor(U(rng) * 6.8e8);
            t = std::nextafter((float)(k * pllm::PIO2), (float)((i & 8) ? 1e10 : -1e10));
        } else {
            const double mag = std::exp2(-30.0 + 60.0 * U(rng));
            t = (float)(mag * ((i & 1) ? 1 : -1));
        }
        const pllm::SinCos r = pllm::sincos_f32(t);
        if (!r.ok) { sc_bad++; continue; }
        sc_ok++;
        if ((float)r.c != ref_cos(t) || (float)r.s != ref_sin(t)) {
            if (sc_mis < 10) std::printf("sincos MISMATCH t=%.9g c=%.17g ref=%.9g s=%.17g ref=%.9g\n", t, r.c, ref_cos(t), r.s, ref_sin(t));
            sc_mis++;
        }
    }
    std::printf("sincos: ok %ld fallback %ld (%.2e) mismatches %ld\n", sc_ok, sc_bad, (double)sc_bad / N, sc_mis);

    // 2) phase detector on realistic inputs: (eI, eQ) = x*(RN cos t, -RN sin t)
    long pd_ok = 0, pd_bad = 0, pd_mis = 0;
    for (long i = 0; i < N; i++) {
        const float t = (float)(U(rng) * std::exp2(1.0 + 28.0 * U(rng)));
        const pllm::SinCos r = pllm::sincos_f32(t);
        const float fbI = ref_cos(t), fbQ = ref_sin(t);
        float x = (float)((U(rng) - 0.5) * std::exp2(-12.0 * U(rng)));
        if (i % 1000 == 0) x = 0.0f;
        const float eI = x * fbI, eQ = x * (-fbQ);
        const pllm::Phase p = pllm::phase_detect(eI, eQ, r.c, r.s, r.mr, r.q3);
        if (!p.ok) { pd_bad++; continue; }
        pd_ok++;
        const float ref = (float)std::atan2((double)eQ, (double)eI);
        if (p.ef != ref) {
            if (pd_mis < 10) std::printf("atan2 MISMATCH t=%.9g x=%.9g e=%.17g ref=%.9g\n", t, x, p.e, ref);
            pd_mis++;
        }
    }
    std::printf("phase:  ok %ld fallback %ld (%.2e) mismatches %ld\n", pd_ok, pd_bad, (double)pd_bad / N, pd_mis);

    // 3) whole PLL trajectories (pll.cpp:34-53) with fast path + per-step fallback vs reference
    long steps = 0, diff = 0, fallbacks = 0;
    for (int sig = 0; sig < 8; sig++) {
        const float freq = (sig & 1) ? 114e3f : 19e3f, Fs = 240000.0f;
        const float bw = (sig & 1) ? 0.001f : 0.01f, nco = (sig & 1) ? 0.5f : 2.0f;
        const float Cp = 2.666, Ci = 3.555;
        const float Kp = bw * Cp, Ki = bw * bw * Ci;
        float fbI = 1, fbQ = 0, integ = 0, ph = 0, rfbI = 1, rfbQ = 0, rinteg = 0, rph = 0;
        double toff = 0, rtoff = 0;
        double c = 1, s = 0, mr = 0;
        int q3 = 0;
        const long n = N / 8;
        for (long i = 0; i < n; i++) {
            const float xin = (float)(0.1 * std::cos(2 * M_PI * (freq + 3.0 * sig) / Fs * i + sig) +
                                      0.01 * (U(rng) - 0.5));
            // reference
            {
                const float eI = xin * rfbI, eQ = xin * (-rfbQ);
                const float e = std::atan2((double)eQ, (double)eI);
                rinteg = rinteg + Ki * e;
                rph = rph + Kp * e + rinteg;
                rtoff += 1.0;
                const float t = 2 * 3.14159265358979323846 * (freq / Fs) * rtoff + rph;
                rfbI = std::cos((double)t);
                rfbQ = std::sin((double)t);
            }
            // fast
            {
                const float eI = xin * fbI, eQ = xin * (-fbQ);
                const pllm::Phase p = pllm::phase_detect(eI, eQ, c, s, mr, q3);
                float e;
                if (p.ok) e = p.ef; else { e = (float)std::atan2((double)eQ, (double)eI); fallbacks++; }
                integ = integ + Ki * e;
                ph = ph + Kp * e + integ;
                toff += 1.0;
                const float t = (float)(2 * 3.14159265358979323846 * (freq / Fs) * toff + (double)ph);
                const pllm::SinCos r = pllm::sincos_f32(t);
                c = r.c; s = r.s; mr = r.mr; q3 = r.q3;
                if (r.ok) { fbI = (float)r.c; fbQ = (float)r.s; }
                else { fbI = (float)std::cos((double)t); fbQ = (float)std::sin((double)t); fallbacks++; }
            }
            steps++;
            if (fbI != rfbI || fbQ != rfbQ || ph != rph || integ != rinteg) {
                if (diff < 5) std::printf("PLL diverged sig %d step %ld\n", sig, i);
                diff++;
                fbI = rfbI; fbQ = rfbQ; ph = rph; integ = rinteg;   // resync and keep counting
            }
        }
        (void)nco;
    }
    std::printf("pll:    steps %ld diverged %ld fallbacks %ld (%.2e per step)\n", steps, diff, fallbacks,
                (double)fallbacks / steps);
    return (sc_mis || pd_mis || diff) ? 1 : 0;
}
