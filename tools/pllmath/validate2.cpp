// validate2.cpp -- CPU validation of the v2 PLL step of pll_math.h (pll_rx, sincos2_f32,
// base_angle, phase_detect2) against glibc libm, i.e. against the reference's own arithmetic
// (src/pll.cpp:34-53). Checks that every fast result the kernel would accept equals
// RN_f32(glibc f64), records max |Y/X| (the analytic bound is 2^-23) and the fallback rates.
//   g++ -O2 -std=c++17 -ffp-contract=off -I real-time-sdr_amd/csrc tools/pllmath/validate2.cpp -o /tmp/validate2
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>

#include "pll_math.h"

int main(int argc, char** argv) {
    const long N = argc > 1 ? std::atol(argv[1]) : 20000000;
    std::mt19937_64 rng(777);
    std::uniform_real_distribution<double> U(0.0, 1.0);
    // 1) sincos2 vs libm over log-uniform magnitudes and near multiples of pi/2
    long sc_ok = 0, sc_bad = 0, sc_mis = 0;
    for (long i = 0; i < N; i++) {
        float t;
        if (i % 4 == 3) {
            const double k = std::floor(U(rng) * 6.8e8);
            t = std::nextafter((float)(k * pllm::PIO2), (float)((i & 8) ? 1e10 : -1e10));
        } else {
            t = (float)(std::exp2(-30.0 + 60.0 * U(rng)) * ((i & 1) ? 1 : -1));
        }
        if (!(std::fabs(t) < pllm::T_MAX)) continue;
        const pllm::SinCos2 r = pllm::sincos2_f32(t);
        if (!(r.tie > 128u)) { sc_bad++; continue; }
        sc_ok++;
        if ((float)r.c != (float)std::cos((double)t) || (float)r.s != (float)std::sin((double)t)) {
            if (sc_mis < 10) std::printf("sincos2 MISMATCH t=%.9g\n", t);
            sc_mis++;
        }
        // the reduction's quadrant bookkeeping: -t == -q pi/2 + mr (mod 2pi)
        const double back = std::remainder(-(double)t - (-(double)(int32_t)r.q * pllm::PIO2 + r.mr), pllm::TWO_PI);
        if (std::fabs(back) > 1e-9 * std::max(1.0, std::fabs((double)t) * 1e-6)) {
            if (sc_mis < 10) std::printf("reduction MISMATCH t=%.9g back=%g\n", t, back);
            sc_mis++;
        }
    }
    std::printf("sincos2: ok %ld fallback %ld (%.2e) mismatches %ld\n", sc_ok, sc_bad, (double)sc_bad / N, sc_mis);

    // 1b) the reduced-frame sincos_rn (k_pll) on the same argument mix: accepted roundings, rotated
    // by i^q, must equal RN_f32(glibc cos t), RN_f32(glibc sin t)
    {
        long ok = 0, bad = 0, mis = 0;
        std::mt19937_64 rng2(4242);
        for (long i = 0; i < N; i++) {
            float t;
            if (i % 4 == 3) {
                const double k = std::floor(U(rng2) * 6.8e8);
                t = std::nextafter((float)(k * pllm::PIO2), (float)((i & 8) ? 1e10 : -1e10));
            } else {
                t = (float)(std::exp2(-30.0 + 60.0 * U(rng2)) * ((i & 1) ? 1 : -1));
            }
            if (!(std::fabs(t) < pllm::T_MAX)) continue;
            const pllm::SinCosRN r = pllm::sincos_rn(t);
            if (!(r.tie > pllm::TIE_MIN)) { bad++; continue; }
            ok++;
            float c = (float)r.cr, sn = (float)r.sr;
            pllm::rot_q(1u - r.nq1, c, sn);
            if (c != (float)std::cos((double)t) || sn != (float)std::sin((double)t)) {
                if (mis < 10) std::printf("sincos_rn MISMATCH t=%.9g\n", t);
                mis++;
            }
        }
        std::printf("sincos_rn: ok %ld fallback %ld (%.2e) mismatches %ld\n", ok, bad, (double)bad / N, mis);
        sc_mis += mis;
    }

    // 2) phase detector v2 on (eI, eQ) = x (RN cos t, -RN sin t), base from the same t
    long pd_ok = 0, pd_bad = 0, pd_mis = 0;
    double dmax = 0.0;
    for (long i = 0; i < N; i++) {
        const float t = (float)((U(rng) - 0.5) * std::exp2(1.0 + 28.0 * U(rng)));
        const pllm::SinCos2 r = pllm::sincos2_f32(t);
        const double c = std::cos((double)t), s = std::sin((double)t);   // accurate c, s
        const float fbI = (float)c, fbQ = (float)s;
        float x = (float)((U(rng) - 0.5) * std::exp2(-40.0 * U(rng) * U(rng)));
        if (i % 1000 == 0) x = 0.0f;
        if (i % 1000 == 1) x = 1e-30f;
        if (i % 1000 == 2) x = -std::ldexp(1.0f, -60);
        const float eI = x * fbI, eQ = x * (-fbQ);
        const double rx = pllm::pll_rx(x);
        const double base = pllm::base_angle(pllm::lo_word(rx), r.q, r.b, r.mr);
        const pllm::Phase2 p = pllm::phase_detect2(eI, eQ, c, s, rx, base);
        const double Y = (double)eI * s + (double)eQ * c, X = (double)eI * c - (double)eQ * s;
        if (std::isfinite(rx) && X != 0.0) dmax = std::max(dmax, std::fabs(Y / X));
        const bool ok = std::fabs(p.e) < pllm::PI - 0x1p-30 && p.split == 0u;
        if (!ok) { pd_bad++; continue; }
        pd_ok++;
        const float ref = (float)std::atan2((double)eQ, (double)eI);
        if (p.ef != ref) {
            if (pd_mis < 10) std::printf("atan2 MISMATCH t=%.9g x=%.9g e=%.17g ref=%.9g\n", t, x, p.e, ref);
            pd_mis++;
        }
    }
    std::printf("phase2: ok %ld fallback %ld (%.2e) mismatches %ld max|Y/X| 2^%.2f\n", pd_ok, pd_bad,
                (double)pd_bad / N, pd_mis, std::log2(dmax));

    // 3) whole trajectories: v2 fast step (with per-step libm fallback) vs the reference loop
    long steps = 0, diff = 0, fb_e = 0, fb_sc = 0;
    for (int sig = 0; sig < 8; sig++) {
        const float freq = (sig & 1) ? 114e3f : 19e3f, Fs = 240000.0f;
        const float bw = (sig & 1) ? 0.001f : 0.01f;
        const float Cp = 2.666, Ci = 3.555;
        const float Kp = bw * Cp, Ki = bw * bw * Ci;
        const double w = 2 * 3.14159265358979323846 * (freq / Fs);
        // a consistent state: feedback = RN_f32 of cos/sin of the previous step's trigArg
        // (pll.cpp:47-50); the kernel checks this and falls back to libm when it does not hold
        double toff = sig >= 4 ? 3.0e6 : 0.0, rtoff = toff;
        const float t0 = (float)(w * toff);
        float fbI = (float)std::cos((double)t0), fbQ = (float)std::sin((double)t0), integ = 0, ph = 0;
        float rfbI = fbI, rfbQ = fbQ, rinteg = 0, rph = 0;
        // carried from the previous step: sincos of t_prev = w*toff + ph
        pllm::SinCos2 sc = pllm::sincos2_f32((float)(w * toff + (double)ph));
        double c = std::cos((double)(float)(w * toff + (double)ph)), s = std::sin((double)(float)(w * toff + (double)ph));
        const long n = N / 8;
        for (long i = 0; i < n; i++) {
            const float xin = (float)(0.1 * std::cos(2 * M_PI * (freq + 3.0 * sig) / Fs * i + sig) +
                                      0.01 * (U(rng) - 0.5));
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
            {
                const float eI = xin * fbI, eQ = xin * (-fbQ);
                const double rx = pllm::pll_rx(xin);
                const double base = pllm::base_angle(pllm::lo_word(rx), sc.q, sc.b, sc.mr);
                const pllm::Phase2 p = pllm::phase_detect2(eI, eQ, c, s, rx, base);
                float e = p.ef;
                if (!(std::fabs(p.e) < pllm::PI - 0x1p-30 && p.split == 0u)) {
                    e = (float)std::atan2((double)eQ, (double)eI);
                    fb_e++;
                }
                integ = integ + Ki * e;
                ph = ph + Kp * e + integ;
                toff += 1.0;
                const float t = (float)(w * toff + (double)ph);
                sc = pllm::sincos2_f32(t);
                c = sc.c; s = sc.s;
                fbI = (float)c; fbQ = (float)s;
                if (!(sc.tie > pllm::TIE_MIN)) {
                    c = std::cos((double)t); s = std::sin((double)t);
                    fbI = (float)c; fbQ = (float)s;
                    fb_sc++;
                }
            }
            steps++;
            if (fbI != rfbI || fbQ != rfbQ || ph != rph || integ != rinteg) {
                if (diff < 5) std::printf("PLL diverged sig %d step %ld\n", sig, i);
                diff++;
                fbI = rfbI; fbQ = rfbQ; ph = rph; integ = rinteg;
            }
        }
    }
    std::printf("pll2:   steps %ld diverged %ld fallbacks e %ld (%.2e) sincos %ld (%.2e)\n", steps, diff, fb_e,
                (double)fb_e / steps, fb_sc, (double)fb_sc / steps);

    // 4) reduced-frame trajectories (k_pll): feedback carried as RN(cos r), RN(sin r) and q
    long rsteps = 0, rdiff = 0, rfb_e = 0, rfb_sc = 0;
    for (int sig = 0; sig < 8; sig++) {
        const float freq = (sig & 1) ? 114e3f : 19e3f, Fs = 240000.0f;
        const float bw = (sig & 1) ? 0.001f : 0.01f;
        const float Cp = 2.666, Ci = 3.555;
        const float Kp = bw * Cp, Ki = bw * bw * Ci;
        const double w = 2 * 3.14159265358979323846 * (freq / Fs);
        double toff = sig >= 4 ? 3.0e6 : 0.0, rtoff = toff;
        const float t0 = (float)(w * toff);
        float rfbI = (float)std::cos((double)t0), rfbQ = (float)std::sin((double)t0), rinteg = 0, rph = 0;
        // kernel state: pll_load
        float integ = 0, ph = 0;
        pllm::SinCosRN sc = pllm::sincos_rn(t0);
        float fI0 = (float)sc.cr, fQ0 = (float)sc.sr;
        {
            float a = fI0, b = fQ0;
            pllm::rot_q(1u - sc.nq1, a, b);
            if (a != rfbI || b != rfbQ) std::printf("load: inconsistent state\n");
        }
        double cr = sc.cr, sr = sc.sr, mr = -sc.r;
        uint32_t nq1 = sc.nq1, bsg = sc.b;
        const long n = N / 8;
        for (long i = 0; i < n; i++) {
            const float xin = (float)(0.1 * std::cos(2 * M_PI * (freq + 3.0 * sig) / Fs * i + sig) +
                                      0.01 * (U(rng) - 0.5));
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
            {
                const float eI0 = xin * fI0, eQ0 = xin * (-fQ0);
                const double rx = pllm::pll_rx(xin);
                const double base = pllm::base_angle_n(pllm::lo_word(rx), nq1, bsg, mr);
                const pllm::Phase2 p = pllm::phase_detect_r(eI0, eQ0, cr, sr, rx, base);
                float e = p.ef;
                if (!(std::fabs(p.e) < pllm::PI - 0x1p-30 && p.split == 0u)) {
                    float a = eI0, b = -eQ0;
                    pllm::rot_q(1u - nq1, a, b);
                    e = (float)std::atan2((double)(-b), (double)a);
                    rfb_e++;
                }
                integ = integ + Ki * e;
                ph = ph + Kp * e + integ;
                toff += 1.0;
                const float t = (float)(w * toff + (double)ph);
                sc = pllm::sincos_rn(t);
                cr = sc.cr; sr = sc.sr; mr = -sc.r; nq1 = sc.nq1; bsg = sc.b;
                fI0 = (float)cr; fQ0 = (float)sr;
                if (!(sc.tie > pllm::TIE_MIN)) {
                    double cv = std::cos((double)t), sv = std::sin((double)t);
                    pllm::rot_q(nq1 - 1u, cv, sv);
                    cr = cv; sr = sv;
                    fI0 = (float)cr; fQ0 = (float)sr;
                    rfb_sc++;
                }
            }
            rsteps++;
            float fbI = fI0, fbQ = fQ0;
            pllm::rot_q(1u - nq1, fbI, fbQ);
            if (fbI != rfbI || fbQ != rfbQ || ph != rph || integ != rinteg) {
                if (rdiff < 5) std::printf("reduced-frame PLL diverged sig %d step %ld\n", sig, i);
                rdiff++;
                break;
            }
        }
    }
    std::printf("pllR:   steps %ld diverged %ld fallbacks e %ld (%.2e) sincos %ld (%.2e)\n", rsteps, rdiff, rfb_e,
                (double)rfb_e / rsteps, rfb_sc, (double)rfb_sc / rsteps);
    diff += rdiff;
    return (sc_mis || pd_mis || diff) ? 1 : 0;
}
