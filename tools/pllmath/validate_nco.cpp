// validate_nco.cpp -- CPU check of the NCO's fast cosine (pll_math.h cos_rn_f32, used by k_stereo_out,
// k_rds_mix and k_nco_out for pll.cpp:52) against glibc: every value the fast path accepts must equal
// RN_f32(glibc cos((double)a)). Arguments: log-uniform magnitudes in [2^-30, 2^30), f32 neighbours
// of multiples of pi/2 (the reduction's worst cases), and the NCO's own arguments t * 2 and t * 0.5
// of PLL-like phases. Prints one JSON line; exit status 1 on any mismatch.
//   g++ -O2 -std=c++17 -ffp-contract=off -I real-time-sdr_amd/csrc tools/pllmath/validate_nco.cpp
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>

#include "pll_math.h"

int main(int argc, char** argv) {
    const long N = argc > 1 ? std::atol(argv[1]) : 10000000;
    std::mt19937_64 rng(9151);
    std::uniform_real_distribution<double> U(0.0, 1.0);
    long ok = 0, slow = 0, mis = 0;
    for (long i = 0; i < N; i++) {
        float a;
        switch (i % 4) {
            case 0: {
                const double k = std::floor(U(rng) * 6.8e8);
                a = std::nextafter((float)(k * pllm::PIO2), (float)((i & 8) ? 1e10 : -1e10));
                break;
            }
            case 1: {   // stereo: t * 2 (ncoScale 2, stereo.cpp:77), t a 19 kHz phase after up to ~1 h
                const float t = (float)(2 * pllm::PI * 19e3 / 240e3 * std::floor(U(rng) * 8.6e8) + U(rng) - 0.5);
                a = t * 2.0f + 0.0f;
                break;
            }
            case 2: {   // RDS: t * 0.5 (rds.cpp:119), a 114 kHz phase
                const float t = (float)(2 * pllm::PI * 114e3 / 240e3 * std::floor(U(rng) * 3.5e8) + U(rng) - 0.5);
                a = t * 0.5f + 0.0f;
                break;
            }
            default:
                a = (float)(std::exp2(-30.0 + 60.0 * U(rng)) * ((i & 1) ? 1 : -1));
        }
        bool acc = false;
        const float c = pllm::cos_rn_f32(a, acc);
        if (!acc) { slow++; continue; }
        ok++;
        if (c != (float)std::cos((double)a)) {
            if (mis < 10) std::fprintf(stderr, "MISMATCH a=%.9g fast=%.9g glibc=%.9g\n", a, c, (float)std::cos((double)a));
            mis++;
        }
    }
    std::printf("{\"n\": %ld, \"accepted\": %ld, \"fallback\": %ld, \"f32_mismatch\": %ld}\n", N, ok, slow, mis);
    return mis ? 1 : 0;
}
