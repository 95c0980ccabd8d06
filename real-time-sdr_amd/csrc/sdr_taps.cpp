// sdr_taps.cpp -- host-side tap design of libsdr_amd.so (runs once per context, on the CPU).
//
// The filters are part of the reference's per-thread setup, not of the per-block hot path; the
// kernels only consume the taps. Each formula keeps the reference's operand types so the taps are
// bit-identical (compiled with -ffp-contract=off, no fast-math):
//   impulseResponseLPF  src/filter.cpp:13-29 (4-arg) and :33-50 (5-arg, integer gain u)
//   impulseResponseBPF  src/filter.cpp:55-71 (integer (num_taps-1)/2 in the sinc argument, :66)
//   impulseResponseAPF  src/filter.cpp:73-78
//   impulseResponseRRC  src/filter.cpp:80-102
#include <cmath>
#include <cstddef>

#include "sdr_amd.h"

#pragma clang fp contract(off)

namespace {
constexpr double kPi = 3.14159265358979323846;  // include/dy4.h:13
}

extern "C" int sdr_impulse_response_lpf(float Fs, float Fc, unsigned short num_taps, float* h) {
    if (!h || num_taps == 0) return SDR_E_INVALID;
    const float cutoff = Fc / (Fs / 2.0);
    const double centre = (num_taps - 1.0) / 2.0;
    for (int i = 0; i < num_taps; i++) {
        float v;
        if (i == centre) {
            v = cutoff;
        } else {
            const double arg = kPi * cutoff * (i - centre);
            v = cutoff * std::sin(arg) / (kPi * cutoff * (i - centre));
        }
        const double w = std::sin(i * kPi / ((float)num_taps));
        v = v * w * w;
        h[i] = v;
    }
    return SDR_OK;
}

extern "C" int sdr_impulse_response_lpf_gain(float Fs, float Fc, unsigned short num_taps, int u, float* h) {
    if (!h || num_taps == 0) return SDR_E_INVALID;
    const float cutoff = Fc / (Fs / 2.0);
    const double centre = (num_taps - 1.0) / 2.0;
    for (int i = 0; i < num_taps; i++) {
        float v;
        const float gain_cut = u * cutoff;  // the reference multiplies u*cutoff in float first
        if (i == centre) {
            v = gain_cut;
        } else {
            v = gain_cut * std::sin(kPi * cutoff * (i - centre)) / (kPi * cutoff * (i - centre));
        }
        const double w = std::sin(i * kPi / ((float)num_taps));
        v = v * w * w;
        h[i] = v;
    }
    return SDR_OK;
}

extern "C" int sdr_impulse_response_bpf(float Fs, const float* Fb, unsigned short num_taps, float* h) {
    if (!h || !Fb || num_taps == 0) return SDR_E_INVALID;
    const float centre_norm = ((Fb[1] + Fb[0]) / 2) / (Fs / 2);
    const float pass_norm = ((Fb[1] - Fb[0])) / (Fs / 2);
    for (int i = 0; i < num_taps; i++) {
        float v;
        if (i == (num_taps - 1.0) / 2.0) {
            v = pass_norm;
        } else {
            const int m = i - (num_taps - 1) / 2;
            v = pass_norm * ((std::sin(kPi * (pass_norm / 2) * m)) / (kPi * (pass_norm / 2) * m));
        }
        v = v * std::cos(i * kPi * centre_norm);
        const double w = std::sin(i * kPi / ((float)num_taps));
        v = v * w * w;
        h[i] = v;
    }
    return SDR_OK;
}

extern "C" int sdr_impulse_response_apf(float gain, unsigned short num_taps, float* h) {
    if (!h || num_taps == 0) return SDR_E_INVALID;
    for (int i = 0; i < num_taps; i++) h[i] = 0.0f;
    h[(std::size_t)((num_taps - 1.0) / 2.0)] = gain;
    return SDR_OK;
}

extern "C" int sdr_impulse_response_rrc(float Fs, unsigned short num_taps, float* h) {
    if (!h || num_taps == 0) return SDR_E_INVALID;
    const float T_symbol = 1 / 2375.0;
    const float beta = 0.90;
    for (int i = 0; i < num_taps; i++) {
        const float t = (i - (float)num_taps / 2.0) / Fs;
        if (t == 0.0) {
            h[i] = 1.0 + beta * ((4.0 / kPi) - 1);
        } else if ((t == (-T_symbol / (4.0 * beta))) | (t == (T_symbol / (4.0 * beta)))) {
            h[i] = (beta / std::sqrt(2.0)) * ((1 - 2.0 / kPi) * (std::sin(kPi / (4.0 * beta)))) +
                   ((1 - 2.0 / kPi) * (std::cos(kPi / (4 * beta))));
        } else {
            const double a = 4.0 * beta * t / T_symbol;
            h[i] = (std::sin(kPi * t * (1 - beta) / T_symbol) +
                    4.0 * beta * (t / T_symbol) * std::cos(kPi * t * (1 + beta) / T_symbol)) /
                   (kPi * t * (1 - a * a) / T_symbol);
        }
    }
    return SDR_OK;
}
