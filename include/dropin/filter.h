// filter.h (drop-in) -- the reference's FIR design and convolution interface (include/filter.h:18-24),
// implemented by libsdr_host.so on the MI355X kernels of libsdr_amd.so (include/sdr_amd.h).
#ifndef SDR_DROPIN_FILTER_H
#define SDR_DROPIN_FILTER_H

#include <cmath>
#include <iostream>
#include <vector>

void impulseResponseLPF(float Fs, float Fc, unsigned short num_taps, std::vector<float> &h);
void impulseResponseLPF(float Fs, float Fc, unsigned short num_taps, std::vector<float> &h, int u);
void impulseResponseBPF(float Fs, float *Fb, unsigned short num_taps, std::vector<float> &h);
void impulseResponseAPF(float gain, unsigned short num_taps, std::vector<float> &h);
void impulseResponseRRC(float Fs, unsigned short num_taps, std::vector<float> &h);
// y = decimate-by-D FIR of x; state holds the previous block's tail (>= h.size()-1 samples)
void convolveFIR(std::vector<float> &y, const std::vector<float> &x, const std::vector<float> &h,
                 std::vector<float> &state, int D);
// y = U/D rational resampler of x (phase restarts every call, like filter.cpp:131)
void convolveFIR(std::vector<float> &y, const std::vector<float> &x, const std::vector<float> &h,
                 std::vector<float> &state, int U, int D);

#endif
