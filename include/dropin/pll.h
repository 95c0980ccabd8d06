// pll.h (drop-in) -- pllblock_args and fmpll (reference include/pll.h:10-20) on the MI355X kernels.
#ifndef SDR_DROPIN_PLL_H
#define SDR_DROPIN_PLL_H

#include <cmath>
#include <complex>
#include <iostream>
#include <vector>

// Field order and types of the reference struct; layout-identical to sdr_pll_state (sdr_amd.h).
struct pllblock_args {
    float feedbackI;
    float feedbackQ;
    float integrator;
    float phaseEst;
    double trigOffset;
    float lastCarrier;
};

// pllOut must hold pllIn.size()+1 samples; pllOut[0] takes the previous call's last sample.
void fmpll(const std::vector<float> &pllIn, float freq, float Fs, std::vector<float> &pllOut,
           pllblock_args &block, float ncoScale = 1.0, float phaseAdjust = 0.0, float normBandwidth = 0.01);

#endif
