// demod.h (drop-in) -- fmDemodNoArctan (reference include/demod.h:5) on the MI355X kernels.
#ifndef SDR_DROPIN_DEMOD_H
#define SDR_DROPIN_DEMOD_H

#include <cmath>
#include <iostream>
#include <vector>

void fmDemodNoArctan(const std::vector<float> &I, const std::vector<float> &Q, float &prev_I, float &prev_Q,
                     std::vector<float> &fm_demod);

#endif
