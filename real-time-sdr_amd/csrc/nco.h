// nco.h -- the PLL's NCO output (pll.cpp:52): carrier = RN32(cos((double)(t * ncoScale + phaseAdjust)))
// of an f32 phase t, with the reference's f32 rounding of the argument and glibc's f64 cos.
// The fast path is pll_math.h cos_rn_f32 (correctly rounded to f32 with a proof per value: the PLL
// step's reduction and kernels, one of them selected by the quadrant); a value it cannot prove is
// recomputed in double-double (pll_math.h dd_sincos_f32 returns glibc's RN64).
// Shared by k_nco_out (sdr_pll.hip) and the fused post stages (sdr_kernels.hip).
#pragma once

#include <hip/hip_runtime.h>

#include "pll_math.h"

namespace sdrk {

// glibc's cos of pll.cpp:52 for the arguments the fast path cannot decide (out of line: rare)
static __device__ __noinline__ float nco_cos_slow(float a) {
    double s, c;
    if (__builtin_fabs(a) <= 3.4028234663852886e38f)
        pllm::dd_sincos_f32(a, &s, &c);
    else
        sincos((double)a, &s, &c);   // inf / NaN: every libm agrees
    return (float)c;
}

static __device__ __forceinline__ float nco_carrier(float t, float ncoScale, float phaseAdjust) {
    const float a = t * ncoScale + phaseAdjust;   // two f32 roundings, as the reference
    bool ok;
    const float c = pllm::cos_rn_f32(a, ok);
    return ok ? c : nco_cos_slow(a);
}

}  // namespace sdrk
