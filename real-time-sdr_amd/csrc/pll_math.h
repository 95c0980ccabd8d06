// pll_math.h -- fast, correctly-rounded-to-f32 transcendentals for the PLL recurrence.
//
// The reference PLL (src/pll.cpp:34-53) evaluates, per sample and on f32 arguments, the f64 libm
// functions atan2 (:39), sin/cos (:49-50) and rounds each result to f32. Whenever a double
// approximation v of f(x) carries a proven error bound eps and both v-eps and v+eps round to the
// same float, that float is RN_f32(f(x)) -- which equals the reference's RN_f32(glibc f64 f(x))
// except when glibc's own <=1-ulp f64 error straddles an f32 rounding midpoint (~2^-28 per call,
// shared with any other libm). When the test fails the caller redoes the step with the f64 libm
// path (OCML), exactly as the reference computes it.
//
//  * pll_sincos: f32 t -> cos t, sin t. Cody-Waite reduction by pi/2 with a 22/22/53-bit split
//    (exact first two products for |t| < 2^30), fdlibm's k_sin kernel and a refitted degree-8
//    cos kernel on |r| <= pi/4 (relative error < 2^-51), Estrin evaluation. Also returns
//    -t mod 2pi as (q mod 4, -r).
//  * pll_phase_detect: atan2(eQ, eI) for (eI, eQ) = x*(RN(cos t), -RN(sin t)) (pll.cpp:36-39).
//    Rotating (eI, eQ) by +t with the f64 cos/sin of the previous step leaves a residual angle
//    |delta| < 2^-20, so atan2 = -t + pi*[X<0] + Y/X (mod 2pi) with no polynomial at all.
//
// Shared by the HIP kernel and the CPU validation (tools/pllmath/validate.cpp): identical code,
// except the reciprocal seed (device: v_rcp_f64; host: an f32 reciprocal, i.e. a worse seed).
#pragma once

#include <cmath>
#include <cstdint>

#if defined(__HIPCC__)
#define PLLM_HD __host__ __device__ __forceinline__
#else
#define PLLM_HD inline
#endif

namespace pllm {

// pi/2 split: P1, P2 have 22 significant bits (k*P exact for |k| < 2^31), P3 is the f64 rest.
constexpr double P1 = 1.5707964897155762;             // 0x3FF921FB80000000 (22 bits)
constexpr double P2 = -1.6292068494294654e-07;        // 0xBE85DDE980000000 (22 bits)
constexpr double P3 = 5.390302858158119e-15;          // 0x3CF8469898CC5170 = RN(pi/2 - P1 - P2)
constexpr double TWO_OVER_PI = 0.6366197723675814;
constexpr double PI = 3.141592653589793;
constexpr double TWO_PI = 6.283185307179586;
constexpr double PIO2 = 1.5707963267948966;
// fdlibm k_sin.c / k_cos.c coefficients (|x| <= pi/4)
constexpr double S1 = -1.66666666666666324348e-01, S2 = 8.33333333332248946124e-03,
                 S3 = -1.98412698298579493134e-04, S4 = 2.75573137070700676789e-06,
                 S5 = -2.50507602534068634195e-08, S6 = 1.58969099521155010221e-10;
// cos kernel: degree-4 Q (one coefficient fewer than fdlibm), refitted near-minimax for the
// relative error of cos on |r| <= pi/4 by tools/pllmath/fit_poly.py: 2^-51.7 in double evaluation
constexpr double C1 = 0.04166666666659653, C2 = -0.0013888888877611482, C3 = 2.4801580707202765e-05,
                 C4 = -2.755552309095219e-07, C5 = 2.0645117778725974e-09;
// error bounds used by the rounding test (generous: measured errors are far smaller)
constexpr double EPS_ABS_E = 0x1p-45;      // absolute, phase detector output (|e| <= pi)
constexpr double T_MAX = 0x1p30;           // reduction valid below this

PLLM_HD double fma_(double a, double b, double c) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_fma(a, b, c);
#else
    return std::fma(a, b, c);
#endif
}

PLLM_HD double rcp_seed(double x) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_rcp(x);
#else
    return (double)(1.0f / (float)x);    // ~2^-24: a worse seed than the device's
#endif
}

// true when every value in [v-eps, v+eps] rounds to the same f32 as v
PLLM_HD bool f32_rounding_safe(double v, double eps) {
    return (float)(v - eps) == (float)(v + eps);
}

// Same test for a RELATIVE error of at most 64 f64 ulps (2^-47 relative), on the mantissa bits:
// RN_f32 of a normal double depends only on its low 29 mantissa bits relative to the tie
// pattern 0x10000000; the rounding is safe when they are more than 64 away from it.
// (Valid for |v| >= 2^-126, i.e. f32-normal results -- cos/sin of an f32 argument always are.)
PLLM_HD bool f32_rounding_safe_rel64(double v) {
    const uint64_t bits = __builtin_bit_cast(uint64_t, v);
    const uint32_t m = (uint32_t)bits & 0x1FFFFFFFu;
    return (uint32_t)(m - 0x10000000u + 64u) > 128u;
}

// distance (in f64 ulps, offset by 64) of the low 29 mantissa bits from the f32 tie pattern;
// the rounding is safe iff the value is > 128 (see f32_rounding_safe_rel64)
PLLM_HD uint32_t tie_distance64(double v) {
    const uint64_t bits = __builtin_bit_cast(uint64_t, v);
    return ((uint32_t)bits & 0x1FFFFFFFu) - 0x10000000u + 64u;
}

struct SinCos {
    double c, s;     // cos t, sin t (relative error < 2^-50)
    double mr;       // -r, r = t - q*pi/2 in [-pi/4, pi/4] (absolute error < 2^-50)
    int q3;          // q mod 4: -t = -q3*pi/2 - r (mod 2pi)
    bool ok;         // (float)c and (float)s are RN_f32(cos t), RN_f32(sin t); reduction valid
    uint32_t tie;    // min(tie_distance64(c), tie_distance64(s)): ok needs tie > 128 and |t| < T_MAX
};

PLLM_HD SinCos sincos_f32(float t) {
    const double x = (double)t;
    const double kd = __builtin_rint(x * TWO_OVER_PI);
    double r = fma_(-kd, P1, x);
    r = fma_(-kd, P2, r);
    r = fma_(-kd, P3, r);
    const double z = r * r;
    const double z2 = z * z;
    const double z4 = z2 * z2;
    // sin r = r + r^3 (S1 + z S2 + z^2 (S3 + z S4) + z^4 (S5 + z S6))   (Estrin)
    const double sp = fma_(z4, fma_(z, S6, S5), fma_(z2, fma_(z, S4, S3), fma_(z, S2, S1)));
    const double sr = fma_(r * z, sp, r);
    // cos r = (1 - z/2) + z^2 (C1 + z C2 + z^2 (C3 + z C4) + z^4 C5)
    const double cp = fma_(z4, C5, fma_(z2, fma_(z, C4, C3), fma_(z, C2, C1)));
    const double cr = fma_(z2, cp, fma_(z, -0.5, 1.0));
    const int q = (int)kd;                   // |kd| < 2^30 when the reduction is valid
    const bool swap = (q & 1) != 0;
    const double a = swap ? sr : cr;
    const double b = swap ? cr : sr;
    SinCos o;
    // signs as bit flips of the high word: cos t < 0 in quadrants 1, 2 (bit 1 of q + 1), sin t < 0
    // in quadrants 2, 3 (bit 1 of q)
    o.c = __builtin_bit_cast(double, __builtin_bit_cast(uint64_t, a) ^
                                         ((uint64_t)(((uint32_t)(q + 1) << 30) & 0x80000000u) << 32));
    o.s = __builtin_bit_cast(double, __builtin_bit_cast(uint64_t, b) ^
                                         ((uint64_t)(((uint32_t)q << 30) & 0x80000000u) << 32));
    o.mr = -r;
    o.q3 = q & 3;
    o.tie = tie_distance64(o.c) < tie_distance64(o.s) ? tie_distance64(o.c) : tie_distance64(o.s);
    o.ok = (__builtin_fabs(x) < T_MAX) && o.tie > 128u;
    return o;
}

struct Phase {
    double e;        // atan2(eQ, eI) in [-pi, pi]
    double d;        // residual angle Y/X; the fast path needs |d| < 2^-18 and |e| < pi - 2^-30
    float ef;        // RN_f32(e + eps): equals RN_f32(e) whenever split == 0
    uint32_t split;  // bits(RN_f32(e - eps)) ^ bits(RN_f32(e + eps)): 0 iff the f32 rounding is safe
    bool ok;         // ef == RN_f32(atan2(eQ, eI))
};

// atan2(eQ, eI) given c, s = f64 cos t, sin t of the previous step's t and -t mod 2pi as
// -q3*pi/2 + mr (mr = -r of the reduction): NaN mr (invalid reduction) makes e NaN.
PLLM_HD Phase phase_detect(float eI, float eQ, double c, double s, double mr, int q3) {
    const double dI = (double)eI, dQ = (double)eQ;
    const double X = fma_(dI, c, -(dQ * s));      // Re((eI + i eQ)(c + i s))
    const double Y = fma_(dI, s, dQ * c);         // Im(...)
    const double r0 = rcp_seed(X);
    const double cc = fma_(-X, r0, 1.0);
    const double qq = Y * r0;
    const double d = fma_(qq, cc, qq);            // Y/X (rel. error ~ seed error^2); NaN/inf if X == 0
    // atan2 = -t + pi*[X < 0] + d = (2*[X < 0] - q3) * pi/2 + (mr + d)   (mod 2pi)
    const int k = (X < 0.0 ? 2 : 0) - q3;
    const double e0 = fma_((double)k, PIO2, mr + d);
    const double e = fma_(-__builtin_rint(e0 * (1.0 / TWO_PI)), TWO_PI, e0);   // into [-pi, pi]
    Phase o;
    o.e = e;
    o.d = d;
    o.ef = (float)(e + EPS_ABS_E);
    o.split = __builtin_bit_cast(uint32_t, (float)(e - EPS_ABS_E)) ^ __builtin_bit_cast(uint32_t, o.ef);
    o.ok = (__builtin_fabs(d) < 0x1p-18) && (__builtin_fabs(e) < PI - 0x1p-30) && o.split == 0u;
    return o;
}

}  // namespace pllm
