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
// sin kernel of the k_pll step (sincos_kernels): degree-4 P, refitted the same way (fit_poly.py):
// 2^-47.48 relative error in double Horner evaluation on |r| <= pi/4 -- 46 f64 ulps at most, inside
// the tie test's 128-ulp margin, and 0.5 (eps_s + eps_c) < 2^-48.3 of phase-detector error, inside
// EPS_ABS_E2 with the 2^-45.9 of the Y * rx substitution
constexpr double SR1 = -0.1666666666663035, SR2 = 0.008333333325077597, SR3 = -0.00019841263728549816,
                 SR4 = 2.755533964014372e-06, SR5 = -2.4760453463432028e-08;
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

// ------------------------------------------------------------------------------------------
// v2 step (k_pll): shorter dependent chain and no f64 reciprocal inside the recurrence.
//
//  * rx = pll_rx(x): the PLL input's reciprocal, computed by the kernel that PRODUCES the input
//    (it does not depend on the PLL state). f64 RN(1/x) with its two low mantissa bits replaced
//    by 2*[x < 0] (a <= 3-ulp perturbation), or a NaN when |x| < 2^-60 or x is not finite.
//  * sincos2_f32: the same reduction and kernels as sincos_f32, but kd comes from one fma with
//    the 1.5*2^52 rounding constant, whose low word is q itself (no f64 -> int conversion).
//  * phase_detect2: with (eI, eQ) = x * (RN c, -RN s), rotating by +t gives X = x (1 + delta),
//    |delta| <= 2^-23, and Y = x c s (alpha + a - beta - b) for the four f32 rounding errors,
//    so |Y / X| <= 2^-23 whenever |x| >= 2^-60 (subnormal products then only touch terms below
//    2^-66). d = Y * rx replaces Y / X with an absolute error <= |Y/x| (|delta| + 2^-51).
//    Bounded jointly (round 6): with p = a + alpha + a alpha, q = b + beta + b beta (|p|, |q| <=
//    2u + u^2, u = 2^-24), Y/x = c s (p - q) + O(u^2) and delta = c^2 p + s^2 q + O(u^2), so
//    |Y/x| |delta| <= sqrt(C (1 - C)) |p - q| |C p + (1 - C) q| with C = c^2, whose maximum over the
//    box is (2u)^2 / 2 = 2^-47 (at p = -q, C = (1 + 1/sqrt 2) / 2; tests/test_pll_math.py checks it
//    on a grid) -- not the 2^-45.9 of bounding |d| <= 2^-23 and |delta| <= 2^-23 separately, which
//    cannot both be reached. atan2(eQ, eI) = base + d where base = -t + pi [x < 0] (mod 2pi) is
//    prepared from the PREVIOUS step's quadrant before this step's input is touched (base_angle).
//    EPS_ABS_E2 bounds the distance from e to the reference's f64 atan2: the substitution's 2^-47,
//    the kernels' 0.5 (eps_s + eps_c) < 2^-48.3, Y's own roundings (the lane-pair form rounds both
//    products, 2^-54 |x| each: 2^-53), base's and the final add's roundings (2^-52 each), the
//    representation of pi/2 times |m| <= 2 (2^-52.8), glibc atan2's own <= 1 ulp (2^-51):
//    2^-46.36 in all, under 2^-46 (round 6; 2^-45 in round 5, 2^-44 before: each halving halves the
//    e-bracket chunk redos). Measured on the shipped lane-pair step (tools/pllmath/validate_e3.cpp,
//    sdr_pll.hip pll_step_split operation for operation): 2^-47.2 over 2e7 samples, no accepted
//    rounding different from the reference's; the v2 detector (validate_e2.cpp) 2^-47.8.
// ------------------------------------------------------------------------------------------
constexpr double MAGIC = 6755399441055744.0;   // 1.5 * 2^52: fma(x, c, MAGIC) - MAGIC = rint(x c)
constexpr double EPS_ABS_E2 = 0x1p-46;

PLLM_HD double pll_rx(float x) {
    const float ax = __builtin_fabs(x);
    if (!(ax >= 0x1p-60f) || !(ax <= 3.4028234663852886e38f))
        return __builtin_bit_cast(double, (uint64_t)0x7FF8000000000000ull | (x < 0.0f ? 2u : 0u));
    const double r = 1.0 / (double)x;
    const uint64_t b = (__builtin_bit_cast(uint64_t, r) & ~(uint64_t)3) | (x < 0.0f ? 2u : 0u);
    return __builtin_bit_cast(double, b);
}

struct SinCos2 {
    double c, s;     // cos t, sin t (relative error < 2^-50)
    double mr;       // -r, r = t - q*pi/2 in [-pi/4, pi/4]
    uint32_t q;      // q (mod 2^32)
    uint32_t b;      // [r < 0]
    uint32_t tie;    // min(tie_distance64(c), tie_distance64(s)); (float)c, (float)s are RN_f32 when > 128
};

// valid for |t| < T_MAX (the caller checks the range)
PLLM_HD SinCos2 sincos2_f32(float t) {
    const double x = (double)t;
    const double kdp = fma_(x, TWO_OVER_PI, MAGIC);
    const double kd = kdp - MAGIC;
    const uint32_t q = (uint32_t)__builtin_bit_cast(uint64_t, kdp);
    double r = fma_(-kd, P1, x);
    r = fma_(-kd, P2, r);
    r = fma_(-kd, P3, r);
    const double z = r * r;
    const double z2 = z * z;
    const double z4 = z2 * z2;
    const double sp = fma_(z4, fma_(z, S6, S5), fma_(z2, fma_(z, S4, S3), fma_(z, S2, S1)));
    const double sr = fma_(r * z, sp, r);
    const double cp = fma_(z4, C5, fma_(z2, fma_(z, C4, C3), fma_(z, C2, C1)));
    const double cr = fma_(z2, cp, fma_(z, -0.5, 1.0));
    const bool swap = (q & 1u) != 0;
    const double a = swap ? sr : cr;
    const double bb = swap ? cr : sr;
    SinCos2 o;
    o.c = __builtin_bit_cast(double, __builtin_bit_cast(uint64_t, a) ^
                                         ((uint64_t)(((q + 1u) << 30) & 0x80000000u) << 32));
    o.s = __builtin_bit_cast(double, __builtin_bit_cast(uint64_t, bb) ^
                                         ((uint64_t)((q << 30) & 0x80000000u) << 32));
    o.mr = -r;
    o.q = q;
    o.b = (uint32_t)(__builtin_bit_cast(uint64_t, r) >> 63);
    const uint32_t tc = tie_distance64(o.c), ts = tie_distance64(o.s);
    o.tie = tc < ts ? tc : ts;
    return o;
}

// -t + pi*[x < 0] (mod 2pi) as m*pi/2 + mr with m in {-2..1} chosen so the sum lies in [-pi, pi]:
// with m0 = (2[x<0] - q) mod 4, m = ((m0 + b + 1) mod 4) - 1 - b (b = [mr > 0]; m0 = 2 picks +pi
// when mr < 0 and -pi otherwise). nlo: low word of pll_rx(x) (bit 1 = [x < 0]).
PLLM_HD double base_angle(uint32_t nlo, uint32_t q, uint32_t b, double mr) {
    const int m = (int)((nlo - q + b + 1u) & 3u) - (int)(b + 1u);
    return fma_((double)m, PIO2, mr);
}

struct Phase2 {
    double e;        // atan2(eQ, eI), |error| <= EPS_ABS_E2 (NaN when rx is)
    float ef;        // RN_f32(e)
    uint32_t split;  // bits(RN_f32(e - eps)) ^ bits(RN_f32(e + eps)): 0 iff the f32 rounding is safe
};

PLLM_HD Phase2 phase_detect2(float eI, float eQ, double c, double s, double rx, double base) {
    const double dI = (double)eI, dQ = (double)eQ;
    const double Y = fma_(dI, s, dQ * c);
    const double e = fma_(Y, rx, base);   // base + d with one rounding
    Phase2 o;
    o.e = e;
    o.ef = (float)e;
    o.split = __builtin_bit_cast(uint32_t, (float)(e - EPS_ABS_E2)) ^
              __builtin_bit_cast(uint32_t, (float)(e + EPS_ABS_E2));
    return o;
}

PLLM_HD uint32_t lo_word(double v) { return (uint32_t)__builtin_bit_cast(uint64_t, v); }

// ------------------------------------------------------------------------------------------
// Reduced-frame step (k_pll). With t = q pi/2 + r, cos t + i sin t = i^q (cos r + i sin r), and
// RN_f32 commutes with multiplying by i^q (it only swaps and negates components), so
//   fbI + i fbQ = i^q (fI0 + i fQ0),  fI0 = RN(cos r), fQ0 = RN(sin r)            (pll.cpp:49-50)
//   eI - i eQ   = i^q (eI0 - i eQ0),  eI0 = RN(x fI0), eQ0 = RN(-x fQ0)           (pll.cpp:36-37)
// and the rotated residual X + iY = (eI + i eQ)(c + i s) equals (eI0 + i eQ0)(cos r + i sin r).
// The recurrence therefore never needs the quadrant swap/sign of cos t, sin t: it carries
// (fI0, fQ0) and q, and the quadrant enters only through base_angle. rot_q applies i^q to a pair
// (exactly), for the state at block boundaries and for the libm fallbacks.
// ------------------------------------------------------------------------------------------
struct SinCosR {
    double cr, sr;   // cos r, sin r (relative error < 2^-50)
    double mr;       // -r
    uint32_t q, b;   // quadrant, [r < 0]
    uint32_t tie;    // min(tie_key64(cr), tie_key64(sr)); the roundings are safe iff tie > TIE_MIN
};

// 8 x tie_distance64(v) (mod 2^32) in one shift-add: the shift drops the 3 low f32 mantissa bits
// that sit above the 29-bit field. tie_distance64(v) > 128 <=> tie_key64(v) > TIE_MIN.
constexpr uint32_t TIE_MIN = 128u << 3;
PLLM_HD uint32_t tie_key64(double v) { return ((uint32_t)__builtin_bit_cast(uint64_t, v) << 3) + 0x80000200u; }

// pi/2 as RN64 + the f64 rest: with t an f32 and |t| < 2^30, t - kd*PIO2_HI is exact (a multiple of
// 2^-52 below 1 in magnitude), so two fmas reduce with one rounding plus |kd| 2^-107
constexpr double PIO2_HI = 0x1.921fb54442d18p+0, PIO2_LO = 0x1.1a62633145c07p-54;

// valid for |t| < T_MAX (the caller checks the range)
PLLM_HD SinCosR sincos_r(float t) {
    const double x = (double)t;
    const double kdp = fma_(x, TWO_OVER_PI, MAGIC);
    const double kd = kdp - MAGIC;
    const double r = fma_(-kd, PIO2_LO, fma_(-kd, PIO2_HI, x));
    const double z = r * r;
    const double z2 = z * z;
    const double z4 = z2 * z2;
    const double sp = fma_(z4, fma_(z, S6, S5), fma_(z2, fma_(z, S4, S3), fma_(z, S2, S1)));
    const double cp = fma_(z4, C5, fma_(z2, fma_(z, C4, C3), fma_(z, C2, C1)));
    SinCosR o;
    o.sr = fma_(r * z, sp, r);
    o.cr = fma_(z2, cp, fma_(z, -0.5, 1.0));
    o.mr = -r;
    o.q = (uint32_t)__builtin_bit_cast(uint64_t, kdp);
    o.b = (uint32_t)(__builtin_bit_cast(uint64_t, r) >> 63);
    const uint32_t tc = tie_key64(o.cr), ts = tie_key64(o.sr);
    o.tie = tc < ts ? tc : ts;
    return o;
}

// ------------------------------------------------------------------------------------------
// v3 step pieces (k_pll): fewer instructions per step, same values.
//  * sincos_rn: the reduction rounds -t (2/pi) against MAGIC + 1, so the low word of the rounded
//    value is nq1 = 1 - q (mod 2^32) -- exactly what base_angle needs -- and kdn = -kd folds its
//    sign into the two reduction fmas. Both kernels by Horner (2 multiplies fewer than Estrin's
//    z^2, z^4 powers, a longer dependent chain: +1.8 %; a two-level form, +3.4 %, is
//    tools/patches/pll_variants.patch) with the refitted 5-coefficient sin (SR1..SR5, one fma fewer
//    than fdlibm's).
//  * base_angle_n(nlo, nq1, b, mr) = base_angle(nlo, 1 - nq1, b, mr): one 3-input add.
// ------------------------------------------------------------------------------------------
constexpr double MAGIC1 = 6755399441055745.0;   // 1.5 * 2^52 + 1

struct SinCosRN {
    double cr, sr;   // cos r, sin r (relative error < 2^-51.7, 2^-47.4)
    double r;        // t - q pi/2 in [-pi/4, pi/4]
    uint32_t nq1;    // 1 - q (mod 2^32)
    uint32_t b;      // [r < 0]
    uint32_t tie;    // min(tie_key64(cr), tie_key64(sr)); the roundings are safe iff tie > TIE_MIN
    uint32_t tc, ts; // the two keys
};

PLLM_HD void sincos_kernels(double r, double& cr, double& sr) {
    const double z = r * r;
    double sp = fma_(z, SR5, SR4);
    sp = fma_(z, sp, SR3);
    sp = fma_(z, sp, SR2);
    sp = fma_(z, sp, SR1);
    double cp = fma_(z, C5, C4);
    cp = fma_(z, cp, C3);
    cp = fma_(z, cp, C2);
    cp = fma_(z, cp, C1);
    cp = fma_(z, cp, -0.5);
    sr = fma_(r * z, sp, r);
    cr = fma_(z, cp, 1.0);
}

// valid for |t| < T_MAX (the caller checks the range)
PLLM_HD SinCosRN sincos_rn(float t) {
    const double x = (double)t;
    const double kdp = fma_(x, -TWO_OVER_PI, MAGIC1);   // MAGIC1 + rint(-x 2/pi)
    const double kdn = kdp - MAGIC1;                      // -kd
    const double r = fma_(kdn, PIO2_LO, fma_(kdn, PIO2_HI, x));
    SinCosRN o;
    sincos_kernels(r, o.cr, o.sr);
    o.r = r;
    o.nq1 = (uint32_t)__builtin_bit_cast(uint64_t, kdp);
    o.b = (uint32_t)(__builtin_bit_cast(uint64_t, r) >> 63);
    o.tc = tie_key64(o.cr);
    o.ts = tie_key64(o.sr);
    o.tie = o.tc < o.ts ? o.tc : o.ts;
    return o;
}

// RN_f32(cos a) of an f32 argument (the NCO output, pll.cpp:52) from the sincos_rn reduction and
// kernels: cos(q pi/2 + r) = cos r, -sin r, -cos r, sin r for q = 0, 1, 2, 3 (mod 4), so only the
// selected kernel's f32 rounding needs its tie proof (one key instead of two; sincos_f32 also
// reduced in three fmas and evaluated fdlibm's longer sin). ok: the result is RN_f32(cos a), i.e.
// |a| < T_MAX and the selected value is more than 128 f64 ulps from an f32 tie (the sin kernel's
// error is <= 46 ulps, the cos kernel's far less; tools/pllmath/validate_nco.cpp checks it against
// glibc). Otherwise the caller recomputes (double-double, pll_math.h dd_sincos_f32).
PLLM_HD float cos_rn_f32(float a, bool& ok) {
    const SinCosRN sc = sincos_rn(a);
    const uint32_t q = 1u - sc.nq1;
    double v = (q & 1u) ? sc.sr : sc.cr;
    const uint32_t key = tie_key64(v);
    if (((q + 1u) >> 1) & 1u) v = -v;                     // RN_f32 is odd: the sign after the test
    ok = (__builtin_fabs((double)a) < T_MAX) && key > TIE_MIN;
    return (float)v;
}

PLLM_HD double base_angle_n(uint32_t nlo, uint32_t nq1, uint32_t b, double mr) {
    const int m = (int)((nlo + nq1 + b) & 3u) - (int)(b + 1u);
    return fma_((double)m, PIO2, mr);
}

// (a, b) <- i^q (a + i b): q mod 4 = 1 -> (-b, a), 2 -> (-a, -b), 3 -> (b, -a)
template <typename T>
PLLM_HD void rot_q(uint32_t q, T& a, T& b) {
    const T a0 = a, b0 = b;
    switch (q & 3u) {
        case 1: a = -b0; b = a0; break;
        case 2: a = -a0; b = -b0; break;
        case 3: a = b0; b = -a0; break;
        default: break;
    }
}

// the residual angle of the reduced frame (same value as phase_detect2's, see above)
PLLM_HD Phase2 phase_detect_r(float eI0, float eQ0, double cr, double sr, double rx, double base) {
    return phase_detect2(eI0, eQ0, cr, sr, rx, base);
}

// ------------------------------------------------------------------------------------------
// Fallbacks: glibc's f64 results, reproduced. glibc's sin/cos/atan2 return the correctly rounded
// f64 value RN64(f(x)) (all but a vanishing fraction of inputs), and the reference then rounds that
// to f32. The device libm (OCML) differs from glibc by 1-2 f64 ulps on 3-27% of inputs
// (profiles/r01/libm_flip.json); harmless on random inputs, but the fast path falls back exactly on
// the inputs that sit next to an f32 rounding midpoint, where a 1-ulp difference flips the f32
// result. So the fallbacks evaluate f in double-double arithmetic (error < 2^-100 relative) and
// return its leading double, which is RN64(f(x)) -- glibc's value -- and round that to f32.
// ------------------------------------------------------------------------------------------
// generated by tools/pllmath/dd_consts.py
constexpr double DD_PIO2_1 = 0x1.921fb00000000p+0;  // 22 bits
constexpr double DD_PIO2_2 = 0x1.5110b00000000p-22;  // 22 bits
constexpr double DD_PIO2_3 = 0x1.18469898cc517p-44;
constexpr double DD_PIO2_4 = 0x1.b839a252049c1p-104;
constexpr double DD_PI_HI = 0x1.921fb54442d18p+1, DD_PI_LO = 0x1.1a62633145c07p-53;
constexpr double DD_PIO2_HI = 0x1.921fb54442d18p+0, DD_PIO2_LO = 0x1.1a62633145c07p-54;
constexpr double DD_INV_FACT[32][2] = {
    {0x1.0000000000000p+0, 0x0.0p+0},  // 1/0!
    {0x1.0000000000000p+0, 0x0.0p+0},  // 1/1!
    {0x1.0000000000000p-1, 0x0.0p+0},  // 1/2!
    {0x1.5555555555555p-3, 0x1.5555555555555p-57},  // 1/3!
    {0x1.5555555555555p-5, 0x1.5555555555555p-59},  // 1/4!
    {0x1.1111111111111p-7, 0x1.1111111111111p-63},  // 1/5!
    {0x1.6c16c16c16c17p-10, -0x1.f49f49f49f49fp-65},  // 1/6!
    {0x1.a01a01a01a01ap-13, 0x1.a01a01a01a01ap-73},  // 1/7!
    {0x1.a01a01a01a01ap-16, 0x1.a01a01a01a01ap-76},  // 1/8!
    {0x1.71de3a556c734p-19, -0x1.c154f8ddc6c00p-73},  // 1/9!
    {0x1.27e4fb7789f5cp-22, 0x1.cbbc05b4fa99ap-76},  // 1/10!
    {0x1.ae64567f544e4p-26, -0x1.c062e06d1f209p-80},  // 1/11!
    {0x1.1eed8eff8d898p-29, -0x1.2aec959e14c06p-83},  // 1/12!
    {0x1.6124613a86d09p-33, 0x1.f28e0cc748ebep-87},  // 1/13!
    {0x1.93974a8c07c9dp-37, 0x1.05d6f8a2efd1fp-92},  // 1/14!
    {0x1.ae7f3e733b81fp-41, 0x1.1d8656b0ee8cbp-97},  // 1/15!
    {0x1.ae7f3e733b81fp-45, 0x1.1d8656b0ee8cbp-101},  // 1/16!
    {0x1.952c77030ad4ap-49, 0x1.ac981465ddc6cp-103},  // 1/17!
    {0x1.6827863b97d97p-53, 0x1.eec01221a8b0bp-107},  // 1/18!
    {0x1.2f49b46814157p-57, 0x1.2650f61dbdcb4p-112},  // 1/19!
    {0x1.e542ba4020225p-62, 0x1.ea72b4afe3c2fp-120},  // 1/20!
    {0x1.71b8ef6dcf572p-66, -0x1.d043ae40c4647p-120},  // 1/21!
    {0x1.0ce396db7f853p-70, -0x1.aebcdbd20331cp-124},  // 1/22!
    {0x1.761b41316381ap-75, -0x1.3423c7d91404fp-130},  // 1/23!
    {0x1.f2cf01972f578p-80, -0x1.9ada5fcc1ab14p-135},  // 1/24!
    {0x1.3f3ccdd165fa9p-84, -0x1.58ddadf344487p-139},  // 1/25!
    {0x1.88e85fc6a4e5ap-89, -0x1.71c37ebd16540p-143},  // 1/26!
    {0x1.d1ab1c2dccea3p-94, 0x1.054d0c78aea14p-149},  // 1/27!
    {0x1.0a18a2635085dp-98, 0x1.b9e2e28e1aa54p-153},  // 1/28!
    {0x1.259f98b4358adp-103, 0x1.eaf8c39dd9bc5p-157},  // 1/29!
    {0x1.3932c5047d60ep-108, 0x1.832b7b530a627p-162},  // 1/30!
    {0x1.434d2e783f5bcp-113, 0x1.0b87b91be9affp-167},  // 1/31!
};

struct DD {
    double hi, lo;
};
PLLM_HD DD two_sum(double a, double b) {
    const double s = a + b;
    const double bb = s - a;
    return {s, (a - (s - bb)) + (b - bb)};
}
PLLM_HD DD quick_two_sum(double a, double b) {  // |a| >= |b|
    const double s = a + b;
    return {s, b - (s - a)};
}
PLLM_HD DD two_prod(double a, double b) {
    const double p = a * b;
    return {p, fma_(a, b, -p)};
}
PLLM_HD DD dd_add(DD a, DD b) {
    DD s = two_sum(a.hi, b.hi);
    const DD t = two_sum(a.lo, b.lo);
    s.lo += t.hi;
    s = quick_two_sum(s.hi, s.lo);
    s.lo += t.lo;
    return quick_two_sum(s.hi, s.lo);
}
PLLM_HD DD dd_neg(DD a) { return {-a.hi, -a.lo}; }
PLLM_HD DD dd_mul(DD a, DD b) {
    DD p = two_prod(a.hi, b.hi);
    p.lo += a.hi * b.lo + a.lo * b.hi;
    return quick_two_sum(p.hi, p.lo);
}
PLLM_HD DD dd_mul_d(DD a, double b) {
    DD p = two_prod(a.hi, b);
    p.lo += a.lo * b;
    return quick_two_sum(p.hi, p.lo);
}
PLLM_HD DD dd_div(DD a, DD b) {
    const double q1 = a.hi / b.hi;
    DD r = dd_add(a, dd_neg(dd_mul_d(b, q1)));
    const double q2 = r.hi / b.hi;
    r = dd_add(r, dd_neg(dd_mul_d(b, q2)));
    const double q3 = r.hi / b.hi;
    return dd_add(quick_two_sum(q1, q2), DD{q3, 0.0});
}

// sum_{k<=14} (-1)^k z^k / (2k+o)!  (o = 0: cos r, o = 1: sin r / r), Horner; |z| <= 0.62 leaves
// a truncation error below 2^-110
PLLM_HD DD dd_trig_series(DD z, int o) {
    DD p = {DD_INV_FACT[28 + o][0], DD_INV_FACT[28 + o][1]};
    for (int k = 13; k >= 0; k--) {
        p = dd_mul(p, dd_neg(z));
        p = dd_add(p, DD{DD_INV_FACT[2 * k + o][0], DD_INV_FACT[2 * k + o][1]});
    }
    return p;
}

// cos t, sin t in double-double for |t| < 2^30, t a double for which t - k*P1 below is exact
// (f32 arguments, or any |t| <= 4). Reduction by the 22/22/53/53-bit pi/2 split: k*P1 and k*P2
// are exact; the rest in double-double (error < 2^-125 absolute).
PLLM_HD void dd_sincos_dd(double t, DD& c, DD& s) {
    const double kd = __builtin_rint(t * TWO_OVER_PI);
    const double a = fma_(-kd, DD_PIO2_1, t);
    DD r = two_sum(a, -(kd * DD_PIO2_2));
    r = dd_add(r, dd_neg(two_prod(kd, DD_PIO2_3)));
    r = dd_add(r, DD{-(kd * DD_PIO2_4), 0.0});
    const DD z = dd_mul(r, r);
    const DD cr = dd_trig_series(z, 0);
    const DD sr = dd_mul(dd_trig_series(z, 1), r);
    // cos t + i sin t = i^q (cos r + i sin r)
    switch ((int)kd & 3) {
        case 0: c = cr; s = sr; break;
        case 1: c = dd_neg(sr); s = cr; break;
        case 2: c = dd_neg(cr); s = dd_neg(sr); break;
        default: c = sr; s = dd_neg(cr); break;
    }
}

// RN64(cos t), RN64(sin t): glibc's cos/sin of pll.cpp:49-50 and :52
PLLM_HD void dd_sincos(double t, double* s_out, double* c_out) {
    DD c, s;
    dd_sincos_dd(t, c, s);
    *c_out = c.hi;
    *s_out = s.hi;
}

// 2/pi in 24-bit chunks: chunk k holds bits 24k+1 .. 24k+24 after the binary point
// (tools/pllmath/dd_consts.py, from pi in exact rational arithmetic)
constexpr uint32_t IPIO2_24[16] = {
    0xA2F983, 0x6E4E44, 0x1529FC, 0x2757D1, 0xF534DD, 0xC0DB62, 0x95993C, 0x439041,
    0xFE5163, 0xABDEBB, 0xC561B7, 0x246E3A, 0x424DD2, 0xE00649, 0x2EEA09, 0xD1921C};

// Payne-Hanek reduction of a finite f32 |t| >= 2^30: t = M 2^E with M < 2^24 an integer, so
// t (2/pi) = sum_k M c_k 2^(E - 24(k+1)), every product M c_k < 2^48 exact in f64. Terms whose
// scale makes them multiples of 4 drop out (only t (2/pi) mod 4 matters), the leading kept terms
// are reduced mod 4 exactly, the rest down to 2^-120 are summed in double-double. Returns the
// quadrant q (mod 4) and r = (t (2/pi) - q) pi/2 in double-double, |r| <= pi/4 (+2^-100); the
// reduction error is below 2^-110 absolute (the closest f32 to a multiple of pi/2 is ~2^-30 away,
// so r keeps > 2^-80 relative accuracy: RN64 of cos/sin stays exact).
PLLM_HD int dd_reduce_f32_large(float t, DD& r) {
    const uint32_t bits = __builtin_bit_cast(uint32_t, t) & 0x7FFFFFFFu;
    const int E = (int)(bits >> 23) - 127 - 23;
    const double M = (double)((bits & 0x7FFFFFu) | 0x800000u);
    DD acc = {0.0, 0.0};
    for (int k = 0; k < 16; k++) {
        const int s = E - 24 * (k + 1);              // term = (M c_k) 2^s
        if (s >= 2) continue;                        // a multiple of 4
        if (s + 48 < -120) break;                    // below 2^-120 (and every later term)
        double p = M * (double)IPIO2_24[k];          // exact, < 2^48
        if (s > -48) {                               // p 2^s may reach 4: keep p mod 2^(2-s)
            const double m = __builtin_ldexp(1.0, 2 - s);
            p = p - __builtin_floor(p / m) * m;      // exact (power-of-two modulus)
        }
        acc = dd_add(acc, DD{__builtin_ldexp(p, s), 0.0});
    }
    double q = __builtin_rint(acc.hi);
    DD f = dd_add(acc, DD{-q, 0.0});
    if (f.hi > 0.5) { f = dd_add(f, DD{-1.0, 0.0}); q += 1.0; }
    if (f.hi < -0.5) { f = dd_add(f, DD{1.0, 0.0}); q -= 1.0; }
    r = dd_mul(f, DD{DD_PIO2_HI, DD_PIO2_LO});
    int qi = (int)q & 3;
    if (t < 0.0f) {                                  // t = -|t|: negate r and q
        r = dd_neg(r);
        qi = (4 - qi) & 3;
    }
    return qi;
}

// RN64(cos t), RN64(sin t) for any finite f32 t (glibc's sin/cos of pll.cpp:49-50 and :52 for
// arguments beyond the Cody-Waite range of dd_sincos_dd as well)
PLLM_HD void dd_sincos_f32(float t, double* s_out, double* c_out) {
    if (__builtin_fabs(t) < 0x1p30f) {
        dd_sincos((double)t, s_out, c_out);
        return;
    }
    DD r;
    const int q = dd_reduce_f32_large(t, r);
    const DD z = dd_mul(r, r);
    const DD cr = dd_trig_series(z, 0);
    const DD sr = dd_mul(dd_trig_series(z, 1), r);
    double c, s;
    switch (q) {                                     // cos t + i sin t = i^q (cos r + i sin r)
        case 0: c = cr.hi; s = sr.hi; break;
        case 1: c = -sr.hi; s = cr.hi; break;
        case 2: c = -cr.hi; s = -sr.hi; break;
        default: c = sr.hi; s = -cr.hi; break;
    }
    *c_out = c;
    *s_out = s;
}

// RN64(atan2(y, x)) (glibc's atan2 of pll.cpp:39) for f32 inputs. th0 is any approximation within a
// few ulps (the device libm's); rotating (x, y) by -th0 in double-double leaves a residual angle
// |d| < 2^-48, and atan2(y, x) = th0 + d - d^3/3 to 2^-140. Zeros, infinities and NaN return th0:
// their results are exact special values in every libm.
PLLM_HD double dd_atan2_f32(float y, float x, double th0) {
    if (!(__builtin_fabs(th0) <= 4.0) || (x == 0.0f && y == 0.0f) || !(__builtin_fabs(x) < 0x1p127f) ||
        !(__builtin_fabs(y) < 0x1p127f))
        return th0;
    DD c, s;
    dd_sincos_dd(th0, c, s);
    // (X + iY) = (x + iy)(c - is)
    const DD X = dd_add(dd_mul_d(c, (double)x), dd_mul_d(s, (double)y));
    const DD Y = dd_add(dd_mul_d(c, (double)y), dd_neg(dd_mul_d(s, (double)x)));
    const DD d = dd_div(Y, X);
    const double d3 = d.hi * d.hi * d.hi * (1.0 / 3.0);
    return dd_add(two_sum(th0, d.hi), DD{d.lo - d3, 0.0}).hi;
}

}  // namespace pllm
