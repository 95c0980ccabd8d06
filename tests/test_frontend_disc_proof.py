"""CPU: the exact front end's discriminator proof (real-time-sdr_amd/csrc/sdr_frontend.hip,
fe_disc_store, SDR_FE_DISC). The reference's value is RN32(RN64(num / den)) with num an f32 and
den = RN64(I^2 + Q^2) (demod.cpp:11-18). The kernel computes q = RN64(num * r1), r1 = r0 + r0 *
RN64(1 - den * r0) (two fmas) from the hardware reciprocal r0, and accepts RN32(q) when the low 29
mantissa bits of q are more than FE_TIE_ULPS = 2048 ulps from the f32 tie pattern (the tie key) and
RN32(q) is not subnormal. Here every fma is evaluated exactly (fractions) with an adversarial r0 whose
relative error is the bound the proof allows (2^-22, GPU-measured 2^-24.4 in
tests/test_gpu_primitives.py): on samples drawn close to f32 rounding ties, no accepted quotient
may differ from the reference's, and on ordinary samples almost every quotient is accepted."""
from __future__ import annotations

from fractions import Fraction

import numpy as np

TIE_ULPS = 2048


def _rn64(x: Fraction) -> float:
    return float(x)          # correctly rounded (round-half-even), as an f64 fma's single rounding


def _key(q: float) -> int:
    lo = int(np.float64(q).view(np.uint64)) & 0xFFFFFFFF
    return ((lo << 3) + 0x80000000 + 8 * TIE_ULPS) & 0xFFFFFFFF


def _fast(num: np.float32, den: float, eps0: float):
    r0 = float(np.float64(1.0 / den) * (1.0 + eps0))          # the hardware reciprocal, off by ~eps0
    e = _rn64(1 - Fraction(den) * Fraction(r0))
    r1 = _rn64(Fraction(r0) + Fraction(r0) * Fraction(e))
    q = _rn64(Fraction(float(num)) * Fraction(r1))
    v = np.float32(q)
    accepted = _key(q) > 16 * TIE_ULPS and not (0 < abs(float(v)) < 2.0 ** -126)
    return v, accepted


def _samples(rng, n):
    I = rng.normal(0, 0.3, n).astype(np.float32)
    Q = rng.normal(0, 0.3, n).astype(np.float32)
    Ip = rng.normal(0, 0.3, n).astype(np.float32)
    Qp = rng.normal(0, 0.3, n).astype(np.float32)
    num = I * (Q - Qp) - Q * (I - Ip)                          # f32, no fma (demod.cpp:17)
    den = I.astype(np.float64) ** 2 + Q.astype(np.float64) ** 2
    return num, den


def test_discriminator_proof_never_accepts_a_wrong_rounding():
    rng = np.random.default_rng(2026)
    num, den = _samples(rng, 1 << 21)
    qd = num.astype(np.float64) / den                          # RN64(num / den)
    ref = qd.astype(np.float32)                                # the reference's value
    # distance of RN64(num/den) from the f32 tie pattern, in f64 ulps: keep the closest samples
    lo29 = (qd.view(np.uint64) & np.uint64(0x1FFFFFFF)).astype(np.int64)
    dist = np.abs(lo29 - (1 << 28))
    near = np.argsort(dist)[:1500]
    assert (dist[near] <= TIE_ULPS).sum() >= 5                 # the draw reaches inside the tie band
    wrong = checked = 0
    for i in near:
        for eps0 in (2.0 ** -22, -(2.0 ** -22), 0.0):
            v, ok = _fast(num[i], float(den[i]), eps0)
            if ok:
                checked += 1
                wrong += int(v.view(np.uint32) != ref[i].view(np.uint32))
    assert wrong == 0
    assert checked > 100                                       # outside the band: accepted and right


def test_discriminator_proof_accepts_ordinary_samples():
    rng = np.random.default_rng(7)
    num, den = _samples(rng, 4000)
    ref = (num.astype(np.float64) / den).astype(np.float32)
    acc = 0
    for i in range(len(num)):
        v, ok = _fast(num[i], float(den[i]), 2.0 ** -22)
        if ok:
            acc += 1
            assert v.view(np.uint32) == ref[i].view(np.uint32)
    assert acc >= len(num) - 2                                 # rejection rate ~ 4097 / 2^29 per output
