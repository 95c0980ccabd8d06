"""Host checks of the PLL math shared with the kernels (real-time-sdr_amd/csrc/pll_math.h).

The double-double fallbacks must reproduce glibc's f64 sin/cos/atan2 (the reference's libm,
pll.cpp:39, :49-52) after the f32 rounding the reference applies: tools/pllmath/validate_dd.cpp
compares them with this host's glibc on random PLL-like arguments and on arguments whose cosine
lies next to an f32 rounding midpoint, and fails on any f32 difference. The same header is
compiled for the device; the device results are compared with glibc by tools/pllmath/libm_flip.hip
(profiles/r01/libm_flip.json).
"""
from __future__ import annotations

import json
import pathlib
import shutil
import subprocess

import numpy as np
import pytest

ROOT = pathlib.Path(__file__).resolve().parents[1]


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_dd_fallbacks_match_glibc(tmp_path):
    exe = tmp_path / "validate_dd"
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-I", str(ROOT / "real-time-sdr_amd/csrc"),
                    str(ROOT / "tools/pllmath/validate_dd.cpp"), "-o", str(exe)], check=True)
    r = subprocess.run([str(exe), "300000"], capture_output=True, text=True, timeout=120)
    res = json.loads(r.stdout)
    assert r.returncode == 0, res
    for f in ("cos", "sin", "atan2"):
        assert res[f]["f32_mismatch"] == 0
        # f64 differences are glibc's own misroundings (|err| just over 0.5 ulp): rare
        assert res[f]["f64_mismatch"] < 0.005 * res["n"]
    # |t| >= 2^30 (Payne-Hanek in double-double): the PLL's phase passes 2^30 after ~25 min (RDS)
    assert res["large"]["f32_mismatch"] == 0
    assert res["large"]["f64_mismatch"] < 0.005 * 2 * res["large"]["n"]


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_nco_fast_cosine_matches_glibc(tmp_path):
    """The NCO output RN_f32(cos(t * ncoScale + phaseAdjust)) (pll.cpp:52) of the fused post stages
    (k_stereo_out, k_rds_mix) and k_nco_out: pll_math.h cos_rn_f32 (the PLL step's reduction and
    kernels, one kernel selected by the quadrant, one tie proof) must equal glibc's f64 cos rounded to
    f32 on every value it accepts -- near multiples of pi/2 and the stereo / RDS NCO arguments
    included (tools/pllmath/validate_nco.cpp)."""
    exe = tmp_path / "validate_nco"
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-I", str(ROOT / "real-time-sdr_amd/csrc"),
                    str(ROOT / "tools/pllmath/validate_nco.cpp"), "-o", str(exe)], check=True)
    r = subprocess.run([str(exe), "4000000"], capture_output=True, text=True, timeout=120)
    res = json.loads(r.stdout)
    assert r.returncode == 0 and res["f32_mismatch"] == 0, (res, r.stderr[-500:])
    assert res["fallback"] < 1e-4 * res["n"]


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_phase_detector_error_inside_e_bracket(tmp_path):
    """The e bracket EPS_ABS_E2 = 2^-46 (pll_math.h: analytic bound 2^-46.36 on |e - glibc atan2|)
    against the measured error of the phase detector the kernels ship: the lane-pair step of
    sdr_pll.hip pll_step_split evaluated operation for operation (tools/pllmath/validate_e3.cpp:
    sincos_rn's refitted kernels, Y = qA + qB from the two f32 products, base_angle_n) and glibc's f64
    atan2, each against a 64-bit-mantissa atan2l. The measured sum must stay inside the bracket with
    margin (2^-47.2 at 2e7 samples), and no sample whose bracket test passes may round differently
    from the reference."""
    exe = tmp_path / "validate_e3"
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-I", str(ROOT / "real-time-sdr_amd/csrc"),
                    str(ROOT / "tools/pllmath/validate_e3.cpp"), "-o", str(exe)], check=True)
    r = subprocess.run([str(exe), "2000000"], capture_output=True, text=True, timeout=120)
    res = json.loads(r.stdout)
    assert r.returncode == 0 and res["n"] > 1_900_000 and res["wrong"] == 0, res
    assert res["log2_eps"] == -46.0
    assert res["log2_sum"] < res["log2_eps"] - 0.8, res


def test_substitution_error_joint_bound():
    """pll_math.h's bound on the Y * rx substitution: |Y/x| |delta| <= max over the box |p|, |q| <= m of
    sqrt(C (1 - C)) |p - q| |C p + (1 - C) q| = m^2 / 2, m = 2u + u^2 (2^-47 for u = 2^-24), rather
    than m^2 from bounding the two factors separately. Grid over C and the box (the maximum of a
    product of two linear forms in (p, q) for fixed C lies on the box's boundary)."""
    C = np.linspace(0.0, 1.0, 2001)[:, None]
    s = np.linspace(-1.0, 1.0, 801)[None, :]
    best = 0.0
    for p, q in ((np.ones_like(s), s), (s, np.ones_like(s)), (-np.ones_like(s), s), (s, -np.ones_like(s))):
        h = np.sqrt(C * (1 - C)) * np.abs(p - q) * np.abs(C * p + (1 - C) * q)
        best = max(best, float(h.max()))
    assert 0.4999 < best <= 0.5 + 1e-12
