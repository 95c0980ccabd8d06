"""CPU: the C-ABI library loads, exports every symbol include/sdr_amd.h declares, rejects bad
arguments without touching a GPU, and its host-side tap design equals the reference's taps."""
from __future__ import annotations

import ctypes as C
import re

import numpy as np

from conftest import ROOT


def _declared(header: str) -> list[str]:
    text = (ROOT / "include" / header).read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(sdr_[a-z0-9_]+)\s*\(", text)))


def test_library_exports_every_declared_symbol(pkg):
    lib = pkg.lib()
    names = _declared("sdr_amd.h")
    assert len(names) >= 20
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing


def test_host_library_exports_the_multi_receiver_engine():
    """include/sdr_multi.h's entry point lives in libsdr_host.so (the engine behind sdr_multi and the
    bench's queue_plumbed leg); it rejects a NULL options block without touching a GPU."""
    host = C.CDLL(str(ROOT / "real-time-sdr_amd" / "libsdr_host.so"))
    names = _declared("sdr_multi.h")
    assert names == ["sdr_multi_run"]
    assert all(hasattr(host, n) for n in names)
    host.sdr_multi_run.argtypes = [C.c_void_p, C.c_void_p]
    assert host.sdr_multi_run(None, None) == -1


def test_errors_are_status_codes(pkg):
    lib = pkg.lib()
    assert lib.sdr_version() >= 1
    assert lib.sdr_ctx_info(None, None) == -1
    assert b"null" in lib.sdr_last_error()
    assert lib.sdr_frontend(None, None, 0, None) == -1
    assert lib.sdr_convolve_fir(None, 0, None, 0, 1, 10, None, 101, None, 100, 1, None) == -1
    assert lib.sdr_impulse_response_lpf(2.4e6, 1e5, 101, None) == -1
    assert lib.sdr_stream_create_cu_range(None, 0, 0, 64, 0) == -1   # NULL out: no HIP call made
    assert lib.sdr_stream_destroy(None) == -1
    assert b"NULL" in lib.sdr_last_error()


def test_diagnosis_counters_absent_in_product_build(pkg):
    """sdr_diag_pll_counts (not part of sdr_amd.h) only works in -DSDR_PLL_COUNT=1 diagnosis builds;
    the shipped library answers -1 without touching a GPU, and bench.py then reports no redo rate."""
    out = (C.c_ulonglong * 10)()
    assert pkg.lib().sdr_diag_pll_counts(out, 0) == -1
    # the per-wave totals of -DSDR_PLL_WAVES=1 builds (bench.py pll.waves) likewise
    waves = (C.c_ulonglong * (8 * 4))()
    assert pkg.lib().sdr_diag_pll_waves(waves, 4) == -1
    # and the wave placement of -DSDR_PLL_HWID=1 builds (tools/diag_pll_place.py)
    hwid = (C.c_ulonglong * (5 * 4))()
    assert pkg.lib().sdr_diag_pll_hwid(hwid, 4) == -1


def test_product_taps_equal_reference_taps(pkg, golden):
    cases = {
        "rf": pkg.impulse_response_lpf(2.4e6, 1e5, 101),
        "audio": pkg.impulse_response_lpf(240000.0, 16000.0, 101, 1),
        "pilot": pkg.impulse_response_bpf(240000.0, 18.5e3, 19.5e3, 101),
        "stereo": pkg.impulse_response_bpf(240000.0, 22e3, 54e3, 101),
        "carrier": pkg.impulse_response_bpf(240000.0, 37.5e3, 38.5e3, 101),
        "apf": pkg.impulse_response_apf(1.0, 101),
        "rds": pkg.impulse_response_bpf(240000.0, 54e3, 60e3, 101),
        "rds_sq": pkg.impulse_response_bpf(240000.0, 113.5e3, 114.5e3, 101),
        "rds_bb": pkg.impulse_response_lpf(240000.0 * 247, 3e3, 24947, 247),
        "rrc": pkg.impulse_response_rrc(2375.0 * 39, 101),
    }
    for name, h in cases.items():
        assert np.array_equal(h.view(np.uint32), golden["taps_" + name].view(np.uint32)), name


def test_struct_layouts(pkg):
    # pllblock_args: 4 floats, a double, a float -> 32 bytes with the double 8-aligned (include/pll.h:10-17)
    assert C.sizeof(pkg.PllState) == 32
    assert pkg.PllState.trigOffset.offset == 16
    assert C.sizeof(pkg.Info) == 15 * 4
