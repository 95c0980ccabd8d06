"""Host-side planning in bench.py (no GPU): the PLL stream's CU split by channel count."""
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import bench  # noqa: E402


def test_pll_cus_split():
    # the headline keeps one PLL wave per CU on 64 CUs; capacity counts trade PLL CUs for side-chain CUs
    assert bench.pll_cus(1024) == 64
    assert bench.pll_cus(1536) in (32, 64)
    assert bench.pll_cus(2048) == 32
    assert bench.pll_cus(4096) == 64
    for n in (1, 32, 100, 512, 1024, 3000, 8192):
        waves = 2 * ((2 * n + 63) // 64)
        cus = bench.pll_cus(n)
        assert cus in (16, 32, 64, 128)
        assert waves <= 4 * cus            # at most four waves per CU (one per SIMD)
