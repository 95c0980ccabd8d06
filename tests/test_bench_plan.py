"""Host-side planning in bench.py (no GPU): the PLL stream's CU split by channel count."""
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import bench  # noqa: E402


def _se_balanced(cus: int) -> bool:
    """Stand-in for sdr_plls_fits on CPU: masks [0, n) whose CUs fall evenly on every XCC's four
    shader engines (n <= 32 with n % 8 == 0, or n % 32 == 0), the ones the library's placement rule
    accepts at full residency (sdr_internal.h CuPlacement, profiles/r06/cumask/)."""
    return cus % 32 == 0 or (cus <= 32 and cus % 8 == 0)


def test_pll_cus_split():
    # the headline keeps one PLL wave per CU on 64 CUs; capacity counts trade PLL CUs for side-chain CUs
    assert bench.pll_cus(1024, _se_balanced) == 64
    assert bench.pll_cus(1536, _se_balanced) == 32
    assert bench.pll_cus(2048, _se_balanced) == 32
    assert bench.pll_cus(4096, _se_balanced) == 64
    for n in (1, 32, 100, 512, 1024, 3000, 8192):
        waves = 2 * ((2 * n + 63) // 64)
        cus = bench.pll_cus(n, _se_balanced)
        assert _se_balanced(cus)
        assert waves <= 4 * cus            # at most four waves per CU (one per SIMD)
    # only what the library accepts is picked: with 64 refused, 1024 channels fall back to 32 + 2 per CU
    assert bench.pll_cus(1024, lambda c: c != 64) in (72, 80, 32)


