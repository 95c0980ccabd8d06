"""GPU, world_size 1: bench.py's timed phase as the driver runs it (bench.run_rank with the real
GpuStepper), at a small width: the persistent PLL launch per phase, the first block's front end and
pre-PLL FIRs and the last block's post stage on the all-CU stream, mono after the PLL signal. Every
block's captured mono, stereo and RDS bits of the sampled channels bit-exact against the oracle
(bench.verify_captured), and the timeline the bench reports (fill, drain, PLL span) present.
Reference: project.cpp:134-136, rffrontend.cpp:58-71, mono.cpp:34-42, stereo.cpp:77-107,
rds.cpp:105-167."""
from __future__ import annotations

import argparse
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


@pytest.mark.timeout(300)
def test_bench_phase_edges_world1(monkeypatch):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    sys.path.insert(0, str(ROOT))
    import bench
    monkeypatch.setenv("SDR_BENCH_CPU_CORES", "4")
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    args = argparse.Namespace(channels=48, warmup=3, steps=5, no_gather=True, no_isolated=True,
                              no_cpu_baseline=False, cpu_timing=False, numerics="exact", gpus=1, backend="nccl")
    res = bench.run_rank(args, 1, 0, 0)
    assert res["verified"] is True, res.get("cpu_baseline", {}).get("verified")
    pll = res["pll"]
    assert pll["mode"] == "persistent", pll["mode"]
    tl = pll["timeline"]
    assert tl["fill_ms"] > 0 and tl["drain_ms"] > 0 and tl["pll_span_ms"] > 0, tl
    assert res["steps"] == 5 and res["n_gpus"] == 1
