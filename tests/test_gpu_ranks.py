"""GPU, world_size 2 on ONE device: bench.py's own rank path (bench.run_rank with the real GpuStepper:
device-generated channels, the three CU-masked stage streams, the persistent PLL launch, the gather
stream) in two processes at once, joined over gloo with a host-staged gather of every block-step's
stereo audio and RDS bits to rank 0. This is the multi-GPU path of BASELINE configs[4] on the one
GPU a test box has: both ranks' persistent PLL launches, signal kernels and gather streams are live
on the same device together, so a PLL queue shared with a later dispatch would show up here as the
5 s wait error (sdr_plls_report) instead of on an 8-GPU node.

Checks: rank 0's line (n_gpus 2, weak scaling, whole-job samples), the PLL mode, each rank's
captured channels bit-exact against the oracle, and the rows rank 0 received from each rank equal
to the rows that rank produced (digests). Reference: project.cpp:134-136 (the stage threads),
pll.cpp:34-53, stereo.cpp:77-107, rds.cpp:105-167."""
from __future__ import annotations

import os
import socket
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

WORLD = 2
NCH = 64            # channels per rank
WARMUP, STEPS = 2, 6


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank: int, port: int, q):
    import argparse
    sys.path.insert(0, str(ROOT))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(WORLD),
                      LOCAL_RANK="0", SDR_BENCH_CPU_CORES="4")
    import bench
    args = argparse.Namespace(channels=NCH, warmup=WARMUP, steps=STEPS, no_gather=False, no_isolated=True,
                              no_cpu_baseline=False, numerics="exact", gpus=WORLD, backend="gloo")
    try:
        res = bench.run_rank(args, WORLD, rank, 0, backend="gloo")
        q.put((rank, res))
    except BaseException as e:
        q.put((rank, repr(e)))
        raise


@pytest.mark.timeout(600)
def test_bench_rank_path_world2_one_device():
    import torch
    import torch.multiprocessing as mp
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    got = {}
    try:
        for _ in range(WORLD):
            rank, res = q.get(timeout=540)
            assert not isinstance(res, str), f"rank {rank} failed: {res}"
            got[rank] = res
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    assert all(p.exitcode == 0 for p in procs)
    res0 = got[0]
    assert got[1] is None, "only rank 0 reports"
    assert res0["n_gpus"] == WORLD and res0["scaling"] == "weak"
    assert res0["config"]["channels_total"] == WORLD * NCH
    assert res0["steps"] == STEPS and res0["warmup"] == WARMUP
    assert res0["pll"]["mode"].startswith("persistent"), res0["pll"]["mode"]
    # one untimed priming round (RCCL's lazy set-up outside any pending PLL launch) + one per block
    assert res0["gathered"]["ranks"] == WORLD and res0["gathered"]["steps"] == 1 + WARMUP + STEPS
    vr = res0["verified_ranks"]
    assert vr["ranks_oracle_ok"], vr["mismatches"]
    assert vr["gather_rows_equal"] is True
    assert sorted(vr["channels"]) == [0, 1] and min(vr["channels"][1]) >= NCH
    assert res0["verified"] is True
