"""CPU, world_size 2 over gloo: the multi-GPU path's channel sharding and per-block-step gather to
rank 0 (real-time-sdr_amd/sharding.py), and bench.py's own rank path (bench.run_rank: warm-up,
barrier-bracketed timing, max over ranks, gather, result line) driven end to end with a CPU stepper.
Each rank runs its own channel shard through the oracle's per-channel pipeline (the CPU checker; on
the GPU box this is the HIP pipeline) and the stereo audio and RDS bits gathered on rank 0 must equal
a single-process run over all channels."""
from __future__ import annotations

import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ROOT, load_pkg

NCH_PER_RANK = 2
NBLOCKS = 8          # RDS decoding starts at block 6 (rds.cpp:135)
WORLD = 2


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _channel_outputs(ch: int):
    import sys
    sys.path.insert(0, str(ROOT / "oracle"))
    import oracle
    pkg = load_pkg()
    import real_time_sdr_amd.synth as synth
    src = synth.FMMultiplexSource(ch)
    c = oracle.Channel(0, True)
    lr, bits = [], []
    for _ in range(NBLOCKS):
        fm = c.frontend(src.next_block())
        lr.append(c.stereo(fm))
        r = c.rds(fm)
        b = np.zeros(pkg.SDR_MAX_BITS, np.uint8)
        if r.get("bits") is not None:
            b[:len(r["bits"])] = r["bits"]
        bits.append(b)
    return np.stack(lr), np.stack(bits)


def _worker(rank: int, port: int, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        _work(rank, q)
    except BaseException as e:  # report instead of leaving the parent waiting
        q.put((rank, repr(e), None))
        raise
    finally:
        dist.destroy_process_group()


def _work(rank: int, q):
    pkg = load_pkg()
    from real_time_sdr_amd.sharding import BlockGather, channel_range, max_over_ranks
    first, n = channel_range(NCH_PER_RANK, rank)
    outs = [_channel_outputs(first + j) for j in range(n)]
    lr0 = outs[0][0]
    g = BlockGather(torch, dist, WORLD, {"lr": ((n,) + lr0.shape[1:], torch.int16),
                                         "bits": ((n, pkg.SDR_MAX_BITS), torch.uint8)}, "cpu")
    gathered = []
    for b in range(NBLOCKS):
        lr = torch.from_numpy(np.stack([o[0][b] for o in outs]))
        bits = torch.from_numpy(np.stack([o[1][b] for o in outs]))
        res = g.gather(lr=lr, bits=bits)
        if rank != 0:
            assert res is None
            continue
        gathered.append((torch.cat(res["lr"]).numpy().copy(), torch.cat(res["bits"]).numpy().copy()))
    t = max_over_ranks(torch, dist, 1.0 + rank, "cpu")
    q.put((rank, gathered, t))


def test_channel_range():
    load_pkg()
    import real_time_sdr_amd.sharding as sh
    assert sh.channel_range(1024, 0) == (0, 1024)
    assert sh.channel_range(1024, 7) == (7168, 1024)
    with pytest.raises(ValueError):
        sh.channel_range(0, 0)


@pytest.mark.timeout(300)
def test_two_rank_gather_equals_single_process():
    load_pkg()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    results = {}
    for _ in range(WORLD):
        rank, gathered, t = q.get(timeout=240)
        assert not isinstance(gathered, str), f"rank {rank} failed: {gathered}"
        results[rank] = (gathered, t)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref = [_channel_outputs(c) for c in range(WORLD * NCH_PER_RANK)]
    for rank, (gathered, t) in results.items():
        assert t == 2.0, "max over ranks"
        if rank != 0:
            assert gathered == [], "only rank 0 receives the gather"
            continue
        for b in range(NBLOCKS):
            lr, bits = gathered[b]
            for c in range(WORLD * NCH_PER_RANK):
                assert np.array_equal(lr[c], ref[c][0][b]), f"rank {rank} block {b} channel {c} audio"
                assert np.array_equal(bits[c], ref[c][1][b]), f"rank {rank} block {b} channel {c} bits"
    # RDS decodes from block 6 on: the gathered bits are not trivially empty
    assert any(results[0][0][b][1].any() for b in range(6, NBLOCKS))


# ---------------------------------------------------------------- bench.py's rank path, world 2
class _OracleStepper:
    """bench.run_rank's stepper interface over the oracle (CPU): one block of every channel of this
    rank per step, then the gather hook bench.py's GPU stepper calls after its post stage."""

    last = None

    def __init__(self, args, nch, first, local, nblocks):
        import types
        import oracle
        pkg = load_pkg()
        import real_time_sdr_amd.synth as synth
        self.pkg, self.nch = pkg, nch
        self.srcs = [synth.FMMultiplexSource(first + j) for j in range(nch)]
        self.chans = [oracle.Channel(0, True) for _ in range(nch)]
        self.info = types.SimpleNamespace(block_iq=synth.BLOCK_IQ)
        self.received = []
        self.steps = []
        _OracleStepper.last = self

    def outputs_spec(self):
        return {"lr": ((self.nch, 2940), torch.int16), "bits": ((self.nch, self.pkg.SDR_MAX_BITS), torch.uint8)}

    def step(self, b, gather=None):
        lr, bits = [], []
        for src, c in zip(self.srcs, self.chans):
            fm = c.frontend(src.next_block())
            lr.append(c.stereo(fm))
            r = c.rds(fm)
            v = np.zeros(self.pkg.SDR_MAX_BITS, np.uint8)
            if r.get("bits") is not None:
                v[:len(r["bits"])] = r["bits"]
            bits.append(v)
        self.steps.append(b)
        if gather is not None:
            res = gather(lr=torch.from_numpy(np.stack(lr)), bits=torch.from_numpy(np.stack(bits)))
            if res is not None:
                self.received.append((torch.cat(res["lr"]).numpy().copy(), torch.cat(res["bits"]).numpy().copy()))

    def synchronize(self):
        pass

    def report(self, warmup, elapsed, steps):
        return {"stepper": "oracle (CPU test)"}

    def captured(self):
        return None


class _PendingStepper(_OracleStepper):
    """The oracle stepper declaring what the GPU stepper declares with a persistent PLL: a launch is
    pending from each begin_phase to the phase's synchronize (bench.LaunchWindow guards that span),
    and a prime_gather round before the first phase. Records the order of the rank path's calls."""

    launch_pending = True

    def __init__(self, *a, **k):
        super().__init__(*a, **k)
        self.log = []

    def prime_gather(self, gather):
        self.log.append("prime")
        z = self.outputs_spec()
        res = gather(lr=torch.zeros(z["lr"][0], dtype=z["lr"][1]), bits=torch.zeros(z["bits"][0], dtype=z["bits"][1]))
        assert (res is None) == (dist.get_rank() != 0)

    def begin_phase(self, n):
        self.log.append(f"begin {n}")

    def step(self, b, gather=None):
        self.log.append(f"step {b}")
        super().step(b, gather)

    def synchronize(self):
        self.log.append("sync")


class _CollectiveInWindowStepper(_PendingStepper):
    """Misbehaves: a barrier inside the timed phase's pending-launch window."""

    def step(self, b, gather=None):
        super().step(b, gather)
        if b == 3:
            dist.barrier()


def _bench_worker(rank: int, port: int, q, factory=None):
    import argparse
    import bench
    factory = factory or _OracleStepper
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(WORLD))
    args = argparse.Namespace(channels=NCH_PER_RANK, warmup=2, steps=NBLOCKS - 2, no_gather=False,
                              no_isolated=True, no_cpu_baseline=True, numerics="exact")
    try:
        res = bench.run_rank(args, WORLD, rank, 0, stepper_factory=factory, backend="gloo")
        st = _OracleStepper.last
        q.put((rank, res, st.received, getattr(st, "log", st.steps)))
    except BaseException as e:
        q.put((rank, repr(e), None, None))
        raise


@pytest.mark.timeout(300)
def test_bench_rank_path_world2_gloo():
    """bench.run_rank on 2 gloo ranks: one result line on rank 0 with n_gpus 2 and the whole job's
    samples, and every block's audio + RDS bits of both shards gathered to rank 0 bit-exactly."""
    import sys
    sys.path.insert(0, str(ROOT))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bench_worker, args=(r, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    got = {}
    for _ in range(WORLD):
        rank, res, received, steps = q.get(timeout=240)
        assert not isinstance(res, str), f"rank {rank} failed: {res}"
        got[rank] = (res, received, steps)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res0 = got[0][0]
    assert got[1][0] is None and got[1][1] == [], "only rank 0 reports and receives"
    assert res0["n_gpus"] == WORLD and res0["scaling"] == "weak"
    assert res0["config"]["channels_total"] == WORLD * NCH_PER_RANK
    assert res0["steps"] == NBLOCKS - 2 and res0["warmup"] == 2
    want_value = WORLD * NCH_PER_RANK * 73500 * (NBLOCKS - 2) / (res0["ms_per_step"] * (NBLOCKS - 2) / 1e3) / 1e6
    assert abs(res0["value"] - want_value) / want_value < 1e-2
    assert res0["gathered"]["ranks"] == WORLD and res0["gathered"]["steps"] == NBLOCKS
    assert got[0][2] == list(range(NBLOCKS)) and got[1][2] == list(range(NBLOCKS))
    ref = [_channel_outputs(c) for c in range(WORLD * NCH_PER_RANK)]
    received = got[0][1]
    assert len(received) == NBLOCKS
    for b in range(NBLOCKS):
        lr, bits = received[b]
        for c in range(WORLD * NCH_PER_RANK):
            assert np.array_equal(lr[c], ref[c][0][b]), f"block {b} channel {c} audio"
            assert np.array_equal(bits[c], ref[c][1][b]), f"block {b} channel {c} bits"


def test_bench_gpus_flag_fails_without_gpus():
    """bench.py --gpus 2 starts two ranks itself; with fewer GPUs visible it fails loudly."""
    import subprocess
    import sys
    if torch.cuda.device_count() >= 2:
        pytest.skip("2+ GPUs visible")
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--steps", "1", "--warmup", "0"],
                       capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode != 0
    assert "GPU(s) visible" in r.stderr


def test_cpu_baseline_untimed_above_one_gpu():
    """At N > 1 the CPU baseline legs are not re-timed (they are quoted on the N = 1 line); the
    rank-0 line still carries the object, with value None and the reason."""
    import argparse
    import sys
    sys.path.insert(0, str(ROOT))
    import bench
    res = bench.cpu_baseline_leg(argparse.Namespace(), None, timing=False)
    assert res["value"] is None and "N > 1" in res["sample"] and "verified" not in res


def _run_bench_ranks(factory):
    import sys
    sys.path.insert(0, str(ROOT))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bench_worker, args=(r, port, q, factory)) for r in range(WORLD)]
    for p in procs:
        p.start()
    got = {}
    for _ in range(WORLD):
        rank, res, received, log = q.get(timeout=240)
        got[rank] = (res, received, log)
    for p in procs:
        p.join(timeout=60)
    return got, [p.exitcode for p in procs]


@pytest.mark.timeout(300)
def test_bench_rank_path_primes_gather_before_pending_launch():
    """With a persistent launch per phase (the GPU stepper's default), run_rank does one untimed gather
    round before the first begin_phase (RCCL's lazy set-up and the capture buffers happen outside any
    pending launch), and inside each phase's window only the per-step gathers run: the rows gathered
    to rank 0 still equal a single-process run, block for block."""
    got, codes = _run_bench_ranks(_PendingStepper)
    assert codes == [0, 0], got
    for rank in range(WORLD):
        res, received, log = got[rank]
        assert not isinstance(res, str), f"rank {rank} failed: {res}"
        want = (["prime", "sync", "begin 2", "step 0", "step 1", "sync", "sync", "begin 6"] +
                [f"step {b}" for b in range(2, NBLOCKS)] + ["sync"])
        assert log[:len(want)] == want, log
    res0, received, _ = got[0]
    assert res0["gathered"]["steps"] == NBLOCKS + 1          # the priming round + one per block-step
    assert len(received) == NBLOCKS
    ref = [_channel_outputs(c) for c in range(WORLD * NCH_PER_RANK)]
    for b in range(NBLOCKS):
        lr, bits = received[b]
        for c in range(WORLD * NCH_PER_RANK):
            assert np.array_equal(lr[c], ref[c][0][b]) and np.array_equal(bits[c], ref[c][1][b]), (b, c)


@pytest.mark.timeout(300)
def test_bench_rank_path_rejects_collective_in_launch_window():
    """A torch.distributed call other than the per-step gather while a phase's persistent launch is
    pending (here a barrier in the timed phase) fails the run on every rank instead of stalling the
    blocking PLL stream (bench.LaunchWindow)."""
    got, codes = _run_bench_ranks(_CollectiveInWindowStepper)
    for rank in range(WORLD):
        res = got[rank][0]
        assert isinstance(res, str) and "pending persistent PLL launch" in res, (rank, res)
    assert all(c != 0 for c in codes)
