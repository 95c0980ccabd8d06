"""CPU, world_size 2 over gloo: the multi-GPU path's channel sharding and per-block-step gather
(real-time-sdr_amd/sharding.py, used by bench.py). Each rank runs its own channel shard through the
oracle's per-channel pipeline (the CPU checker; on the GPU box this is the HIP pipeline) and the
gathered stereo audio and RDS bits on every rank must equal a single-process run over all channels."""
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
        gathered.append((res["lr"].numpy().copy(), res["bits"].numpy().copy()))
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
        for b in range(NBLOCKS):
            lr, bits = gathered[b]
            for c in range(WORLD * NCH_PER_RANK):
                assert np.array_equal(lr[c], ref[c][0][b]), f"rank {rank} block {b} channel {c} audio"
                assert np.array_equal(bits[c], ref[c][1][b]), f"rank {rank} block {b} channel {c} bits"
    # RDS decodes from block 6 on: the gathered bits are not trivially empty
    assert any(results[0][0][b][1].any() for b in range(6, NBLOCKS))
