"""GPU parity at the bench's width: 1024 distinct channels x 8 blocks through the full exact
pipeline in bench.py's split-stage schedule (front end + pre-PLL FIRs, both PLLs in one dispatch,
post stage, each on its own CU-masked HIP stream), including hostile channels a 1024-channel
receiver meets -- silence (all bytes 128: I = Q = 0, demod.cpp:10-12 and atan2(+-0, +-0) in the
PLL), rail (all 255), saturated, random bytes, no pilot, no RDS, DC offset, a pilot 3 Hz off
(phaseEst drifts), a 40 kHz carrier offset, and a weak signal. Every output of every channel and
block (fm_demod, mono, stereo, rds_clean, cdr offset, symbols, bits) is compared bit for bit with the
oracle run on the same input bytes in a CPU process pool.

Reference: rffrontend.cpp:58-71, demod.cpp:8-19, pll.cpp:34-53, stereo.cpp:69-114, rds.cpp:95-167."""
from __future__ import annotations

import concurrent.futures as cf
import multiprocessing as mp
import os
import sys
import tempfile

import numpy as np
import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

NCH = 1024
NBLOCKS = 8
HOSTILE_EACH = 3          # channels per hostile kind, spread over the batch


def _kinds(synth):
    kinds = ["normal"] * NCH
    hostile = [k for k in synth.KINDS if k != "normal"]
    slots = np.linspace(5, NCH - 7, len(hostile) * HOSTILE_EACH).astype(int)
    for i, s in enumerate(slots):
        kinds[s] = hostile[i % len(hostile)]
    return kinds


def _check(args):
    """Worker: oracle on channels [lo, hi) of the memory-mapped inputs, compared with the GPU."""
    path, lo, hi = args
    sys.path.insert(0, str(ROOT / "oracle"))
    import oracle
    d = {k: np.load(os.path.join(path, k + ".npy"), mmap_mode="r")
         for k in ("iq", "fm", "mono", "lr", "clean", "offset", "nsym", "symbols", "nbits", "bits")}
    bad = []
    for c in range(lo, hi):
        ref = oracle.run_channel(np.ascontiguousarray(d["iq"][:, c]), 0, True)
        for b in range(NBLOCKS):
            where = f"ch{c} b{b}"
            if not np.array_equal(d["fm"][b, c].view(np.uint32), ref["fm_demod"][b].view(np.uint32)):
                bad.append(f"fm_demod {where}")
            if not np.array_equal(d["mono"][b, c], ref["mono"][b]):
                bad.append(f"mono {where}")
            if not np.array_equal(d["lr"][b, c], ref["stereo"][b]):
                bad.append(f"stereo {where}")
            if not np.array_equal(d["clean"][b, c].view(np.uint32), ref["rds_clean"][b].view(np.uint32)):
                bad.append(f"rds_clean {where}")
            if ref["bits"][b] is None:
                if int(d["nbits"][b, c]) != -1:
                    bad.append(f"nbits {where}")
                continue
            if int(d["offset"][b, c]) != int(ref["offset"][b]):
                bad.append(f"offset {where}")
            ns = int(d["nsym"][b, c])
            if ns != len(ref["symbols"][b]) or not np.array_equal(d["symbols"][b, c, :ns], ref["symbols"][b]):
                bad.append(f"symbols {where}")
            nb = int(d["nbits"][b, c])
            if nb != len(ref["bits"][b]) or not np.array_equal(d["bits"][b, c, :nb], ref["bits"][b]):
                bad.append(f"bits {where}")
    return bad


def test_full_width_hostile_channels_bit_exact(pkg, synth):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    sys.path.insert(0, str(ROOT))
    import bench
    dev = torch.device("cuda", 0)
    kinds = _kinds(synth)
    iq = bench.make_input(torch, NCH, NBLOCKS, first_channel=0, device=dev, kinds=kinds, seed=5)
    pipe = pkg.Pipeline(NCH, mode=0, rds_on=True, device=0)
    info = pipe.info
    created: list[int] = []
    try:
        s_fe, s_pll, s_post = bench.cu_masked_streams(torch, pkg, dev, "64", created)
    except (RuntimeError, AttributeError):
        s_fe, s_pll, s_post = (torch.cuda.Stream(dev) for _ in range(3))
    E = lambda: torch.cuda.Event()  # noqa: E731
    pre_done, pll_done, post_done = ([E() for _ in range(NBLOCKS)] for _ in range(3))
    u8, i32 = torch.uint8, torch.int32
    cap = {"fm": torch.empty(NBLOCKS, NCH, info.block_if, dtype=torch.float32, device=dev),
           "mono": torch.empty(NBLOCKS, NCH, info.n_audio, dtype=torch.int16, device=dev),
           "lr": torch.empty(NBLOCKS, NCH, 2 * info.n_audio, dtype=torch.int16, device=dev),
           "clean": torch.empty(NBLOCKS, NCH, info.n_rds, dtype=torch.float32, device=dev),
           "offset": torch.empty(NBLOCKS, NCH, dtype=i32, device=dev),
           "nsym": torch.empty(NBLOCKS, NCH, dtype=i32, device=dev),
           "symbols": torch.empty(NBLOCKS, NCH, pkg.SDR_MAX_SYMS, dtype=u8, device=dev),
           "nbits": torch.empty(NBLOCKS, NCH, dtype=i32, device=dev),
           "bits": torch.empty(NBLOCKS, NCH, pkg.SDR_MAX_BITS, dtype=u8, device=dev)}
    for b in range(NBLOCKS):                               # bench.GpuStepper.step, outputs captured
        if b >= 2:
            s_fe.wait_event(post_done[b - 2])
        pipe.frontend(iq[b], stream=s_fe)
        pipe.fm_demod(cap["fm"][b], stream=s_fe)
        pipe.mono(cap["mono"][b], stream=s_fe)
        pipe.stereo_pre(stream=s_fe)
        pipe.rds_pre(stream=s_fe)
        pre_done[b].record(s_fe)
        s_pll.wait_event(pre_done[b])
        pipe.plls(stream=s_pll)
        pll_done[b].record(s_pll)
        s_post.wait_event(pll_done[b])
        pipe.stereo_post(cap["lr"][b], stream=s_post)
        pipe.rds_post(cap["clean"][b], bits=True, stream=s_post)
        with torch.cuda.stream(s_post):
            for k in ("offset", "nsym", "symbols", "nbits", "bits"):
                cap[k][b].copy_(getattr(pipe, k))
        post_done[b].record(s_post)
    torch.cuda.synchronize(dev)
    host = {k: v.cpu().numpy() for k, v in cap.items()}
    host["iq"] = iq.cpu().numpy()
    pipe.close()
    bench.destroy_masked_streams(torch, pkg, dev, created)
    del iq, cap
    with tempfile.TemporaryDirectory() as tmp:
        for k, v in host.items():
            np.save(os.path.join(tmp, k + ".npy"), np.ascontiguousarray(v))
        del host
        workers = max(1, min(16, os.cpu_count() or 1))
        step = (NCH + 4 * workers - 1) // (4 * workers)
        jobs = [(tmp, lo, min(NCH, lo + step)) for lo in range(0, NCH, step)]
        bad = []
        with cf.ProcessPoolExecutor(workers, mp_context=mp.get_context("spawn")) as ex:
            for r in ex.map(_check, jobs):
                bad.extend(r)
    assert not bad, f"{len(bad)} mismatches, first: {bad[:10]} (kinds: {set(kinds)})"
