"""GPU parity at the bench's width: 1024 distinct channels x 8 blocks through the full exact
pipeline in bench.py's split-stage schedule (front end + pre-PLL FIRs, both PLLs, post stage, each
on its own CU-masked HIP stream), for both PLL schedules: one sdr_plls dispatch per block, and the
bench's default, ONE persistent sdr_plls_launch for all blocks with per-block signal / wait. Inputs
include hostile channels a 1024-channel
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


KEYS = ("fm", "mono", "lr", "clean", "offset", "nsym", "symbols", "nbits", "bits")
# persistent_packed: the PLL stream on 16 CUs -- 64 waves, four per CU in workgroups of four sharing a
# trigArg table, the LDS-staged lane-pair loop (sdr_pll.hip pll_run_split_coal, k_pll_multi<..., 4,
# true>) that the 2048- and 4096-channel capacity lines run
SCHEDULES = ("dispatch", "persistent", "persistent_parts", "persistent_release", "persistent_packed")


def _check(args):
    """Worker: oracle on channels [lo, hi) of the memory-mapped inputs, compared with the GPU outputs
    of every schedule (the oracle runs once per channel)."""
    path, lo, hi = args
    sys.path.insert(0, str(ROOT / "oracle"))
    import oracle
    iq = np.load(os.path.join(path, "iq.npy"), mmap_mode="r")
    runs = {sch: {k: np.load(os.path.join(path, f"{sch}_{k}.npy"), mmap_mode="r") for k in KEYS}
            for sch in SCHEDULES if os.path.exists(os.path.join(path, f"{sch}_fm.npy"))}
    bad = {sch: [] for sch in runs}
    for c in range(lo, hi):
        ref = oracle.run_channel(np.ascontiguousarray(iq[:, c]), 0, True)
        for sch, d in runs.items():
            for b in range(NBLOCKS):
                where = f"ch{c} b{b}"
                if not np.array_equal(d["fm"][b, c].view(np.uint32), ref["fm_demod"][b].view(np.uint32)):
                    bad[sch].append(f"fm_demod {where}")
                if not np.array_equal(d["mono"][b, c], ref["mono"][b]):
                    bad[sch].append(f"mono {where}")
                if not np.array_equal(d["lr"][b, c], ref["stereo"][b]):
                    bad[sch].append(f"stereo {where}")
                if not np.array_equal(d["clean"][b, c].view(np.uint32), ref["rds_clean"][b].view(np.uint32)):
                    bad[sch].append(f"rds_clean {where}")
                if ref["bits"][b] is None:
                    if int(d["nbits"][b, c]) != -1:
                        bad[sch].append(f"nbits {where}")
                    continue
                if int(d["offset"][b, c]) != int(ref["offset"][b]):
                    bad[sch].append(f"offset {where}")
                ns = int(d["nsym"][b, c])
                if ns != len(ref["symbols"][b]) or not np.array_equal(d["symbols"][b, c, :ns], ref["symbols"][b]):
                    bad[sch].append(f"symbols {where}")
                nb = int(d["nbits"][b, c])
                if nb != len(ref["bits"][b]) or not np.array_equal(d["bits"][b, c, :nb], ref["bits"][b]):
                    bad[sch].append(f"bits {where}")
    return bad


def _run_schedule(torch, pkg, bench, iq, dev, schedule: str) -> dict:
    """bench.GpuStepper.step on a fresh context with its outputs captured: front end + pre-PLL FIRs on
    one CU-masked stream, the PLLs on another (one sdr_plls dispatch per block, or ONE persistent
    sdr_plls_launch for all blocks with per-block signal / wait -- the bench's default), the post
    stage on a third."""
    pipe = pkg.Pipeline(NCH, mode=0, rds_on=True, device=0)
    info = pipe.info
    created: list[int] = []
    pll_cus = "16" if schedule == "persistent_packed" else "64"
    if schedule == "persistent_packed":   # four waves per CU in groups of four: the staged loop
        assert pipe.plls_fits(16) == {"waves": 64, "groups": 16, "resident": 16, "fits": True}
    try:
        s_fe, s_pll, s_post, _ = bench.cu_masked_streams(torch, pkg, dev, pll_cus, created)
    except (RuntimeError, AttributeError):
        if schedule.startswith("persistent"):
            pytest.skip("no CU-masked streams: the bench does not run the persistent PLL without them")
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
    persistent = schedule.startswith("persistent")
    parts = 4 if schedule == "persistent_parts" else 0
    if persistent:
        pipe.plls_launch(NBLOCKS, stream=s_pll)
    for b in range(NBLOCKS):                               # bench.GpuStepper.step, outputs captured
        # persistent_release: no wait of the caller's own -- the library orders the reuse of block
        # b-2's parity (its mono / stereo post / RDS mixer release counts, sdr_frontend's wait)
        if b >= 2 and schedule != "persistent_release":
            s_fe.wait_event(post_done[b - 2])
        if parts and b == 0:
            # the pipeline fill: the launch's first block in sample ranges, each published to the PLLs
            pipe.frontend_pre_parts(iq[b], parts, stream=s_fe)
            pipe.fm_demod(cap["fm"][b], stream=s_fe)
            pipe.mono(cap["mono"][b], stream=s_fe)
        else:
            pipe.frontend(iq[b], stream=s_fe)
            pipe.fm_demod(cap["fm"][b], stream=s_fe)
            pipe.mono(cap["mono"][b], stream=s_fe)
            pipe.pre(stream=s_fe)                          # stereo_pre + rds_pre, one staged window
            if persistent:
                pipe.plls_signal(stream=s_fe)
        if persistent:
            pipe.plls_wait(stream=s_post)
        else:
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
    if persistent:
        ms = pipe.plls_report(stream=s_pll)                # raises if a block's wait timed out
        assert len(ms) == NBLOCKS
    host = {k: v.cpu().numpy() for k, v in cap.items()}
    pipe.close()
    bench.destroy_masked_streams(torch, pkg, dev, created)
    return host


@pytest.fixture(scope="module")
def width_mismatches(pkg, synth, tmp_path_factory):
    """Both schedules on the same 1024 hostile channels; one oracle pass checks both."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    sys.path.insert(0, str(ROOT))
    import bench
    dev = torch.device("cuda", 0)
    kinds = _kinds(synth)
    iq = bench.make_input(torch, NCH, NBLOCKS, first_channel=0, device=dev, kinds=kinds, seed=5)
    tmp = str(tmp_path_factory.mktemp("width"))
    np.save(os.path.join(tmp, "iq.npy"), iq.cpu().numpy())
    for sch in SCHEDULES:
        host = _run_schedule(torch, pkg, bench, iq, dev, sch)
        for k, v in host.items():
            np.save(os.path.join(tmp, f"{sch}_{k}.npy"), np.ascontiguousarray(v))
        del host
    del iq
    workers = max(1, min(16, os.cpu_count() or 1))
    step = (NCH + 4 * workers - 1) // (4 * workers)
    jobs = [(tmp, lo, min(NCH, lo + step)) for lo in range(0, NCH, step)]
    bad = {sch: [] for sch in SCHEDULES}
    with cf.ProcessPoolExecutor(workers, mp_context=mp.get_context("spawn")) as ex:
        for r in ex.map(_check, jobs):
            for sch, v in r.items():
                bad[sch].extend(v)
    return bad, set(kinds)


@pytest.mark.parametrize("schedule", SCHEDULES)
def test_full_width_hostile_channels_bit_exact(width_mismatches, schedule):
    bad, kinds = width_mismatches
    assert not bad[schedule], f"{schedule}: {len(bad[schedule])} mismatches, first: {bad[schedule][:10]} (kinds: {kinds})"
