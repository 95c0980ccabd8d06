#!/usr/bin/env python3
"""Throughput benchmark of the MI355X FM/RDS hot path (BASELINE.json metric).

One step = one block (73 500 I/Q pairs = 30.6 ms of signal) of every channel through the full
reference pipeline of `project 0 r` plus the mono stage: RF front end (u8 I/Q -> FIR /10 ->
discriminator), mono audio, stereo audio (pilot PLL, mixer, resamplers), RDS DSP (BPF, squaring,
PLL, mixer, 247/640 resampler, RRC) and RDS bit recovery (cdr, slicer, Manchester, differential).
Channels are independent and sharded across GPUs (weak scaling: 1024 channels per GPU); inputs are
synthetic FM multiplex I/Q, generated on the host and resident in HBM before the timed region.

Three HIP streams per GPU mirror the reference's three threads (project.cpp:134-136): the front end
produces block b+1 while the stereo and RDS chains consume block b, ordered by events exactly like
the ThreadSafeQueue protocol (include/threadsafequeue.h:24-74).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--channels C] [--no-cpu-baseline]
For N > 1 launch with torch.distributed.run (one process per GPU, RCCL gather of audio + RDS bits).
"""
from __future__ import annotations

import argparse
import json
import os
import pathlib
import shutil
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parent
HBM_PEAK_GBS = 8000.0           # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)


def _load_pkg():
    import importlib.util
    d = ROOT / "real-time-sdr_amd"
    if "real_time_sdr_amd" in sys.modules:
        return sys.modules["real_time_sdr_amd"]
    spec = importlib.util.spec_from_file_location("real_time_sdr_amd", d / "__init__.py",
                                                  submodule_search_locations=[str(d)])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["real_time_sdr_amd"] = mod
    spec.loader.exec_module(mod)
    return mod


def cu_masked_streams(torch, pkg, dev, spec: str):
    """(fe, pll, post) streams on disjoint CUs through the C ABI (sdr_stream_create_cu_range):
    the PLL stream on CUs [0, n), the other two on the rest."""
    import ctypes as C
    n = int(spec)
    L = pkg.lib()
    L.sdr_stream_create_cu_range.restype = C.c_int
    L.sdr_stream_create_cu_range.argtypes = [C.POINTER(C.c_void_p), C.c_int, C.c_int, C.c_int, C.c_int]
    out = []
    for exclude in (1, 0, 1):
        h = C.c_void_p()
        rc = L.sdr_stream_create_cu_range(C.byref(h), dev.index, 0, n, exclude)
        if rc != 0:
            raise RuntimeError(f"sdr_stream_create_cu_range: {rc} {L.sdr_last_error()}")
        _MASKED_STREAMS.append(h.value)
        out.append(torch.cuda.ExternalStream(h.value, device=dev))
    return tuple(out)


_MASKED_STREAMS: list[int] = []


def destroy_masked_streams(torch, pkg, dev) -> None:
    """sdr_stream_destroy the streams cu_masked_streams made (torch does not own them)."""
    import ctypes as C
    if not _MASKED_STREAMS:
        return
    torch.cuda.synchronize(dev)
    L = pkg.lib()
    L.sdr_stream_destroy.restype = C.c_int
    L.sdr_stream_destroy.argtypes = [C.c_void_p]
    while _MASKED_STREAMS:
        L.sdr_stream_destroy(C.c_void_p(_MASKED_STREAMS.pop()))


def _synth_module():
    import importlib.util
    spec = importlib.util.spec_from_file_location("sdr_synth", ROOT / "real-time-sdr_amd" / "synth.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _synth_channel(channel: int, nblocks: int) -> np.ndarray:
    """nblocks consecutive u8 I/Q blocks of one synthetic channel (numpy only, no GPU)."""
    synth = _synth_module()
    src = synth.FMMultiplexSource(channel)
    return np.stack([src.next_block() for _ in range(nblocks)])


def synth_host_input(nch: int, nblocks: int, first_channel: int) -> np.ndarray:
    """[nblocks][distinct][2*73500] u8 on the host for min(nch, 16) distinct channels, synthesised in
    child processes (about 23 ms per channel-block; call before the GPU is initialised)."""
    import concurrent.futures as cf
    import multiprocessing as mp
    distinct = min(nch, 16)
    workers = max(1, min(distinct, 8, os.cpu_count() or 1))
    if workers == 1 or nblocks * distinct < 64:
        chans = [_synth_channel(first_channel + c, nblocks) for c in range(distinct)]
    else:
        with cf.ProcessPoolExecutor(workers, mp_context=mp.get_context("spawn")) as ex:
            chans = list(ex.map(_synth_channel, [first_channel + c for c in range(distinct)],
                                [nblocks] * distinct))
    return np.ascontiguousarray(np.stack(chans, axis=1))


def make_input(torch, nch: int, nblocks: int, first_channel: int, device, host: np.ndarray | None = None):
    """[nblocks][nch][2*73500] u8 on the device. A few distinct channels are synthesised and tiled
    across the batch (each channel stays a continuous FM stream across blocks)."""
    synth = _synth_module()
    if host is None:
        host = synth_host_input(nch, nblocks, first_channel)
    distinct = host.shape[1]
    # rows padded to a multiple of 16 bytes (147008 for 147000): the front end then stages whole
    # 16-byte I/Q groups
    row = 2 * synth.BLOCK_IQ
    d = torch.empty((nblocks, nch, (row + 15) // 16 * 16), dtype=torch.uint8, device=device)[:, :, :row]
    reps = (nch + distinct - 1) // distinct
    src_t = torch.from_numpy(host).to(device)
    for r in range(reps):
        lo, hi = r * distinct, min(nch, (r + 1) * distinct)
        d[:, lo:hi] = src_t[:, : hi - lo]
    return d


def cpu_baseline(seconds_target: float = 8.0) -> dict | None:
    """Time the reference's own program (oracle/_ref/project, built from the unmodified sources)
    in its 3-thread topology on this host, over a bounded sample piped through stdin."""
    sys.path.insert(0, str(ROOT / "real-time-sdr_amd"))
    import synth
    exe = ROOT / "oracle" / "_ref" / "project"
    nblk_distinct = 32
    src = synth.FMMultiplexSource(0)
    blob = b"".join(src.next_block().tobytes() for _ in range(nblk_distinct))
    samples_per_blob = nblk_distinct * synth.BLOCK_IQ
    if exe.exists():
        reps = 150  # 4800 blocks = 353 M I/Q samples (~10 s at the reference's ~37 MS/s)
        with tempfile.TemporaryFile() as out:
            t0 = time.perf_counter()
            p = subprocess.Popen([str(exe), "0", "r"], stdin=subprocess.PIPE, stdout=out, stderr=subprocess.DEVNULL)
            try:
                for _ in range(reps):
                    p.stdin.write(blob)
                p.stdin.close()
            except BrokenPipeError:
                pass
            p.wait()
            dt = time.perf_counter() - t0
        ms = reps * samples_per_blob / dt / 1e6
        return {"value": round(ms, 3), "unit": "MS/s", "cores": 3, "kind": "reference",
                "sample": f"reference `project 0 r` (src/*.cpp, g++ -O3, 3 threads RF/audio/RDS) on "
                          f"{reps * nblk_distinct} blocks = {reps * samples_per_blob / 1e6:.1f} M I/Q samples "
                          f"of 1 channel via stdin, {dt:.2f} s wall",
                "host_cpu": _cpu_model(), "nproc": os.cpu_count()}
    # fallback: the C restatement, one core, full pipeline
    sys.path.insert(0, str(ROOT / "oracle"))
    import oracle
    ch = oracle.Channel(0, True)
    blocks = [np.frombuffer(blob, np.uint8)[i * 2 * synth.BLOCK_IQ:(i + 1) * 2 * synth.BLOCK_IQ]
              for i in range(nblk_distinct)]
    t0 = time.perf_counter()
    n = 0
    while time.perf_counter() - t0 < seconds_target:
        fm = ch.frontend(blocks[n % nblk_distinct])
        ch.mono(fm)
        ch.stereo(fm)
        ch.rds(fm)
        n += 1
    dt = time.perf_counter() - t0
    return {"value": round(n * synth.BLOCK_IQ / dt / 1e6, 3), "unit": "MS/s", "cores": 1, "kind": "port",
            "sample": f"oracle C restatement, 1 channel x {n} blocks, 1 thread, {dt:.2f} s",
            "host_cpu": _cpu_model(), "nproc": os.cpu_count()}


def _cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--channels", type=int, default=1024, help="channels per GPU")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-gather", action="store_true", help="skip the per-step RCCL gather (N>1)")
    ap.add_argument("--no-isolated", action="store_true", help="skip the isolated front-end timings")
    ap.add_argument("--numerics", choices=("exact", "fast"), default="exact",
                    help="exact: every output bit-identical to the reference; fast: the matrix-core front end "
                         "(fm_demod within 1e-5, RDS bits bit-exact)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    nblocks = args.warmup + args.steps
    # this rank's synthetic input, made in child processes before anything touches the GPU
    host_iq = synth_host_input(args.channels, nblocks, first_channel=rank * args.channels)

    import torch
    import torch.distributed as dist

    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    pkg = _load_pkg()

    from real_time_sdr_amd.sharding import channel_range
    first, nch = channel_range(args.channels, rank)
    assert first == rank * args.channels
    iq = make_input(torch, nch, nblocks, first_channel=first, device=dev, host=host_iq)
    del host_iq
    fast = args.numerics == "fast"
    pipe = pkg.Pipeline(nch, mode=0, rds_on=True, device=local, flags=pkg.FLAG_FAST_FRONTEND if fast else 0)
    info = pipe.info
    # Three streams, one HIP hardware queue each (GPU_MAX_HW_QUEUES is 4 and one serves the null
    # stream; a fourth stream would share a queue and serialise behind it): front end + mono + the
    # FIRs feeding both PLLs; both PLLs in one dispatch; everything after the PLLs. The serial PLLs
    # bound the step, so they run back to back across blocks while the other streams fill the chip.
    # SDR_BENCH_PRIO (A/B): comma list of streams (fe, pll, post) created with high priority
    prio = set(filter(None, os.environ.get("SDR_BENCH_PRIO", "").split(",")))
    s_fe, s_pll, s_post = (torch.cuda.Stream(dev, priority=-1 if n in prio else 0) for n in ("fe", "pll", "post"))
    # SDR_BENCH_CUMASK=<n> (default 64; 0 = no masks): the PLL stream gets CUs [0, n) of its
    # own, the front-end and post streams the complement,
    # so that no other kernel shares a CU's issue slots with the PLL's 32 lone waves. Measured
    # (profiles/r01/ab_cumask.txt): none 0.895 ms/step, 8 CUs 1.86, 16 0.99, 32 0.871, 48-96
    # 0.864-0.870, 128 0.911 (front end starved)
    cu_spec = os.environ.get("SDR_BENCH_CUMASK", "64")
    if cu_spec not in ("", "0"):
        try:
            s_fe, s_pll, s_post = cu_masked_streams(torch, pkg, dev, cu_spec)
        except (RuntimeError, ValueError, AttributeError) as exc:   # plain streams, reported
            print(f"bench: CU-masked streams unavailable ({exc}); unmasked streams", file=sys.stderr)
            destroy_masked_streams(torch, pkg, dev)
            cu_spec = ""
    mono = torch.empty(nch, info.n_audio, dtype=torch.int16, device=dev)
    lr = [torch.empty(nch, 2 * info.n_audio, dtype=torch.int16, device=dev) for _ in range(2)]
    bits = [torch.empty(nch, pkg.SDR_MAX_BITS, dtype=torch.uint8, device=dev) for _ in range(2)]
    clean = torch.empty(nch, info.n_rds, dtype=torch.float32, device=dev)
    ev = lambda: torch.cuda.Event(enable_timing=False)  # noqa: E731
    fe_start = [torch.cuda.Event(enable_timing=True) for _ in range(nblocks)]
    fe_end = [torch.cuda.Event(enable_timing=True) for _ in range(nblocks)]
    # SDR_BENCH_PLL_TIMING=0 (A/B): no timestamp packets on the PLL stream (pll object omitted)
    pll_timing = os.environ.get("SDR_BENCH_PLL_TIMING", "1") != "0"
    pll_start = [torch.cuda.Event(enable_timing=pll_timing) for _ in range(nblocks)]
    pre_done, post_done, gather_done = ([ev() for _ in range(nblocks)] for _ in range(3))
    pll_done = [torch.cuda.Event(enable_timing=pll_timing) for _ in range(nblocks)]
    gather = None
    if world > 1 and not args.no_gather:
        from real_time_sdr_amd.sharding import BlockGather
        gather = BlockGather(torch, dist, world, {"lr": ((nch, 2 * info.n_audio), torch.int16),
                                                  "bits": ((nch, pkg.SDR_MAX_BITS), torch.uint8)}, dev)

    def step(b: int) -> None:
        # the front end of block b reuses block b-2's parity: both consumers must have released it
        # (threadsafequeue.h:29-31), i.e. block b-2's post-PLL work is done
        if b >= 2:
            s_fe.wait_event(post_done[b - 2])
        fe_start[b].record(s_fe)
        pipe.frontend(iq[b], stream=s_fe)                # rffrontend.cpp:58-71
        fe_end[b].record(s_fe)
        pipe.mono(mono, stream=s_fe)                     # mono.cpp:34-42
        pipe.stereo_pre(stream=s_fe)                     # stereo.cpp:74, :80
        pipe.rds_pre(stream=s_fe)                        # rds.cpp:105-116
        pre_done[b].record(s_fe)
        s_pll.wait_event(pre_done[b])
        pll_start[b].record(s_pll)
        pipe.plls(stream=s_pll)                          # stereo.cpp:77 + rds.cpp:119
        pll_done[b].record(s_pll)
        s_post.wait_event(pll_done[b])
        if gather is not None and b >= 2:
            s_post.wait_event(gather_done[b - 2])        # lr/bits slot of block b-2 gathered
        pipe.stereo_post(lr[b % 2], stream=s_post)       # stereo.cpp:83-107
        pipe.rds_post(clean, bits=True, stream=s_post)   # rds.cpp:122-167
        with torch.cuda.stream(s_post):
            bits[b % 2].copy_(pipe.bits)
        post_done[b].record(s_post)
        if gather is not None:
            # final audio / bitstream gather over RCCL (xGMI)
            cur = torch.cuda.current_stream(dev)
            cur.wait_event(post_done[b])
            gather.gather(lr=lr[b % 2], bits=bits[b % 2])
            gather_done[b].record(cur)

    for b in range(args.warmup):
        step(b)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for b in range(args.warmup, nblocks):
        step(b)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    if world > 1:
        from real_time_sdr_amd.sharding import max_over_ranks
        elapsed = max_over_ranks(torch, dist, elapsed, dev)

    # front-end kernel (FIR /10 + discriminator) duration from HIP events on its own stream
    fe_ms = [fe_start[b].elapsed_time(fe_end[b]) for b in range(args.warmup, nblocks)]
    fe_avg_s = float(np.mean(fe_ms)) / 1e3
    fe_bytes = nch * (2 * info.block_iq + 4 * info.block_if)     # u8 I/Q in + f32 fm_demod out
    achieved = fe_bytes / fe_avg_s / 1e9
    # the serial PLL dispatch (both PLLs of a block) that bounds the block-step
    pll_ms = (float(np.mean([pll_start[b].elapsed_time(pll_done[b]) for b in range(args.warmup, nblocks)]))
              if pll_timing else float("nan"))
    total_samples = world * nch * info.block_iq * args.steps
    value = total_samples / elapsed / 1e6

    # informational, outside the timed region: the front-end kernel of both numerics modes alone
    # on the GPU (one stream, the same resident inputs), for comparison with the in-pipeline figure
    isolated = {}
    if rank == 0 and not args.no_isolated:
        for name, flags in (("exact", 0), ("fast", pkg.FLAG_FAST_FRONTEND)):
            p2 = pkg.Pipeline(nch, mode=0, rds_on=True, device=local, flags=flags)
            s2 = torch.cuda.Stream(dev)
            for b in range(min(nblocks, 3)):
                p2.frontend(iq[b], stream=s2)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            reps = 20
            e0.record(s2)
            for b in range(reps):
                p2.frontend(iq[b % nblocks], stream=s2)
            e1.record(s2)
            torch.cuda.synchronize(dev)
            ms = e0.elapsed_time(e1) / reps
            gbs = fe_bytes / (ms / 1e3) / 1e9
            isolated[name] = {"avg_launch_ms": round(ms, 4), "achieved_GBps": round(gbs, 1),
                              "frac": round(gbs / HBM_PEAK_GBS, 4)}
            p2.close()

    if rank == 0:
        # HBM bytes per launch of the same kernel from rocprofv3 PMC passes (FETCH_SIZE x2 gfx950
        # correction + WRITE_SIZE; tools/pmc_summary.py), committed under profiles/
        prof = ROOT / "profiles" / "pmc_frontend.json"
        traffic = None
        if prof.exists():
            try:
                pm = json.loads(prof.read_text())
                if pm.get("channels") == nch:
                    traffic = pm.get(args.numerics, {}).get("hbm_bytes_per_launch")
            except Exception:
                traffic = None
        res = {
            "metric": "IQ MSamples/s/node (mono+stereo+RDS), 1/2/4/8 GPU; HBM GB/s %peak",
            "value": round(value, 2),
            "unit": "MS/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic FM multiplex I/Q (mono+pilot+stereo+RDS 0A), u8, resident in HBM",
            "config": {
                "workload": "BASELINE configs[4] per GPU: full mono+stereo+RDS pipeline (project 0 r + mono), "
                            f"{nch} channels/GPU, mode 0 (2.4 MS/s, 73500 I/Q per block)",
                "channels_per_gpu": nch, "channels_total": world * nch, "block_iq": info.block_iq,
                "mode": 0,
                "pll_cus": (f"PLL stream on CU-mask {cu_spec}, other streams on the rest"
                            if cu_spec not in ("", "0") else "no CU masks"),
                "numerics": ("fast: int8 MFMA front end, fm_demod within 1e-5 of the reference, RDS bits bit-exact"
                             if fast else "exact (bit-exact with the reference)"),
                "parallelism": f"channel-sharded x{world}" + ("" if world == 1 or args.no_gather else " + RCCL all-gather"),
            },
            "roofline": {
                "kernel": ("k_frontend_mfma" if fast else "k_frontend2") +
                          " (u8 I/Q -> 101-tap FIR /10 on I,Q -> FM discriminator)",
                "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                "algorithmic_bytes_per_launch": fe_bytes, "avg_launch_ms": round(fe_avg_s * 1e3, 4),
            },
            "frontend_isolated": isolated or None,
            "pll": {
                "kernel": "k_pll: stereo 19 kHz + RDS 114 kHz PLLs (pll.cpp:4-61), 2 x channels serial "
                          "chains in one dispatch",
                "bound": "serial recurrence: block_if dependent steps per chain, one lane per chain "
                         "(per-wave VALU issue and latency, DESIGN.md 4a)",
                "avg_launch_ms": round(pll_ms, 4),
                "ns_per_step": round(pll_ms * 1e6 / info.block_if, 2),
                "share_of_step": round(pll_ms / (elapsed / args.steps * 1e3), 4),
            },
            "cpu_baseline": None if args.no_cpu_baseline else cpu_baseline(),
        }
        print(json.dumps(res))
    pipe.close()
    destroy_masked_streams(torch, pkg, dev)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
