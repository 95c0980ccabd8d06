#!/usr/bin/env python3
"""Isolated timing of every stage of the exact pipeline on ONE stream (each kernel alone on the
chip), with each stage's VALU or HBM floor beside it.

One iteration = one block of every channel: frontend, mono, pre (stereo_pre + rds_pre), plls (per-block
dispatch), stereo_post, rds_post + rds_bits. HIP events bracket each stage over `iters` blocks of
distinct resident input; under `rocprofv3 --kernel-trace --stats` the same run gives per-kernel
isolated durations, and under `--pmc` the per-kernel counters (tools/gpu/stage_pmc.sh).
  python tools/bench_stages.py [--channels 1024] [--iters 20]
"""
from __future__ import annotations

import argparse
import json
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402

# MI355X: 256 CUs x 4 SIMDs x 32 f32 lanes x 2.4 GHz non-packed f32 lane-ops/s (FP32 vector peak
# 157.3 TFLOP/s counts an FMA as 2); mul and add are separate instructions in exact mode
VALU_LANE_OPS = 256 * 4 * 32 * 2.4e9


def floors(info, nch: int) -> dict:
    """Minimum VALU lane-ops (f32 mul + add per tap) of each stage's FIRs, as microseconds at the
    full-chip f32 VALU rate. The PLL stage is a serial recurrence: no VALU floor."""
    n, T = info.block_if, info.rf_taps
    mac = 2 * T
    ops = {
        "frontend": nch * info.block_if * 2 * mac,                        # I and Q, decimated outputs
        "mono": nch * info.n_audio * mac,
        "pre": nch * n * 4 * mac,                                          # pilot, band, RDS, squared-RDS BPFs
        "stereo_post": nch * info.n_audio * 2 * mac,                       # two resamplers (+ NCO, mixer)
        "rds_post": nch * info.n_rds * 2 * mac,                            # 247/640 resampler + RRC (+ NCO, mixer)
    }
    return {k: round(v / VALU_LANE_OPS * 1e6, 2) for k, v in ops.items()}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--channels", type=int, default=1024)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--blocks", type=int, default=8)
    args = ap.parse_args()
    import torch
    pkg = bench._load_pkg()
    dev = torch.device("cuda", 0)
    nch = args.channels
    iq = bench.make_input(torch, nch, args.blocks, 0, dev)
    pipe = pkg.Pipeline(nch)
    info = pipe.info
    s = torch.cuda.Stream(dev)
    mono = torch.empty(nch, info.n_audio, dtype=torch.int16, device=dev)
    lr = torch.empty(nch, 2 * info.n_audio, dtype=torch.int16, device=dev)
    clean = torch.empty(nch, info.n_rds, dtype=torch.float32, device=dev)
    stages = ("frontend", "mono", "pre", "plls", "stereo_post", "rds_post")
    ev = {k: [] for k in stages}

    def one(b: int, timed: bool) -> None:
        calls = (("frontend", lambda: pipe.frontend(iq[b % args.blocks], stream=s)),
                 ("mono", lambda: pipe.mono(mono, stream=s)),
                 ("pre", lambda: pipe.pre(stream=s)),
                 ("plls", lambda: pipe.plls(stream=s)),
                 ("stereo_post", lambda: pipe.stereo_post(lr, stream=s)),
                 ("rds_post", lambda: pipe.rds_post(clean, bits=True, stream=s)))
        for name, fn in calls:
            if timed:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                fn()
                e1.record(s)
                ev[name].append((e0, e1))
            else:
                fn()

    for b in range(3):
        one(b, False)
    for b in range(3, 3 + args.iters):
        one(b, True)
    torch.cuda.synchronize(dev)
    ms = {k: round(sum(a.elapsed_time(z) for a, z in v) / len(v), 4) for k, v in ev.items()}
    fl = floors(info, nch)
    out = {"channels": nch, "iters": args.iters, "stage_ms": ms,
           "valu_floor_us": fl,
           "frac_of_valu_floor": {k: round(fl[k] / (ms[k] * 1e3), 3) for k in fl},
           "non_pll_ms": round(sum(v for k, v in ms.items() if k != "plls"), 4)}
    pipe.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
