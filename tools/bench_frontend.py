#!/usr/bin/env python3
"""Isolated timing of the fused front end (u8 I/Q -> FIR /10 -> discriminator) on one stream.

Runs `sdr_frontend` back to back over distinct resident input blocks for each numerics mode and
prints per-launch time and algorithmic GB/s (2 B in + 4 B/10 out per I/Q pair) vs the 8 TB/s peak.
  python tools/bench_frontend.py [--channels 1024] [--iters 50]
"""
from __future__ import annotations

import argparse
import json
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--channels", type=int, default=1024)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--blocks", type=int, default=8)
    args = ap.parse_args()
    import torch
    pkg = bench._load_pkg()
    dev = torch.device("cuda", 0)
    iq = bench.make_input(torch, args.channels, args.blocks, 0, dev)
    res = {}
    for name, flags in (("exact", 0), ("fast", pkg.FLAG_FAST_FRONTEND)):
        pipe = pkg.Pipeline(args.channels, flags=flags)
        info = pipe.info
        s = torch.cuda.Stream(dev)
        for b in range(4):
            pipe.frontend(iq[b % args.blocks], stream=s)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for b in range(args.iters):
            pipe.frontend(iq[b % args.blocks], stream=s)
        e1.record(s)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / args.iters
        nbytes = args.channels * (2 * info.block_iq + 4 * info.block_if)
        res[name] = {"ms": round(ms, 4), "GBps": round(nbytes / ms / 1e6, 1),
                     "frac_of_8TBps": round(nbytes / ms / 1e6 / 8000.0, 4),
                     "MSps": round(args.channels * info.block_iq / ms / 1e3, 1)}
        pipe.close()
    print(json.dumps({"channels": args.channels, "frontend": res}))


if __name__ == "__main__":
    main()
