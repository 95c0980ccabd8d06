#!/usr/bin/env python3
"""Isolated timing of the batched PLL (pll.cpp:4-61) on pilot-like input: nch independent
recurrences of n steps each (default 2048 = the stereo + RDS PLLs of 1024 channels).
  python tools/bench_pll.py [--channels 2048] [--iters 5]
"""
from __future__ import annotations

import argparse
import json
import math
import pathlib
import sys

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--channels", type=int, default=2048)
    ap.add_argument("--n", type=int, default=7350)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--cus", type=int, default=0,
                    help="run on a stream CU-masked to CUs [0, cus) (waves per CU = waves / cus)")
    args = ap.parse_args()
    import torch
    pkg = bench._load_pkg()
    dev = torch.device("cuda", 0)
    nch, n = args.channels, args.n
    i = torch.arange(n, dtype=torch.float64, device=dev)
    ph0 = torch.rand(nch, 1, dtype=torch.float64, device=dev) * 2 * math.pi
    x = (0.1 * torch.cos(2 * math.pi * 19e3 / 240e3 * i + ph0)).float()
    x = x + 0.01 * torch.randn(nch, n, device=dev)
    out = torch.empty(nch, n + 1, dtype=torch.float32, device=dev)
    st = pkg.pll_state_tensor(nch, device=dev)
    created = []
    if args.cus > 0:
        s = bench.cu_masked_streams(torch, pkg, dev, str(args.cus), created, all_cus=False)[1]
    else:
        s = torch.cuda.Stream(dev)
    for _ in range(2):
        pkg.fmpll(out, x, 19e3, 240e3, st, 2.0, 0.0, 0.01, stream=s)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(args.iters):
        pkg.fmpll(out, x, 19e3, 240e3, st, 2.0, 0.0, 0.01, stream=s)
    e1.record(s)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / args.iters
    print(json.dumps({"channels": nch, "steps": n, "cus": args.cus or None, "ms_per_call": round(ms, 4),
                      "ns_per_step": round(ms * 1e6 / n, 2)}))
    bench.destroy_masked_streams(torch, pkg, dev, created)


if __name__ == "__main__":
    main()
