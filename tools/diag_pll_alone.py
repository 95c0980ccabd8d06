#!/usr/bin/env python3
"""The PLL dispatch (stereo 19 kHz + RDS 114 kHz PLLs of 1024 channels, sdr_plls) alone on the chip
versus inside the bench pipeline: fills one block's PLL inputs through the real stages, then times
`plls()` back to back on one stream with nothing else running (the per-step cost without other
kernels' HBM traffic), on all CUs and on a 64-CU masked stream as in the bench.
  python tools/diag_pll_alone.py [--iters 10]
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
    ap.add_argument("--iters", type=int, default=10)
    args = ap.parse_args()
    import torch
    pkg = bench._load_pkg()
    dev = torch.device("cuda", 0)
    nch = args.channels
    iq = bench.make_input(torch, nch, 2, first_channel=0, device=dev)
    pipe = pkg.Pipeline(nch, mode=0, rds_on=True, device=0)
    n = pipe.info.block_if
    s = torch.cuda.Stream(dev)
    created: list[int] = []
    _, s_pll, _ = bench.cu_masked_streams(torch, pkg, dev, "64", created)
    res = {"channels": nch, "chains": 2 * nch, "steps": n}
    try:
        for b in range(2):
            pipe.frontend(iq[b], stream=s)
            pipe.stereo_pre(stream=s)
            pipe.rds_pre(stream=s)
            pipe.plls(stream=s)
        s.synchronize()
        for name, st in (("all_cus", s), ("cu_mask_64", s_pll)):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            pipe.plls(stream=st)
            e0.record(st)
            for _ in range(args.iters):
                pipe.plls(stream=st)
            e1.record(st)
            st.synchronize()
            ms = e0.elapsed_time(e1) / args.iters
            res[name] = {"ms_per_block": round(ms, 4), "ns_per_step": round(ms * 1e6 / n, 2)}
    finally:
        pipe.close()
        bench.destroy_masked_streams(torch, pkg, dev, created)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
