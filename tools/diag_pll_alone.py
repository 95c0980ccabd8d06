#!/usr/bin/env python3
"""The PLL dispatch (stereo 19 kHz + RDS 114 kHz PLLs of 1024 channels, sdr_plls) alone on the chip
versus inside the bench pipeline: runs the stages of each block on ONE stream and times
the `plls()` dispatch between them, so nothing else runs beside it (the per-step cost without other
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
    _, s_pll, _, _ = bench.cu_masked_streams(torch, pkg, dev, "64", created)
    res = {"channels": nch, "chains": 2 * nch, "steps": n}
    lr = torch.empty(nch, 2 * pipe.info.n_audio, dtype=torch.int16, device=dev)
    clean = torch.empty(nch, pipe.info.n_rds, dtype=torch.float32, device=dev)
    try:
        for name, st in (("all_cus", s), ("cu_mask_64", s_pll)):
            ev = []
            for b in range(args.iters + 2):
                # the stages before the PLLs on the same stream: nothing overlaps the PLL dispatch
                pipe.frontend(iq[b % 2], stream=st)
                pipe.stereo_pre(stream=st)
                pipe.rds_pre(stream=st)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                pipe.plls(stream=st)
                e1.record(st)
                pipe.stereo_post(lr, stream=st)
                pipe.rds_post(clean, bits=True, stream=st)
                ev.append((e0, e1))
            st.synchronize()
            ms = sum(a.elapsed_time(b) for a, b in ev[2:]) / args.iters
            res[name] = {"ms_per_block": round(ms, 4), "ns_per_step": round(ms * 1e6 / n, 2)}
    finally:
        pipe.close()
        bench.destroy_masked_streams(torch, pkg, dev, created)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
