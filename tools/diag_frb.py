#!/usr/bin/env python3
"""Diagnosis: the 3-filter pass (sdr_pre, k_fir_rb<3> with packed pilot+band pairs) against the
separate stereo_pre + rds_pre FIRs on the same fm_demod: pilot, band and rds_band of every channel.
    python tools/diag_frb.py [NCH]"""
from __future__ import annotations

import pathlib
import sys

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402


def main() -> None:
    nch = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    import torch
    pkg = bench._load_pkg()
    dev = torch.device("cuda", 0)
    iq = bench.make_input(torch, nch, 3, 0, dev)
    outs = []
    for split in (False, True):
        pipe = pkg.Pipeline(nch, mode=0, rds_on=True, device=0)
        got = []
        for b in range(3):
            pipe.frontend(iq[b])
            if split:
                pipe.stereo_pre()
                pipe.rds_pre()
            else:
                pipe.pre()
            torch.cuda.synchronize()
            got.append({k: pipe.buffer(k).cpu().numpy() for k in ("pilot", "band", "rds_band")})
            pipe.plls()
            pipe.stereo_post(torch.empty(nch, 2 * pipe.info.n_audio, dtype=torch.int16, device=dev))
            pipe.rds_post(torch.empty(nch, pipe.info.n_rds, dtype=torch.float32, device=dev), bits=True)
            torch.cuda.synchronize()
        outs.append(got)
        pipe.close()
    for b in range(3):
        for k in ("pilot", "band", "rds_band"):
            a, r = outs[0][b][k].view(np.uint32), outs[1][b][k].view(np.uint32)
            bad = np.argwhere(a != r)
            print(f"block {b} {k}: {len(bad)} mismatches" + (f", first {bad[:5].tolist()} "
                  f"pre {outs[0][b][k][tuple(bad[0])]} split {outs[1][b][k][tuple(bad[0])]}" if len(bad) else ""))


if __name__ == "__main__":
    main()
