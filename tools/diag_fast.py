#!/usr/bin/env python3
"""Diagnostic: fast (MFMA) vs exact front end, per-block error location (indices of the largest
relative differences of fm_demod)."""
import pathlib, sys
import numpy as np
ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT)); sys.path.insert(0, str(ROOT / "tests"))
import bench
import torch
pkg = bench._load_pkg()
import real_time_sdr_amd.synth as s
mode = int(sys.argv[1]) if len(sys.argv) > 1 else 0
align = int(sys.argv[2]) if len(sys.argv) > 2 else 1
nb, nch = 4, 2
pa = pkg.Pipeline(nch, mode=mode)
pb = pkg.Pipeline(nch, mode=mode, flags=pkg.FLAG_FAST_FRONTEND)
info = pa.info
iqs = []
for c in range(nch):
    src = s.FMMultiplexSource(40 + c)
    iqs.append(np.stack([src.next_block(info.block_iq) for _ in range(nb)]))
host = np.stack(iqs, axis=1)
row = host.shape[2]
d = torch.empty(nb, nch, (row + align - 1) // align * align, dtype=torch.uint8, device="cuda")[:, :, :row]
d.copy_(torch.from_numpy(host))
for b in range(nb):
    pa.frontend(d[b]); pb.frontend(d[b])
    x = pa.fm_demod().cpu().numpy().astype(np.float64)
    y = pb.fm_demod().cpu().numpy().astype(np.float64)
    for c in range(nch):
        e = np.abs(x[c] - y[c]) / np.max(np.abs(x[c]))
        idx = np.argsort(e)[-5:][::-1]
        print(f"block {b} ch {c}: max {e.max():.2e} at {list(idx)} vals {[(round(x[c][i],5), round(y[c][i],5)) for i in idx[:3]]}")
