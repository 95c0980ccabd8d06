"""Diagnosis: persistent vs per-block PLL schedule at several widths (GPU outputs compared with each
other; tests/test_gpu_width.py compares both with the oracle)."""
import sys, pathlib, json
ROOT = pathlib.Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT)); sys.path.insert(0, str(ROOT / "tests"))
import numpy as np, torch
import bench
import test_gpu_width as W
pkg = bench._load_pkg()
import real_time_sdr_amd.synth as synth
dev = torch.device("cuda", 0)
out = {}
for nch in [int(a) for a in sys.argv[1:]] or [64, 128, 256, 1024]:
    W.NCH = nch
    kinds = W._kinds(synth) if nch >= 64 else None
    iq = bench.make_input(torch, nch, W.NBLOCKS, 0, dev, kinds=kinds, seed=5)
    a = W._run_schedule(torch, pkg, bench, iq, dev, "dispatch")
    b = W._run_schedule(torch, pkg, bench, iq, dev, "persistent")
    res = {}
    for k in ("fm", "mono", "lr", "clean", "bits"):
        diff = np.array([[not np.array_equal(a[k][bl, c], b[k][bl, c]) for c in range(nch)] for bl in range(W.NBLOCKS)])
        res[k] = {"n": int(diff.sum()), "blocks": diff.sum(1).tolist(),
                  "first_ch": [int(np.argmax(r)) if r.any() else -1 for r in diff]}
    out[nch] = res
    print(nch, json.dumps(res), flush=True)
