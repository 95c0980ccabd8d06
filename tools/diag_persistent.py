#!/usr/bin/env python3
"""Diagnostic: the persistent PLL schedule (sdr_plls_launch/_signal/_wait) against the one-stream
sequential pipeline, block by block (carrier / ipll PLL outputs and stereo audio), for launch
splits given on the command line, e.g. `python tools/diag_persistent.py 5,9 14,0 7,7`."""
import pathlib
import sys

import time

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT)); sys.path.insert(0, str(ROOT / "tests"))
import bench  # noqa: E402
import torch  # noqa: E402
from conftest import channel_input  # noqa: E402

pkg = bench._load_pkg()
import real_time_sdr_amd.synth as synth  # noqa: E402

nch = 40
splits = [[int(v) for v in a.split(",") if int(v) > 0] for a in sys.argv[1:]] or [[5, 9]]
nb = sum(splits[0])
iqs = [channel_input(synth, 300 + c, nb) for c in range(nch)]
d = torch.from_numpy(np.stack(iqs, axis=1)).cuda()
ref = bench._load_pkg().Pipeline(nch)
want = []
for b in range(nb):
    ref.frontend(d[b]); lr = ref.stereo(); ref.rds()
    want.append((ref.buffer("carrier").cpu().numpy(), ref.buffer("ipll").cpu().numpy(), lr.cpu().numpy()))
for split in splits:
    pipe = pkg.Pipeline(nch)
    created = []   # non-blocking torch streams: the legacy null stream never waits on the PLL stream
    s_fe, s_pll, s_post = (torch.cuda.Stream() for _ in range(3))
    lr = torch.empty(nch, 2 * pipe.info.n_audio, dtype=torch.int16, device="cuda")
    starts = np.cumsum([0] + split[:-1])
    res = []
    T0 = time.time()
    for b in range(nb):
        if b in starts:
            pipe.plls_launch(split[list(starts).index(b)], stream=s_pll)
        pipe.frontend(d[b], stream=s_fe)
        pipe.stereo_pre(stream=s_fe); pipe.rds_pre(stream=s_fe)
        pipe.plls_signal(stream=s_fe)
        pipe.plls_wait(stream=s_post)
        pipe.stereo_post(lr, stream=s_post)
        pipe.rds_post(None, bits=False, stream=s_post)
        s_post.synchronize()
        with torch.cuda.stream(s_post):
            lrh = lr.cpu().numpy()
        car = pipe.buffer("carrier", stream=s_post).cpu().numpy()
        ip = pipe.buffer("ipll", stream=s_post).cpu().numpy()
        ok = [np.array_equal(car.view(np.uint32), want[b][0].view(np.uint32)),
              np.array_equal(ip.view(np.uint32), want[b][1].view(np.uint32)),
              np.array_equal(lrh, want[b][2])]
        first = int(np.argmax(car.view(np.uint32)[0] != want[b][0].view(np.uint32)[0])) if not ok[0] else -1
        res.append(("ok" if all(ok) else f"BAD{ok} first-carrier-diff@{first}"))
        print(f"  block {b}: {res[-1]} at {time.time() - T0:.2f} s", flush=True)
    print(split, res, flush=True)
    try:
        print("  report", pipe.plls_report(stream=s_pll)[:3], flush=True)
    except Exception as e:  # noqa: BLE001
        print("  report:", e, flush=True)
    bench.destroy_masked_streams(torch, pkg, torch.device("cuda", 0), created)
    pipe.close()
