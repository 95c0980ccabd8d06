#!/usr/bin/env python3
"""Diagnostic for the sdr_fmpll scratch variants: the reference harness on the CPU
(oracle/_ref/ref_harness) against the same harness over the drop-in layer (oracle/_ref/harness_gpu,
every primitive through libsdr_amd.so, fmpll via sdr_fmpll) with SDR_FMPLL_SCRATCH = stream (per-stream
cached scratch, the default), sync (hipMalloc + synchronise + hipFree) and async (two hipMallocAsync /
hipFreeAsync pairs), each run `reps` times; prints per run which outputs differ from the CPU.
  python tools/diag_fmpll_scratch.py [nblocks] [reps]"""
import json
import os
import pathlib
import subprocess
import sys
import tempfile

import numpy as np

ROOT = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "real-time-sdr_amd"))
import synth  # noqa: E402

nb = int(sys.argv[1]) if len(sys.argv) > 1 else 10
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
src = synth.FMMultiplexSource(0)
iq = np.stack([src.next_block() for _ in range(nb)])
OUTS = ("fm_demod.f32", "mono.i16", "stereo.i16", "rds_clean.f32", "bits.txt")
res = {}
with tempfile.TemporaryDirectory() as d:
    inp = pathlib.Path(d) / "in.u8"
    iq.tofile(inp)
    subprocess.run([str(ROOT / "oracle/_ref/ref_harness"), str(inp), str(nb), "0", "1", f"{d}/cpu_"], check=True,
                   timeout=300)
    ref = {o: pathlib.Path(f"{d}/cpu_{o}").read_bytes() for o in OUTS}
    for mode in (sys.argv[3].split(",") if len(sys.argv) > 3 else ("stream", "sync", "async")):
        runs = []
        for r in range(reps):
            env = dict(os.environ, SDR_FMPLL_SCRATCH=mode)
            subprocess.run([str(ROOT / "oracle/_ref/harness_gpu"), str(inp), str(nb), "0", "1", f"{d}/g_"], check=True,
                           timeout=300, env=env)
            runs.append([o for o in OUTS if pathlib.Path(f"{d}/g_{o}").read_bytes() != ref[o]])
        res[mode] = runs
        print(mode, runs, flush=True)
print(json.dumps({"nblocks": nb, "reps": reps, "differing_outputs_per_run": res}))
