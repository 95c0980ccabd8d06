#!/usr/bin/env python3
"""Per-kernel summary of tools/gpu/stage_pmc.sh: isolated average duration (kernel trace), SQ counters
per wave (VALU instructions, issue and wave quad-cycles, waits) and HBM bytes per launch (FETCH_SIZE,
KiB per dispatch, x2 for gfx950's wide streaming reads per MI355X_MICROARCH.md; WRITE_SIZE as is),
with the kernel's achieved HBM rate and VALU issue fraction.
  python tools/stage_counters.py gpurun_out/<tag>"""
from __future__ import annotations

import collections
import csv
import json
import pathlib
import sys

HBM_GBS = 8000.0


def short(name: str) -> str:
    n = name.replace("void ", "", 1).strip()
    for pre in ("sdrk::(anonymous namespace)::", "(anonymous namespace)::"):
        if n.startswith(pre):
            n = n[len(pre):]
    return n.split("(", 1)[0].strip()


def main() -> None:
    d = pathlib.Path(sys.argv[1])
    dur = {}
    with open(d / "kernel_stats.csv") as f:
        for r in csv.DictReader(f):
            if "::k_" in r["Name"]:
                dur[short(r["Name"])] = {"calls": int(r["Calls"]), "avg_us": float(r["AverageNs"]) / 1e3}
    ctr = collections.defaultdict(lambda: collections.defaultdict(list))
    for p in sorted(d.glob("pmc*.csv")):
        with open(p) as f:
            for r in csv.DictReader(f):
                k = short(r["Kernel_Name"])
                if k in dur:
                    ctr[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {"source": f"tools/gpu/stage_pmc.sh (tools/bench_stages.py, 1024 channels, isolated, per-block PLL dispatch)",
           "note": "per_wave: SQ_* per wave (SQ_WAVE_CYCLES, SQ_ACTIVE_*, SQ_WAIT_* in quad-cycles); "
                   "fetch_bytes = FETCH_SIZE KiB x 1024 x 2 (gfx950 correction for wide reads; narrower "
                   "reads may be over-counted by it), write_bytes = WRITE_SIZE KiB x 1024",
           "kernels": {}}
    for k, t in sorted(dur.items(), key=lambda kv: -kv[1]["avg_us"] * kv[1]["calls"]):
        c = {n: sum(v) / len(v) for n, v in ctr.get(k, {}).items()}
        waves = c.get("SQ_WAVES")
        e = {"avg_us": round(t["avg_us"], 2), "calls": t["calls"]}
        if waves:
            e["waves"] = int(waves)
            e["per_wave"] = {n[3:]: round(v / waves, 1) for n, v in sorted(c.items())
                             if n.startswith("SQ_") and n != "SQ_WAVES"}
            if c.get("SQ_WAVE_CYCLES"):
                e["valu_issue_frac"] = round(c.get("SQ_ACTIVE_INST_VALU", 0) / c["SQ_WAVE_CYCLES"], 3)
        if "FETCH_SIZE" in c:
            e["fetch_bytes"] = int(c["FETCH_SIZE"] * 1024 * 2)
        if "WRITE_SIZE" in c:
            e["write_bytes"] = int(c["WRITE_SIZE"] * 1024)
        if "fetch_bytes" in e and "write_bytes" in e:
            e["hbm_GBps"] = round((e["fetch_bytes"] + e["write_bytes"]) / (t["avg_us"] * 1e3), 1)
            e["hbm_frac"] = round(e["hbm_GBps"] / HBM_GBS, 3)
        out["kernels"][k] = e
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
