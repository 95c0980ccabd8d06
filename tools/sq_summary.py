#!/usr/bin/env python3
"""Average rocprofv3 --pmc counter values per kernel (and per wave) from a counter_collection.csv.
  python tools/sq_summary.py gpurun_out/<tag>/sq1.csv [kernel-substring]"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
pat = sys.argv[2] if len(sys.argv) > 2 else ""
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in rows:
    if pat in r["Kernel_Name"]:
        agg[r["Kernel_Name"][:70]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    waves = sum(d["SQ_WAVES"]) / len(d["SQ_WAVES"]) if "SQ_WAVES" in d else None
    print(k)
    for c, v in sorted(d.items()):
        avg = sum(v) / len(v)
        per = f"  per wave {avg / waves:10.1f}" if waves else ""
        print(f"   {c:24s} n={len(v):3d} avg={avg:14.1f}{per}")
