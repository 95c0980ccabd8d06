#!/usr/bin/env python3
"""profiles/pll_counters.json from rocprofv3 --pmc counter_collection.csv files of the PLL kernel (the
SQ passes of tools/gpu/round.sh, per-block PLL dispatch): VALU instructions, issue and wave
quad-cycles per PLL step and wave. bench.py quotes them beside its live cycles-per-step.
  python tools/pll_counters.py <out.json> <block_if> <csv> [<csv> ...]"""
import collections
import csv
import json
import sys

out, block_if, files = sys.argv[1], int(sys.argv[2]), sys.argv[3:]
agg = collections.defaultdict(list)
for f in files:
    for r in csv.DictReader(open(f)):
        if "k_pll" in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
waves = sum(agg["SQ_WAVES"]) / len(agg["SQ_WAVES"])
per_step = {k: sum(v) / len(v) / waves / block_if for k, v in agg.items() if k != "SQ_WAVES"}
res = {"source": ", ".join(files), "kernel": "k_pll (per-block dispatch)", "waves": waves, "steps_per_wave": block_if,
       "valu_per_step": round(per_step.get("SQ_INSTS_VALU", 0.0), 2),
       "per_step": {k: round(v, 3) for k, v in sorted(per_step.items())},
       "note": "SQ_WAVE_CYCLES, SQ_ACTIVE_INST_* and SQ_WAIT_* count quad-cycles"}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res))
