# SQ / SQC counters of the instruction-fetch microbenchmark (tools/microbench/ifetch.hip), to set
# beside the PLL's (profiles/r05/pll_waves_notab.txt)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05_ipmc}
mkdir -p $O
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_IFETCH SQC_ICACHE_BUSY_CYCLES SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_TC_INST_REQ --output-format csv -d $O/p1 -o r -- tools/microbench/bin/ifetch > $O/p1.log 2>&1 || { tail -20 $O/p1.log; exit 1; }
f=$(find $O/p1 -name "*counter_collection.csv" | head -1)
cp "$f" $O/p1.csv
python3 - <<PY
import csv, collections
rows = list(csv.DictReader(open("$O/p1.csv")))
agg = collections.defaultdict(lambda: collections.defaultdict(float))
order = []
for r in rows:
    key = (r["Dispatch_Id"], r["Kernel_Name"][:40], r["Workgroup_Size_X"] if "Workgroup_Size_X" in r else r.get("Workgroup_Size", ""))
    if key not in agg: order.append(key)
    agg[key][r["Counter_Name"]] += float(r["Counter_Value"])
for k in order:
    d = agg[k]
    w = d.get("SQ_WAVES", 1) or 1
    print(k[0], k[1], k[2], {c: round(v / w, 1) if c.startswith("SQ_") and c != "SQ_WAVES" else round(v, 1) for c, v in sorted(d.items())})
PY
