# Round 5 session D: the instruction-fetch microbenchmark, then the isolated stages under a kernel
# trace (per-kernel isolated durations).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05_d}
mkdir -p $O
timeout -k 10 120 tools/microbench/bin/ifetch > $O/ifetch.jsonl 2> $O/ifetch.err || { tail $O/ifetch.err; exit 1; }
cat $O/ifetch.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/st -o st -- python3 tools/bench_stages.py --iters 20 > $O/stages.json 2> $O/stages.err || { tail -5 $O/stages.err; exit 1; }
f=$(find $O/st -name "*kernel_stats.csv" | head -1)
cp "$f" $O/stage_kernel_stats.csv
python3 - <<PY
import csv
for r in csv.DictReader(open("$O/stage_kernel_stats.csv")):
    if "at::" in r["Name"]: continue
    print(r["Name"][:70], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1))
PY
