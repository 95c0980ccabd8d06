# SQ counter passes (one rocprofv3 --pmc run per group, each under its own time limit) over a
# command; prints the per-kernel averages of kernels matching FILTER.
#   TAG=x FILTER=k_pll CMD="python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-isolated" \
#   PASSES="SQ_WAVES SQ_WAVE_CYCLES ...;SQ_WAVES SQ_WAIT_ANY ..." bash tools/gpu/sq_passes.sh
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-sq}
mkdir -p $O
i=0
IFS=";" read -ra G <<< "$PASSES"
for grp in "${G[@]}"; do
  i=$((i+1))
  echo "[pass $i] $grp"
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $O/p$i -o r -- $CMD > $O/p$i.log 2>&1 || { tail -20 $O/p$i.log; exit 1; }
  f=$(find $O/p$i -name "*counter_collection.csv" | head -1)
  cp "$f" $O/p$i.csv
  python tools/sq_summary.py $O/p$i.csv "$FILTER"
done
