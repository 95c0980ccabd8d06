# SQ counters of the isolated PLL kernel (tools/bench_pll.py: 2048 chains x 7350 steps), one pass
# per counter group, each pass under its own time limit; first failure ends the script.
#   TAG=r02_pll bash tools/gpu/pll_pmc.sh
set -o pipefail
export TMPDIR=/tmp
TAG=${TAG:-pll}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 120 python tools/bench_pll.py --iters 5 > $O/bench_pll.json 2> $O/bench_pll.err || { tail $O/bench_pll.err; exit 1; }
cat $O/bench_pll.json
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_WAVES SQ_WAIT_ANY SQ_INSTS_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_SALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64" \
           ${EXTRA_GROUPS:-}; do
  i=$((i+1))
  echo "[pass $i] $grp"
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $O/pmc$i -o pll -- \
      python3 tools/bench_pll.py --iters 2 > $O/pmc$i.log 2>&1 || { tail -20 $O/pmc$i.log; exit 1; }
  f=$(find $O/pmc$i -name "*counter_collection.csv" | head -1)
  cp "$f" $O/pmc$i.csv
  python tools/sq_summary.py $O/pmc$i.csv k_pll
done
