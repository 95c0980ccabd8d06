# Per-kernel counters of every stage of the exact pipeline, isolated on one stream (tools/bench_stages.py,
# per-block PLL dispatch): a kernel trace, two SQ passes and FETCH_SIZE / WRITE_SIZE in passes of their
# own, each under its own time limit; the first failure ends the script.
#   TAG=r03_stages bash tools/gpu/stage_pmc.sh   -> gpurun_out/$TAG/*.csv, stage_counters.json
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-stages}
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o st -- \
    python3 tools/bench_stages.py --iters 10 > $O/kt.log 2>&1 || { tail -20 $O/kt.log; exit 1; }
find $O/kt -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
rm -rf $O/kt
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY" \
           "SQ_WAVES SQ_INSTS_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_SALU SQ_INSTS_VALU_FMA_F64" \
           FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  echo "[pass $i] $grp"
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $O/pmc$i -o st -- \
      python3 tools/bench_stages.py --iters 3 > $O/pmc$i.log 2>&1 || { tail -20 $O/pmc$i.log; exit 1; }
  f=$(find $O/pmc$i -name "*counter_collection.csv" | head -1)
  cp "$f" $O/pmc$i.csv
  rm -rf $O/pmc$i
done
python3 tools/stage_counters.py $O > $O/stage_counters.json && cat $O/stage_counters.json
