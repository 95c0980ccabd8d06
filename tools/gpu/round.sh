# One GPU session: GPU tests, bench line, rocprofv3 kernel-trace summary of the bench, PMC passes
# (FETCH_SIZE, WRITE_SIZE in separate runs) over the isolated front end, and SQ counter passes over
# the PLL kernel inside the bench. Every GPU step has its own time limit; the first failure ends it.
#   TAG=r02_v2 [TESTS=1] [BENCH=1] [PROF=1] [PMC=1] [PLLPMC=1] bash tools/gpu/round.sh
set -o pipefail
export TMPDIR=/tmp
TAG=${TAG:-r02}
O=gpurun_out/$TAG
mkdir -p $O
step() { echo "[$(date +%T)] $*"; }
if [ "${SMOKE:-1}" = 1 ]; then
  step smoke
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1; rc=$?
  tail -2 $O/smoke.log; [ $rc -eq 0 ] || { tail -30 $O/smoke.log; exit $rc; }
fi
if [ "${TESTS:-1}" = 1 ]; then
  step tests
  timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
  tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || { tail -40 $O/pytest_gpu.log; exit $rc; }
fi
if [ "${BENCH:-1}" = 1 ]; then
  step bench
  timeout -k 10 400 python bench.py ${BENCH_ARGS:-} > $O/bench.json 2> $O/bench.err; rc=$?
  cat $O/bench.json; [ $rc -eq 0 ] || { tail -20 $O/bench.err; exit $rc; }
fi
if [ "${PROF:-1}" = 1 ]; then
  step rocprof kernel-trace
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- \
      python3 bench.py --steps 20 --warmup ${PROF_WARMUP:-5} --no-cpu-baseline --no-isolated > $O/prof.log 2>&1; rc=$?
  [ $rc -eq 0 ] || { tail -20 $O/prof.log; exit $rc; }
  find $O/prof -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
  find $O/prof -name "*kernel_trace.csv" -exec cp {} $O/kernel_trace.csv \;
  grep '^{' $O/prof.log | tail -1 > $O/bench_profiled.json
  python tools/timeline.py $O/kernel_trace.csv --by-grid k_frontend2 > $O/frontend_by_grid.txt && cat $O/frontend_by_grid.txt
  rm -rf $O/prof   # raw traces: gpurun_out/ is only copied back below 64 MiB
  head -14 $O/kernel_stats.csv | cut -c1-160
fi
if [ "${PMC:-1}" = 1 ]; then
  for c in FETCH_SIZE WRITE_SIZE; do
    step pmc $c
    timeout -k 10 300 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $O/pmc_$c -o fe -- \
        python3 tools/bench_frontend.py --iters 10 > $O/pmc_$c.log 2>&1; rc=$?
    [ $rc -eq 0 ] || { tail -20 $O/pmc_$c.log; exit $rc; }
    find $O/pmc_$c -name "*counter_collection.csv" -exec cp {} $O/pmc_$c.csv \;
    rm -rf $O/pmc_$c
  done
  timeout -k 10 60 python tools/pmc_summary.py $O 1024 > $O/pmc_summary.json; cat $O/pmc_summary.json
fi
if [ "${PLLPMC:-1}" = 1 ]; then
  i=0
  for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
             "SQ_WAVES SQ_WAIT_ANY SQ_INSTS_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_SALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64"; do
    i=$((i+1))
    step pll pmc $i
    # per-block dispatch: PMC collection serialises dispatches, which the persistent PLL (waiting
    # on flags set by later dispatches) cannot survive
    SDR_BENCH_PLL=dispatch timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $O/pllpmc$i -o b -- \
        python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-isolated > $O/pllpmc$i.log 2>&1 || { tail -20 $O/pllpmc$i.log; exit 1; }
    f=$(find $O/pllpmc$i -name "*counter_collection.csv" | head -1)
    cp "$f" $O/pllpmc$i.csv
    rm -rf $O/pllpmc$i
    python tools/sq_summary.py $O/pllpmc$i.csv k_pll
  done
fi
step done
