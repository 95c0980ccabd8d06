# One GPU session: GPU tests, bench line, rocprofv3 kernel-trace summary of the bench, and
# PMC passes (FETCH_SIZE, WRITE_SIZE in separate runs) over the isolated front end.
# Every GPU step has its own time limit; the first failure ends the script.
#   TAG=r01b [TESTS=1] [BENCH=1] [PROF=1] [PMC=1] bash tools/gpu/round.sh
set -o pipefail
export TMPDIR=/tmp
TAG=${TAG:-r01}
O=gpurun_out/$TAG
mkdir -p $O
step() { echo "[$(date +%T)] $*"; }
if [ "${TESTS:-1}" = 1 ]; then
  step tests
  timeout -k 10 420 python -m pytest tests -x -q -m gpu > $O/pytest_gpu.log 2>&1; rc=$?
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
      python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-isolated ${BENCH_ARGS:-} > $O/prof.log 2>&1; rc=$?
  [ $rc -eq 0 ] || { tail -20 $O/prof.log; exit $rc; }
  find $O/prof -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
  head -12 $O/kernel_stats.csv | cut -c1-160
fi
if [ "${PMC:-1}" = 1 ]; then
  for c in FETCH_SIZE WRITE_SIZE; do
    step pmc $c
    timeout -k 10 300 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $O/pmc_$c -o fe -- \
        python3 tools/bench_frontend.py --iters 10 > $O/pmc_$c.log 2>&1; rc=$?
    [ $rc -eq 0 ] || { tail -20 $O/pmc_$c.log; exit $rc; }
    find $O/pmc_$c -name "*counter_collection.csv" -exec cp {} $O/pmc_$c.csv \;
  done
  timeout -k 10 60 python tools/pmc_summary.py $O 1024 > $O/pmc_summary.json; cat $O/pmc_summary.json
fi
step done
