# k_frontend3 session: front-end parity tests, isolated exact front end (v3 vs v2), then the
# whole GPU suite, the driver's bench line and a kernel trace. First failure ends it.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-fe3}
mkdir -p $O
step() { echo "[$(date +%T)] $*"; }
step fe tests
timeout -k 10 300 python -u -m pytest tests/test_gpu_pipeline.py -x -q -k "golden or many_channels or knobs or other_modes" \
    --timeout 120 --timeout-method thread > $O/fe_tests.log 2>&1 || { tail -30 $O/fe_tests.log; exit 1; }
tail -2 $O/fe_tests.log
step isolated
for v in 1 0 1 0; do
  SDR_FE_V3=$v timeout -k 10 120 python tools/bench_frontend.py --iters 50 > $O/iso_v$v.json 2>&1 || { cat $O/iso_v$v.json; exit 1; }
  echo "v3=$v $(cat $O/iso_v$v.json)"
done
if [ "${FULL:-1}" = 1 ]; then
  step full tests
  timeout -k 10 700 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
  tail -2 $O/pytest_gpu.log
  step bench
  timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
  cat $O/bench.json
  step rocprof
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- \
      python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-isolated > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
  find $O/prof -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
  rm -rf $O/prof
  head -16 $O/kernel_stats.csv | cut -c1-150
fi
step done
