# bench + rocprofv3 kernel-trace summary (run through gpurun from the repo root)
set -o pipefail
export TMPDIR=/tmp
TAG=${TAG:-r01}
STEPS=${STEPS:-20}
timeout -k 10 400 python bench.py --steps $STEPS --warmup 3 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_$TAG.json; tail -5 gpurun_out/bench_$TAG.err
[ $rc -eq 0 ] || exit $rc
if [ -n "$PROF" ]; then
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/prof_$TAG.log 2>&1
  rc=$?; echo "rocprof rc=$rc"; tail -3 gpurun_out/prof_$TAG.log
  find gpurun_out/prof_$TAG -name "*stats*.csv" | head
fi
exit $rc
