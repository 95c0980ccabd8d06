# bench.py in both numerics modes (+ rocprofv3 kernel-trace stats of the fast run when PROF=1)
set -o pipefail
export TMPDIR=/tmp
TAG=${TAG:-b2}
O=gpurun_out/$TAG
mkdir -p $O
for m in ${MODES:-fast exact}; do
  timeout -k 10 300 python bench.py --steps ${STEPS:-20} --warmup 3 --numerics $m ${BARGS:-} > $O/bench_$m.json 2> $O/bench_$m.err
  rc=$?; echo "bench $m rc=$rc"; cat $O/bench_$m.json; [ $rc -eq 0 ] || { tail -20 $O/bench_$m.err; exit $rc; }
done
if [ -n "$PROF" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-isolated --numerics ${PROFMODE:-fast} > $O/prof.log 2>&1
  rc=$?; echo "rocprof rc=$rc"; tail -3 $O/prof.log; [ $rc -eq 0 ] || exit $rc
  find $O/prof -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
  head -20 $O/kernel_stats.csv
fi
