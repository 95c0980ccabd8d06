# Round-4 session: GPU tests, the driver-shaped bench (20 steps), then the same with the fill parts
# off (SDR_BENCH_FILL_PARTS=1) for the A/B, then the isolated front ends. Every GPU step has its own
# time limit; the first failure ends the script.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r04}
mkdir -p $O
step() { echo "[$(date +%T)] $*"; }
if [ "${TESTS:-1}" = 1 ]; then
  step tests
  timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
  tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || { tail -40 $O/pytest_gpu.log; exit $rc; }
fi
for rep in $(seq ${REPS:-1}); do
  for parts in ${PARTS:-4 1}; do
    step bench parts=$parts rep=$rep
    SDR_BENCH_FILL_PARTS=$parts timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-isolated ${BENCH_ARGS:-} > $O/bench_p${parts}_$rep.json 2> $O/bench_p${parts}_$rep.err || { tail -20 $O/bench_p${parts}_$rep.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/bench_p${parts}_$rep.json'));t=d['pll'].get('timeline',{});print('parts=$parts', d['value'], d['ms_per_step'], d['roofline']['frac'], d['pll']['avg_launch_ms'], t)"
  done
done
step done
