# GPU tests, then the bench with the library's parity release (default) against the explicit wait
# for block b-2's whole post stream (SDR_BENCH_FE_WAIT=post), 20 and 100 steps, plus the per-wave
# diagnosis build at 100 steps.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-rel}
mkdir -p $O
timeout -k 10 420 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
TAG=${TAG:-rel}/s20 BENCH_ARGS="--steps 20" VARIANTS="default default@SDR_BENCH_FE_WAIT=post" REPS=2 bash tools/gpu/ab_bench.sh || exit 1
TAG=${TAG:-rel}/s100 BENCH_ARGS="--steps 100" VARIANTS="default default@SDR_BENCH_FE_WAIT=post waves" REPS=1 bash tools/gpu/ab_bench.sh || exit 1
python3 -c "
import json
d=json.loads(open('$O/s100/b_3.json').read().strip().splitlines()[-1]); p=d['pll']
print(json.dumps(p['timeline'])); print(json.dumps(p['waves']))
"
TAG=${TAG:-rel}/tr bash tools/gpu/trace20.sh || exit 1
