# bench at 20 steps (2 runs) and the per-wave diagnosis at 100 steps, then a kernel trace: the
# front end's dispatch against the post stream's flag wait (tools/timeline.py --gate)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-chain}
mkdir -p $O
TAG=${TAG:-chain}/s20 BENCH_ARGS="--steps 20" VARIANTS="default" REPS=2 bash tools/gpu/ab_bench.sh || exit 1
TAG=${TAG:-chain}/s100 BENCH_ARGS="--steps 100" VARIANTS="default waves" REPS=1 bash tools/gpu/ab_bench.sh || exit 1
python3 -c "
import json
d=json.loads(open('$O/s100/b_2.json').read().strip().splitlines()[-1]); p=d['pll']
print(json.dumps(p['timeline'])); print(json.dumps(p['waves']))
"
TAG=${TAG:-chain}/tr bash tools/gpu/trace20.sh || exit 1
