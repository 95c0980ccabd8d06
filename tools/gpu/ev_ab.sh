# A/B of the bench's per-block timing events (SDR_BENCH_EVENTS=edges: first two and last two blocks
# only) at 20 and 100 steps, the per-wave diagnosis build beside each, and a kernel trace with edges
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-ev}
mkdir -p $O
TAG=${TAG:-ev}/s20 BENCH_ARGS="--steps 20" VARIANTS="default default@SDR_BENCH_EVENTS=edges" REPS=2 bash tools/gpu/ab_bench.sh || exit 1
TAG=${TAG:-ev}/s100 BENCH_ARGS="--steps 100" VARIANTS="waves waves@SDR_BENCH_EVENTS=edges" REPS=1 bash tools/gpu/ab_bench.sh || exit 1
for i in 1 2; do python3 -c "
import json
d=json.loads(open('$O/s100/b_$i.json').read().strip().splitlines()[-1]); p=d['pll']
print(json.dumps(p['timeline'])); print(json.dumps(p['waves']))
"; done
SDR_BENCH_EVENTS=edges TAG=${TAG:-ev}/tr bash tools/gpu/trace20.sh || exit 1
