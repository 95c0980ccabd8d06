# A/B of HIP runtime settings on the bench schedule (per-wave diagnosis build, 100 steps): the
# front end's dispatch waits for earlier post-stream kernels (profiles/r04/release/)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-clr}
mkdir -p $O
TAG=${TAG:-clr} BENCH_ARGS="--steps 100" VARIANTS="${VARIANTS:-waves waves@ROC_SIGNAL_POOL_SIZE=4096 waves@ROC_AQL_QUEUE_SIZE=65536 waves@DEBUG_CLR_MAX_BATCH_SIZE=1}" REPS=1 bash tools/gpu/ab_bench.sh || exit 1
for f in $O/b_*.json; do python3 -c "
import json
d=json.loads(open('$f').read().strip().splitlines()[-1]); w=d['pll']['waves']
print('$f', d['ms_per_step'], 'poll st/rds', w['stereo_19k']['poll_us_per_block_mean'], w['rds_114k']['poll_us_per_block_mean'])
"; done
