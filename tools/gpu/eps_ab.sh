# e-bracket A/B: the GPU suite with the in-tree library, the bench (20/5) interleaved over VARIANTS,
# then the redo-count diagnosis builds (pll.redo in their bench lines)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-eps}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
TAG=$TAG/ab REPS=${REPS:-3} VARIANTS="${VARIANTS:-default e45}" BENCH_ARGS="--steps 20 --warmup 5" bash tools/gpu/ab_bench.sh || exit 1
for v in ${CNT:-cnt46 cnt45}; do
  SDR_AMD_LIB=build/variants/$v.so timeout -k 10 200 python bench.py --no-cpu-baseline --no-isolated --steps 20 --warmup 5 > $O/$v.json 2> $O/$v.err || { tail -5 $O/$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$v.json')); print('$v', d['ms_per_step'], json.dumps(d['pll'].get('redo')))"
done
