# The fill's first FIR tile as two published 1024-sample halves (in-tree) against one 2048-sample
# range (variant fillold): GPU tests, 20-step A/B (fill_ms in each line), a trace of the fill
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-fill}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
TAG=${TAG:-fill}/s20 BENCH_ARGS="--steps 20" VARIANTS="default fillold" REPS=3 bash tools/gpu/ab_bench.sh || exit 1
for f in $O/s20/b_*.json; do python3 -c "import json;d=json.load(open('$f'));print('$f', d['ms_per_step'], d['pll']['timeline'])"; done
TAG=${TAG:-fill}/tr bash tools/gpu/trace20.sh || exit 1
python3 tools/timeline.py $O/tr/kernel_trace.csv --launch 1 --rows 40 | head -42
