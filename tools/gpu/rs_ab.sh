# The RDS resampler's staging (scalar table reads, tap rows loaded with the x tile) against the
# previous form (variant rsold): GPU tests, 20/100-step A/B, the per-wave diagnosis, a kernel trace
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-rs}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
TAG=${TAG:-rs}/s20 BENCH_ARGS="--steps 20" VARIANTS="default rsold" REPS=3 bash tools/gpu/ab_bench.sh || exit 1
TAG=${TAG:-rs}/s100 BENCH_ARGS="--steps 100" VARIANTS="default rsold" REPS=2 bash tools/gpu/ab_bench.sh || exit 1
VARIANTS="waves" TAG=${TAG:-rs}/w bash tools/gpu/clr_ab.sh || exit 1
TAG=${TAG:-rs}/tr bash tools/gpu/trace20.sh || exit 1
python3 tools/timeline.py $O/tr/kernel_trace.csv --launch 1 --rows 70 | tail -22
