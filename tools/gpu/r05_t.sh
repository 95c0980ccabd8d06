# Round 5 session T: the base-angle LDS table in the lane-pair PLL step (SDR_PLL_BASETAB variant):
# GPU parity suite under the variant (pipeline, primitives, width), then the 20-step bench A/B.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05_t}
mkdir -p $O
SDR_AMD_LIB=$PWD/build/variants/bt.so timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_pipeline.py tests/test_gpu_primitives.py tests/test_gpu_width.py > $O/pytest_bt.txt 2>&1 \
  || { echo "parity FAILED"; tail -30 $O/pytest_bt.txt; exit 1; }
echo "bt parity: $(tail -1 $O/pytest_bt.txt)"
TAG=${TAG:-r05_t}/ab VARIANTS="default bt" REPS=3 BENCH_ARGS="--steps 20 --warmup 5" bash tools/gpu/ab_bench.sh
