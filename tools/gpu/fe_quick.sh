# front-end parity tests, then an isolated A/B over variants (tools/gpu/fe_ab.sh), then optionally
# the driver's bench line. First failure ends it.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-feq}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_pipeline.py -x -q -k "golden or many_channels or knobs or other_modes" \
    --timeout 120 --timeout-method thread > $O/fe_tests.log 2>&1 || { tail -30 $O/fe_tests.log; exit 1; }
tail -1 $O/fe_tests.log
TAG=${TAG:-feq} bash tools/gpu/fe_ab.sh || exit 1
if [ "${BENCH:-0}" = 1 ]; then
  timeout -k 10 400 python bench.py --steps 20 --warmup 5 ${BENCH_ARGS:-} > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bench.json'));print(d['value'],d['ms_per_step'],d['roofline']['avg_launch_ms'],d['pll']['avg_launch_ms'],d['pll'].get('timeline'))"
fi
