# Round 5 session J (run with tools/patches/pll_ci_layout.patch applied): the chunk-interleaved PLL input layout -- GPU tests, capacity lines (4 PLL waves
# per CU: 2048 channels on 32 CUs, 1024 on 16) and two driver-shaped bench lines.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05_j}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
TAG=${TAG:-r05_j}/cap CASES="${CASES:-2048@64 2048@32 1024@16 1024@32}" bash tools/gpu/capacity.sh || exit 1
for r in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench20_$r.json 2> $O/bench20_$r.err || { tail -5 $O/bench20_$r.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench20_$r.json')); p=d['pll']; print(d['value'], d['ms_per_step'], p.get('cycles_per_step'), p.get('shader_clock_mhz'), d['roofline']['avg_launch_ms'], d['roofline']['frac'], d.get('verified'))"
done
