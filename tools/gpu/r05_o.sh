# Round 5 session O: 8-wave resampler workgroups and the whole-post front-end wait as defaults --
# all GPU tests, two driver-shaped bench lines, capacity at 2048 channels.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05_o}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
for r in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench20_$r.json 2> $O/bench20_$r.err || { tail -5 $O/bench20_$r.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench20_$r.json')); p=d['pll']; print(d['value'], d['ms_per_step'], p.get('cycles_per_step'), p.get('shader_clock_mhz'), d['roofline']['avg_launch_ms'], d['roofline']['frac'], d['roofline_fast']['frac'], d.get('verified'), p['timeline'])"
done
TAG=${TAG:-r05_o}/cap CASES="2048@64" bash tools/gpu/capacity.sh || exit 1
