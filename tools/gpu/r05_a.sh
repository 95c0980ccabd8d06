# Round 5 session A: the GPU tests, the driver-shaped bench line, then the waves-per-CU study.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05_a
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench20.json 2> $O/bench20.err || { tail -20 $O/bench20.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench20.json'));print(d['value'],d['ms_per_step'],d['roofline'],d['pll'].get('cycles_per_step'),d['pll'].get('timeline'),d['cpu_baseline'].get('dropin_1ch'))"
TAG=r05_a/pllwn bash tools/gpu/pll_waves_notab.sh > $O/pllwn.log 2>&1 || { tail -20 $O/pllwn.log; exit 1; }
