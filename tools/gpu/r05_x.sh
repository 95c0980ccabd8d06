# Round 5 session X: the LDS-staged PLL loop for packed groups only (four waves per CU) and the
# bench's channel-count CU split: full GPU suite, the 1024-channel driver line, capacity lines at
# 1536, 2048 and 4096 channels (default split) and 2048 without the staged loop.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05_x}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
  || { echo "tests FAILED"; tail -30 $O/pytest_gpu.log; exit 1; }
echo "tests: $(tail -1 $O/pytest_gpu.log)"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench20.json 2> $O/bench20.err || { tail -5 $O/bench20.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench20.json')); print('1024', d['value'], d['ms_per_step'], d['roofline']['frac'], d['pll']['cycles_per_step'], d.get('verified'))"
for cfg in "1536 default" "2048 default" "4096 default" "2048 nocoal"; do
  set -- $cfg
  if [ $2 = default ]; then unset SDR_AMD_LIB; else export SDR_AMD_LIB=$PWD/build/variants/$2.so; fi
  timeout -k 10 300 python bench.py --channels $1 --steps 20 --warmup 5 --no-isolated > $O/cap_$1_$2.json 2> $O/cap_$1_$2.err || { tail -5 $O/cap_$1_$2.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/cap_$1_$2.json')); p=d['pll']; print('$1 $2', d['value'], d['ms_per_step'], p.get('mode')[:12], p.get('cycles_per_step'), p.get('timeline',{}).get('pll_idle_ms'), d.get('verified'), d['config'].get('pll_cus', d['config']))"
done
