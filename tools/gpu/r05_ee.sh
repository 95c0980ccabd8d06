# Round 5 session EE: final tree (x-only staged PLL loop for packed groups): smoke, full GPU suite,
# the driver's 20-step line, the 2048-channel capacity line (verified).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05_ee}
mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
  || { echo "tests FAILED"; tail -30 $O/pytest_gpu.log; exit 1; }
echo "tests: $(tail -1 $O/pytest_gpu.log)"
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench20.json 2> $O/bench20.err || { tail -5 $O/bench20.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench20.json')); print('1024', d['value'], d['ms_per_step'], d['roofline']['frac'], d['pll']['cycles_per_step'], d.get('verified'))"
timeout -k 10 300 python bench.py --channels 2048 --steps 20 --warmup 5 --no-isolated > $O/cap_2048.json 2> $O/cap_2048.err || { tail -5 $O/cap_2048.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/cap_2048.json')); p=d['pll']; print('2048', d['value'], d['ms_per_step'], p.get('cycles_per_step'), d.get('verified'), d['config']['pll_cus'])"
