# End-of-session check: GPU tests and the default bench line with its CPU baseline.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-final}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || { tail -40 $O/pytest_gpu.log; exit $rc; }
timeout -k 10 400 python bench.py ${BENCH_ARGS:-} > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]);print(d['value'], d['ms_per_step'], d['steps'], d['pll'].get('timeline'), d.get('cpu_baseline',{}).get('value'))"
