# GPU tests, then the per-wave PLL diagnosis (build/variants/waves.so, -DSDR_PLL_WAVES=1) at 20 and
# 100 steps, then the in-tree library's bench at 20 steps.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-waves}
mkdir -p $O
timeout -k 10 420 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
for st in 20 100; do
  SDR_AMD_LIB=build/variants/waves.so timeout -k 10 240 python bench.py --no-cpu-baseline --no-isolated --steps $st > $O/w$st.json 2> $O/w$st.err || { tail -5 $O/w$st.err; exit 1; }
done
timeout -k 10 240 python bench.py --no-cpu-baseline --no-isolated > $O/b20.json 2> $O/b20.err || { tail -5 $O/b20.err; exit 1; }
python3 -c "
import json
for f in ['w20','w100','b20']:
    d=json.loads(open('$O/'+f+'.json').read().strip().splitlines()[-1]); p=d['pll']
    print(f, d['value'], d['ms_per_step'], p.get('avg_launch_ms'), p.get('cycles_per_step'), json.dumps(p.get('timeline')), json.dumps(p.get('waves')))
"
