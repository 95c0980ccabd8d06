# Round 5 session F: dependent-chain microbenchmark, the bench line with the front end placed against
# the PLL (front_end_vs_pll_us), and the per-wave PLL diagnosis (build/variants/waves.so).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05_f}
mkdir -p $O
timeout -k 10 200 tools/microbench/bin/ifetch > $O/ifetch.jsonl 2> $O/ifetch.err || { tail $O/ifetch.err; exit 1; }
grep dependent $O/ifetch.jsonl
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-isolated > $O/bench20.json 2> $O/bench20.err || { tail -20 $O/bench20.err; exit 1; }
SDR_AMD_LIB=build/variants/waves.so timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-isolated > $O/waves20.json 2> $O/waves20.err || { tail -20 $O/waves20.err; exit 1; }
python3 -c "
import json
for f in ['bench20','waves20']:
    d=json.load(open('$O/'+f+'.json')); p=d['pll']
    print(f, d['value'], d['ms_per_step'], p.get('cycles_per_step'), json.dumps(p.get('timeline')), json.dumps(p.get('waves')))
"
