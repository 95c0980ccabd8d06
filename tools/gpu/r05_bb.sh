# Round 5 session BB: capacity lines at 3072 and 8192 channels on one GPU with the bench's CU split
# (pll_cus), 20 steps, outputs verified against the oracle.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05_bb}
mkdir -p $O
for n in 3072 8192; do
  timeout -k 10 400 python bench.py --channels $n --steps 20 --warmup 5 --no-isolated > $O/cap_$n.json 2> $O/cap_$n.err || { tail -5 $O/cap_$n.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/cap_$n.json')); p=d['pll']; print('$n', d['value'], d['ms_per_step'], p.get('mode')[:12], p.get('cycles_per_step'), p.get('timeline',{}).get('pll_idle_ms'), d.get('verified'), d['config']['pll_cus'])"
done
