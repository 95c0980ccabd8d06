# Round 5 session R: per-wave PLL totals (-DSDR_PLL_WAVES=1) with the round-5 defaults, 20 steps x 2.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05_r}
mkdir -p $O
for r in 1 2; do
  SDR_AMD_LIB=$PWD/build/variants/waves.so timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-isolated > $O/w_$r.json 2> $O/w_$r.err || { tail -5 $O/w_$r.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/w_$r.json')); p=d['pll']; print(d['ms_per_step'], p.get('cycles_per_step'), json.dumps(p.get('waves')))"
done
