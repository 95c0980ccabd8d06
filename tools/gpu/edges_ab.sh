# bench A/B (driver's 20-step line): SDR_BENCH_EDGES=1 (fill/drain blocks on the all-CU stream) vs 0
set -o pipefail
O=gpurun_out/${TAG:-edges}
mkdir -p $O
for rep in 1 2; do
for e in 1 0; do
  SDR_BENCH_EDGES=$e timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-isolated > $O/b_e${e}_$rep.json 2> $O/b_e${e}_$rep.err || { tail -20 $O/b_e${e}_$rep.err; exit 1; }
  python -c "import json;d=json.load(open('$O/b_e${e}_$rep.json'));print('edges=$e',d['value'],d['ms_per_step'],d['roofline']['avg_launch_ms'],d['pll']['avg_launch_ms'],d['pll'].get('timeline'),d['verified'])"
done
done
