# bench A/B over environment settings (driver's 20-step shape): VARS="A=1 A=0" REPS=2
set -o pipefail
O=gpurun_out/${TAG:-envab}
mkdir -p $O
for rep in $(seq ${REPS:-2}); do
for v in ${VARS}; do
  env $v timeout -k 10 300 python bench.py --steps ${STEPS:-20} --warmup 5 --no-cpu-baseline --no-isolated > $O/b_${v}_$rep.json 2> $O/b_${v}_$rep.err || { tail -20 $O/b_${v}_$rep.err; exit 1; }
  python -c "import json;d=json.load(open('$O/b_${v}_$rep.json'));print('$v',d['value'],d['ms_per_step'],d['roofline']['avg_launch_ms'],d['pll']['avg_launch_ms'],d['pll'].get('timeline'))"
done
done
