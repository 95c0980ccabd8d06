# Round 5 session M: why the whole-post front-end wait speeds the PLL -- cycles per step and shader
# clock for both schedules (interleaved), 20 steps.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05_m}
mkdir -p $O
for rep in 1 2; do
  for v in library post; do
    SDR_BENCH_FE_WAIT=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-isolated > $O/b_${v}_$rep.json 2> $O/b_${v}_$rep.err || { tail -5 $O/b_${v}_$rep.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/b_${v}_$rep.json')); p=d['pll']; print('$v', d['ms_per_step'], p['avg_launch_ms'], p.get('cycles_per_step'), p.get('shader_clock_mhz'), d['roofline']['avg_launch_ms'])"
  done
done
