# Capacity lines: bench at more channels per GPU with the PLL stream's CU mask varied
# (CASES="2048@64 2048@32 4096@64"), 20 steps, no CPU baseline or isolated legs.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-cap}
mkdir -p $O
for c in ${CASES:-2048@64 2048@32 4096@64}; do
  ch=${c%@*}; cu=${c#*@}
  echo "[$(date +%T)] channels=$ch cumask=$cu"
  SDR_BENCH_CUMASK=$cu timeout -k 10 400 python bench.py --channels $ch --steps 20 --warmup 5 --no-cpu-baseline --no-isolated > $O/b_${ch}_${cu}.json 2> $O/b_${ch}_${cu}.err || { tail -20 $O/b_${ch}_${cu}.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/b_${ch}_${cu}.json'));p=d['pll'];print('$c', d['value'], d['ms_per_step'], p.get('mode'), p.get('cycles_per_step'), p.get('timeline'))"
done
