# The 20-step line after 5 and after 40 untimed warm-up blocks (does the shader clock settle?)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/warm
mkdir -p $O
i=0
for rep in 1 2; do for w in 5 40; do
  i=$((i+1))
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-isolated --steps 20 --warmup $w > $O/b_$i.json 2> $O/b_$i.err || { tail -5 $O/b_$i.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/b_$i.json'));p=d['pll'];print('warmup $w', d['ms_per_step'], p['cycles_per_step'], p['shader_clock_mhz'], p['timeline']['pll_span_ms'])"
done; done
