# timing-only A/B of the persistent PLL's per-block hand-off (build/variants: relaxdone, noacq)
set -o pipefail
O=gpurun_out/${TAG:-handoff}
mkdir -p $O
for rep in 1 2; do
for v in ${VARIANTS:-default relaxdone noacq}; do
  if [ "$v" = default ]; then L=""; else L="build/variants/$v.so"; fi
  SDR_AMD_LIB=$L timeout -k 10 300 python bench.py --steps ${STEPS:-100} --warmup 5 --no-cpu-baseline --no-isolated > $O/b_${v}_$rep.json 2> $O/b_${v}_$rep.err || { tail -20 $O/b_${v}_$rep.err; exit 1; }
  python -c "
import json;d=json.load(open('$O/b_${v}_$rep.json'));p=d['pll'];t=p.get('timeline') or {}
comp=p['cycles_per_step']*7350/p['shader_clock_mhz']/1e3
print('$v',d['value'],d['ms_per_step'],'pll',p['avg_launch_ms'],'span/blk',round(t.get('pll_span_ms',0)/${STEPS:-100},4),'compute',round(comp,4),'clk',p['shader_clock_mhz'],'idle',t.get('pll_idle_ms'))"
done
done
