# A/B of library variants on the full bench, interleaved REPS times. A variant is
#   default          the in-tree libsdr_amd.so
#   <name>           build/variants/<name>.so (tools/build_variant.sh)
#   <name>@VAR=val   either of the above with an environment setting (e.g. default@SDR_BENCH_FILL_PARTS=1)
#   VARIANTS="default s1 default@SDR_BENCH_FILL_PARTS=1" REPS=2 bash tools/gpu/ab_bench.sh
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-abb}
mkdir -p $O
i=0
for rep in $(seq ${REPS:-2}); do
for v in ${VARIANTS:-default}; do
  i=$((i+1))
  lib=${v%%@*}; envs=""
  [ "$lib" != "$v" ] && envs=${v#*@}
  if [ "$lib" = default ]; then L=""; else L="build/variants/$lib.so"; fi
  env SDR_AMD_LIB=$L $envs timeout -k 10 200 python bench.py --no-cpu-baseline --no-isolated ${BENCH_ARGS:-} > $O/b_$i.json 2> $O/b_$i.err; rc=$?
  [ $rc -eq 0 ] || { tail -5 $O/b_$i.err; exit $rc; }
  echo "$v $(python3 -c "import json; d=json.load(open('$O/b_$i.json')); p=d['pll']; print(d['value'], d['ms_per_step'], 'pll', p.get('avg_launch_ms'), 'cyc/step', p.get('cycles_per_step'), 'MHz', p.get('shader_clock_mhz'), 'idle', (p.get('timeline') or {}).get('pll_idle_ms'), 'outside', (p.get('timeline') or {}).get('outside_span_ms'))")"
done
done
