# isolated exact front end over library variants with env settings: VARIANTS="default feb default@NAME=value"
set -o pipefail
O=gpurun_out/${TAG:-fevar}
mkdir -p $O
for rep in $(seq ${REPS:-2}); do
for v in ${VARIANTS}; do
  lib=${v%%@*}; envs=""
  [ "$lib" != "$v" ] && envs=${v#*@}
  if [ "$lib" = default ]; then L=""; else L="build/variants/$lib.so"; fi
  env SDR_AMD_LIB=$L $envs timeout -k 10 120 python tools/bench_frontend.py --iters 30 > $O/fe_${v}_$rep.json 2>&1 || { tail -5 $O/fe_${v}_$rep.json; exit 1; }
  echo "$v $(python3 -c "import json; d=json.load(open('$O/fe_${v}_$rep.json'.replace('@','@'))) if False else None" 2>/dev/null)$(tail -1 $O/fe_${v}_$rep.json | cut -c1-140)"
done
done
