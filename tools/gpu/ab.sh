# A/B timing of library variants (build/variants/<name>.so, tools/build_variant.sh) on the isolated
# front end; "default" = the in-tree libsdr_amd.so. VARIANTS="default u2" [ENVS="NAME=value"]
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-ab}
mkdir -p $O
for rep in 1 2; do
for v in ${VARIANTS:-default}; do
  if [ "$v" = default ]; then L=""; else L="build/variants/$v.so"; fi
  env SDR_AMD_LIB=$L ${ENVS:-} timeout -k 10 120 python tools/bench_frontend.py --iters 30 > $O/fe_$v.json 2>&1; rc=$?
  echo "$v $(tail -1 $O/fe_$v.json)"; [ $rc -eq 0 ] || exit $rc
done
done
