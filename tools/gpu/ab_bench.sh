# A/B of library variants (build/variants/<name>.so from tools/build_variant.sh; "default" = the
# in-tree libsdr_amd.so) on the full bench, interleaved REPS times.  VARIANTS="default nb3" REPS=2
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-abb}
mkdir -p $O
for rep in $(seq ${REPS:-2}); do
for v in ${VARIANTS:-default}; do
  if [ "$v" = default ]; then L=""; else L="build/variants/$v.so"; fi
  env SDR_AMD_LIB=$L timeout -k 10 200 python bench.py --no-cpu-baseline --no-isolated ${BENCH_ARGS:-} > $O/b_$v.json 2> $O/b_$v.err; rc=$?
  echo "$v $(python3 -c "import json,sys; d=json.load(open('$O/b_$v.json')); print(d['value'], d['ms_per_step'])")"; [ $rc -eq 0 ] || exit $rc
done
done
