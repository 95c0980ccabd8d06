# Isolated front-end A/B over library variants (build/variants/<name>.so; "default" = in-tree lib),
# interleaved REPS times: VARIANTS="default fepf5" [ENVS="NAME=value"] bash tools/gpu/fe_ab.sh
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-feab}
mkdir -p $O
for rep in $(seq ${REPS:-2}); do
for v in ${VARIANTS:-default}; do
  if [ "$v" = default ]; then L=""; else L="build/variants/$v.so"; fi
  env SDR_AMD_LIB=$L ${ENVS:-} timeout -k 10 120 python tools/bench_frontend.py --iters 30 > $O/fe_${v}_$rep.json 2>&1; rc=$?
  echo "$v $(tail -1 $O/fe_${v}_$rep.json)"; [ $rc -eq 0 ] || exit $rc
done
done
