# Isolated front-end A/B over environment settings of the in-tree library, interleaved REPS times:
#   CASES="base SDR_FE_MFMA_WPE=3" bash tools/gpu/fe_env_ab.sh   ("base" = no extra variable;
#   a case may set several variables joined by commas: SDR_FE_NB=16,SDR_FE_MFMA_WPE=3)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-feenv}
mkdir -p $O
for rep in $(seq ${REPS:-2}); do
for c in ${CASES:-base}; do
  if [ "$c" = base ]; then E=""; else E="${c//,/ }"; fi
  n=$(echo "$c" | tr ',=' '__')
  env $E timeout -k 10 120 python tools/bench_frontend.py --iters 30 > $O/fe_${n}_$rep.json 2>&1; rc=$?
  echo "$c $(tail -1 $O/fe_${n}_$rep.json)"; [ $rc -eq 0 ] || exit $rc
done
done
