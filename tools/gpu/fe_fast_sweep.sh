# Isolated front-end timings over the MFMA tile size (SDR_FE_NB) and grid (SDR_FE_WG_PER_CU: 0 =
# one workgroup per tile, k = persistent LDS-DMA grid of k workgroups per CU).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-fefast}
mkdir -p $O
for nb in ${NBS:-16 32 48 64}; do
  for wg in ${WGS:-0 4 8}; do
    SDR_FE_NB=$nb SDR_FE_WG_PER_CU=$wg timeout -k 10 120 python tools/bench_frontend.py --iters 30 > $O/fe_nb${nb}_wg${wg}.json 2>&1; rc=$?
    echo "nb=$nb wg=$wg $(tail -1 $O/fe_nb${nb}_wg${wg}.json)"; [ $rc -eq 0 ] || exit $rc
  done
done
