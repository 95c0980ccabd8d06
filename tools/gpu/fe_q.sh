# Persistent (static round-robin, LDS-DMA double-buffered) MFMA front end: fast-mode parity with
# SDR_FE_WG_PER_CU=K, then isolated timings per K (0 = one tile per workgroup).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-feq}
mkdir -p $O
SDR_FE_WG_PER_CU=${TESTWG:-4} timeout -k 10 300 python -u -m pytest tests -x -q -m gpu -k fast --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; [ $rc -eq 0 ] || { tail -40 $O/pytest.log; exit $rc; }
for k in ${KS:-0 2 3 4 6}; do
  SDR_FE_WG_PER_CU=$k ${ENVS:-} timeout -k 10 120 python tools/bench_frontend.py --iters 30 > $O/fe_k$k.json 2>&1; rc=$?
  echo "k=$k $(tail -1 $O/fe_k$k.json)"; [ $rc -eq 0 ] || exit $rc
done
