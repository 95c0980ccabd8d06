# Front-end variants: fast-mode parity tests, then isolated timings per SDR_FE_NB tile size.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-fesweep}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -x -q -m gpu -k "${TESTK:-fast}" --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; [ $rc -eq 0 ] || { tail -40 $O/pytest.log; exit $rc; }
for nb in ${NBS:-16 24 32}; do
  SDR_FE_NB=$nb timeout -k 10 120 python tools/bench_frontend.py --iters 30 > $O/fe_nb$nb.json 2>&1; rc=$?
  echo "nb=$nb $(cat $O/fe_nb$nb.json | tail -1)"; [ $rc -eq 0 ] || exit $rc
done
if [ -n "$SQ" ]; then
  P1=SQ_WAVES,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_ACTIVE_INST_VALU,SQ_INSTS_VALU,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY
  SDR_FE_NB=${SQNB:-32} timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $P1 --output-format csv -d $O/sq1 -o fe -- python3 tools/bench_frontend.py --iters 10 > $O/sq1.log 2>&1; rc=$?
  [ $rc -eq 0 ] || { tail -20 $O/sq1.log; exit $rc; }
  find $O/sq1 -name "*counter_collection.csv" -exec cp {} $O/sq1.csv \;
fi
