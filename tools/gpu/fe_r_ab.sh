# Isolated exact front end, outputs per lane R (SDR_FE_R, experimental knob), interleaved REPS times.
set -o pipefail
O=gpurun_out/${TAG:-fe_r}
mkdir -p $O
for rep in $(seq ${REPS:-2}); do
  for r in ${RS:-8 16}; do
    SDR_FE_R=$r timeout -k 10 120 python tools/bench_frontend.py --iters 30 > $O/fe_r${r}_$rep.json 2>&1 || { tail -5 $O/fe_r${r}_$rep.json; exit 1; }
    echo "R=$r rep $rep: $(cat $O/fe_r${r}_$rep.json)"
  done
done
