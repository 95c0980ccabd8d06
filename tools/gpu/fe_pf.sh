# prefetching exact front end (k_frontend_pf, SDR_FE_PF=1): the GPU suite with the default front end
# and again with SDR_FE_PF=1, the isolated A/B, then the bench line with each
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-fepf}
mkdir -p $O
if [ "${TESTS:-1}" = 1 ]; then
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
SDR_FE_PF=1 timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu_pf.log 2>&1 || { tail -40 $O/pytest_gpu_pf.log; exit 1; }
tail -1 $O/pytest_gpu_pf.log
fi
TAG=$TAG/ab REPS=${REPS:-3} VARIANTS="${VARIANTS:-default default@SDR_FE_PF=1}" bash tools/gpu/fe_var_ab.sh || exit 1
for v in 0 1; do
  SDR_FE_PF=$v timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_pf$v.json 2> $O/bench_pf$v.err || { tail -20 $O/bench_pf$v.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/bench_pf$v.json').read().strip().splitlines()[-1])
print('pf$v', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['avg_launch_ms'], d['frontend_isolated']['exact']['avg_launch_ms'], d['frontend_isolated']['exact']['frac'])"
done
