# exact front end discriminator A/B: the GPU suite (incl. the v_rcp_f64 bound), isolated front end
# over the product library and VARIANTS, then the bench line
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-fedisc}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -q -s -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log; grep "v_rcp_f64 max" $O/pytest_gpu.log
TAG=$TAG/ab REPS=${REPS:-3} VARIANTS="${VARIANTS:-default disc0}" bash tools/gpu/fe_var_ab.sh || exit 1
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], d['verified'], d['roofline']['frac'], d['roofline']['avg_launch_ms'], d['frontend_isolated']['exact']['avg_launch_ms'], d['frontend_isolated']['exact']['frac'])"
