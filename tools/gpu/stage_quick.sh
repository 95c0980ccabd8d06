# post-stage kernel change: parity tests (pipeline + width), isolated stages, the driver's bench line
set -o pipefail
O=gpurun_out/${TAG:-stq}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_width.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python tools/bench_stages.py > $O/stages.json 2> $O/stages.err || { tail $O/stages.err; exit 1; }
cat $O/stages.json
for rep in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-isolated > $O/b_$rep.json 2> $O/b_$rep.err || { tail -20 $O/b_$rep.err; exit 1; }
  python -c "import json;d=json.load(open('$O/b_$rep.json'));print(d['value'],d['ms_per_step'],d['roofline']['avg_launch_ms'],d['pll']['avg_launch_ms'],d['pll'].get('timeline'))"
done
