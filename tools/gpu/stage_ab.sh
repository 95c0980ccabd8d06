# Isolated stage times (tools/bench_stages.py) of library variants, interleaved REPS times, after the
# pipeline and width parity tests of the default library; then the 20-step bench of each variant.
#   VARIANTS="default vtap0" REPS=3 bash tools/gpu/stage_ab.sh
set -o pipefail
O=gpurun_out/${TAG:-stab}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_width.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in $(seq ${REPS:-2}); do
  for v in ${VARIANTS:-default}; do
    if [ "$v" = default ]; then L=""; else L="build/variants/$v.so"; fi
    SDR_AMD_LIB=$L timeout -k 10 200 python tools/bench_stages.py > $O/st_${v}_$rep.json 2> $O/st_${v}_$rep.err || { tail $O/st_${v}_$rep.err; exit 1; }
    echo "$v rep$rep $(python3 -c "import json;d=json.load(open('$O/st_${v}_$rep.json'));print(d['stage_ms'])")"
  done
done
for rep in $(seq ${REPS:-2}); do
  for v in ${VARIANTS:-default}; do
    if [ "$v" = default ]; then L=""; else L="build/variants/$v.so"; fi
    SDR_AMD_LIB=$L timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-isolated > $O/b_${v}_$rep.json 2> $O/b_${v}_$rep.err || { tail -20 $O/b_${v}_$rep.err; exit 1; }
    echo "$v bench rep$rep $(python3 -c "import json;d=json.load(open('$O/b_${v}_$rep.json'));print(d['value'],d['ms_per_step'],d['pll']['avg_launch_ms'],d['pll'].get('timeline',{}).get('drain_ms'))")"
  done
done
