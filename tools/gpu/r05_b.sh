# Round 5 session B: GPU tests, the driver-shaped bench line, and a rocprofv3 kernel trace + stats of
# the same bench command (its line printed by the profiled run itself) for the roofline cross-check.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05_b}
mkdir -p $O
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
  tail -2 $O/pytest_gpu.log
fi
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 ${BENCH_ARGS:-} > $O/bench20.json 2> $O/bench20.err || { tail -20 $O/bench20.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench20.json'));r=d['roofline'];print('bench20',d['value'],d['ms_per_step'],r['avg_launch_ms'],r['frac'],d['pll'].get('cycles_per_step'),d['pll'].get('shader_clock_mhz'),d['pll'].get('timeline'))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-isolated > $O/tr.json 2> $O/tr.err || { tail -5 $O/tr.err; exit 1; }
f=$(find $O/tr -name "*kernel_trace.csv" | head -1)
cp "$f" $O/kernel_trace.csv
f=$(find $O/tr -name "*kernel_stats.csv" | head -1)
cp "$f" $O/kernel_stats.csv
python -c "import json;d=json.load(open('$O/tr.json'));r=d['roofline'];print('profiled',d['value'],d['ms_per_step'],r['avg_launch_ms'],r['frac'],r.get('launches_timed'))"
python tools/timeline.py $O/kernel_trace.csv --by-grid k_frontend2
