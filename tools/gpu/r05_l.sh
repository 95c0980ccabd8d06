# Round 5 session L: the MFMA front end timed by its own workgroup stamps (isolated leg of bench.py),
# the new timing test, and a rocprofv3 kernel trace of the isolated front ends for the cross-check.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05_l}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_pipeline.py -m gpu -x -v --timeout 120 --timeout-method thread -k "timing or fast_frontend" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench20.json 2> $O/bench20.err || { tail -5 $O/bench20.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench20.json')); print(json.dumps(d['frontend_isolated']))"
rm -rf /tmp/prof_fe
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_fe -o fe -- python tools/bench_frontend.py > $O/bench_frontend.txt 2> $O/bench_frontend.err || { tail -5 $O/bench_frontend.err; exit 1; }
f=$(find /tmp/prof_fe -name "*kernel_stats.csv" | head -1)
cp "$f" $O/fe_kernel_stats.csv
grep -i "frontend" $O/fe_kernel_stats.csv | cut -c1-200
cat $O/bench_frontend.txt | tail -5
