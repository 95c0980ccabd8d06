set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03_v1}; mkdir -p $O
cat /sys/fs/cgroup/cpu.max > $O/cpu_max.txt 2>&1 || true
python -c "import os;print(len(os.sched_getaffinity(0)), os.cpu_count())" >> $O/cpu_max.txt
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 600 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -15 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err; rc=$?; cat $O/bench.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/bench_stages.py > $O/stages.json 2> $O/stages.err; rc=$?; cat $O/stages.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/sprof -o st -- python3 tools/bench_stages.py > $O/sprof.log 2>&1; rc=$?
[ $rc -eq 0 ] || { tail -20 $O/sprof.log; exit $rc; }
find $O/sprof -name "*kernel_stats.csv" -exec cp {} $O/stages_kernel_stats.csv \;
rm -rf $O/sprof
cut -d, -f1-4 $O/stages_kernel_stats.csv | cut -c1-140 | head -30
