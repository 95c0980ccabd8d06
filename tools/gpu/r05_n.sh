# Round 5 session N: k_resample_lc occupancy variants (waves per workgroup, outputs per workgroup) --
# kernel times of the isolated stages (tools/bench_stages.py under a kernel trace) and the GPU tests of
# the RDS path for each variant.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05_n}
mkdir -p $O
for v in default w8 t16 vtap vtap1; do
  if [ $v = default ]; then unset SDR_AMD_LIB; else export SDR_AMD_LIB=$PWD/build/variants/$v.so; fi
  timeout -k 10 300 python -u -m pytest tests/test_gpu_pipeline.py -m gpu -x -q --timeout 120 --timeout-method thread -k "golden or many_channels or other_modes" > $O/pytest_$v.log 2>&1 || { tail -20 $O/pytest_$v.log; exit 1; }
  echo "$v $(tail -1 $O/pytest_$v.log)"
  rm -rf /tmp/prof_$v
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_$v -o st -- python3 tools/bench_stages.py --iters 10 > $O/st_$v.log 2>&1 || { tail -10 $O/st_$v.log; exit 1; }
  f=$(find /tmp/prof_$v -name "*kernel_stats.csv" | head -1)
  cp "$f" $O/kstats_$v.csv
  grep "k_resample_lc" $O/kstats_$v.csv | awk -F, -v v=$v '{print v, $0}' | cut -c1-160
done
