# Round 5 session P: k_stereo_out held to 128 VGPRs (4 waves per SIMD, variant sto4) against the
# default (3) -- isolated stage times, stereo GPU tests; capacity at 2048 channels with the
# release-only front-end wait (the bench's choice past 1024 channels).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05_p}
mkdir -p $O
for v in default sto4; do
  if [ $v = default ]; then unset SDR_AMD_LIB; else export SDR_AMD_LIB=$PWD/build/variants/$v.so; fi
  timeout -k 10 300 python -u -m pytest tests/test_gpu_pipeline.py -m gpu -x -q --timeout 120 --timeout-method thread -k "golden or many_channels or other_modes or fused" > $O/pytest_$v.log 2>&1 || { tail -20 $O/pytest_$v.log; exit 1; }
  echo "$v $(tail -1 $O/pytest_$v.log)"
  rm -rf /tmp/prof_$v
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_$v -o st -- python3 tools/bench_stages.py --iters 10 > $O/st_$v.log 2>&1 || { tail -10 $O/st_$v.log; exit 1; }
  f=$(find /tmp/prof_$v -name "*kernel_stats.csv" | head -1)
  cp "$f" $O/kstats_$v.csv
  grep -E "k_stereo_out|k_mono_out|k_resample_lc" $O/kstats_$v.csv | awk -F, -v v=$v '{print v, $1, $2, $4/1000}' | cut -c1-120
done
unset SDR_AMD_LIB
for r in 1 2; do
  for v in default sto4; do
    if [ $v = default ]; then unset SDR_AMD_LIB; else export SDR_AMD_LIB=$PWD/build/variants/$v.so; fi
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-isolated > $O/b_${v}_$r.json 2> $O/b_${v}_$r.err || { tail -5 $O/b_${v}_$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/b_${v}_$r.json')); p=d['pll']; print('$v', d['ms_per_step'], p.get('cycles_per_step'), p.get('shader_clock_mhz'), d['roofline']['avg_launch_ms'])"
  done
done
unset SDR_AMD_LIB
TAG=${TAG:-r05_p}/cap CASES="2048@64" bash tools/gpu/capacity.sh || exit 1
