# Round 5 session W: the PLL chunk loop through LDS for waves that share a CU (pll_run_split_coal):
# parity (pipeline tests incl. the packed-group launches at 2 and 4 waves per CU), then capacity
# lines with and without it (SDR_PLL_COAL=0 variant: tools/patches/pll_coal_knob.patch restores the knob), 20 steps, 2 interleaved rounds.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05_w}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_pipeline.py \
  > $O/pytest.txt 2>&1 || { echo "parity FAILED"; tail -30 $O/pytest.txt; exit 1; }
echo "parity: $(tail -1 $O/pytest.txt)"
for r in 1 2; do
  for cfg in "1024 16" "2048 64" "2048 32" "1024 64"; do
    set -- $cfg
    for v in default nocoal; do
      if [ $v = default ]; then unset SDR_AMD_LIB; else export SDR_AMD_LIB=$PWD/build/variants/$v.so; fi
      SDR_BENCH_CUMASK=$2 timeout -k 10 200 python bench.py --channels $1 --steps 20 --warmup 5 --no-cpu-baseline --no-isolated > $O/${v}_$1_$2_$r.json 2> $O/${v}_$1_$2_$r.err || { tail -5 $O/${v}_$1_$2_$r.err; exit 1; }
      python3 -c "import json; d=json.load(open('$O/${v}_$1_$2_$r.json')); p=d['pll']; print('$v $1@$2', d['value'], d['ms_per_step'], p.get('mode')[:10], p.get('cycles_per_step'), p.get('shader_clock_mhz'), p.get('timeline',{}).get('pll_idle_ms'))"
    done
  done
done
