# Round 5 session FF: the packed groups' staged loop with a 3-buffer DMA ring (default) against 2 buffers (ring2):
# read: 6 LDS-DMA pieces per chunk instead of 8, ring2) against the default: packed-group parity,

set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05_ff}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_pipeline.py -k "packed_groups or persistent" > $O/pytest_ring2.txt 2>&1 || { echo "parity FAILED"; tail -30 $O/pytest_ring2.txt; exit 1; }
echo "ring2 parity: $(tail -1 $O/pytest_ring2.txt)"
for r in 1 2; do
  for cfg in "1024 16 default" "1024 16 ring2" "2048 32 default" "2048 32 ring2"; do
    set -- $cfg
    if [ $3 = default ]; then unset SDR_AMD_LIB; else export SDR_AMD_LIB=$PWD/build/variants/$3.so; fi
    SDR_BENCH_CUMASK=$2 timeout -k 10 300 python bench.py --channels $1 --steps 20 --warmup 5 --no-cpu-baseline --no-isolated > $O/b_$1_$2_$3_$r.json 2> $O/b_$1_$2_$3_$r.err || { tail -5 $O/b_$1_$2_$3_$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/b_$1_$2_$3_$r.json')); p=d['pll']; print('$1@$2 $3', d['value'], d['ms_per_step'], p.get('cycles_per_step'), p.get('shader_clock_mhz'), p.get('timeline',{}).get('pll_idle_ms'))"
  done
done
