# Round 5 session Y: the LDS-staged PLL loop forced on one-wave groups too (coalall variant) at 1 and
# 2 waves per CU against the default (register prefetch there); the model's CU split at 1536 and 1280
# channels; 20 steps.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05_y}
mkdir -p $O
for cfg in "1024 64 default" "1024 64 coalall" "2048 64 default" "2048 64 coalall" "1536 - default" "1280 - default" "1024 64 default" "1024 64 coalall"; do
  set -- $cfg
  if [ $3 = default ]; then unset SDR_AMD_LIB; else export SDR_AMD_LIB=$PWD/build/variants/$3.so; fi
  if [ $2 = - ]; then unset SDR_BENCH_CUMASK; else export SDR_BENCH_CUMASK=$2; fi
  timeout -k 10 300 python bench.py --channels $1 --steps 20 --warmup 5 --no-cpu-baseline --no-isolated > $O/b_$1_$2_$3.json 2> $O/b_$1_$2_$3.err || { tail -5 $O/b_$1_$2_$3.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/b_$1_$2_$3.json')); p=d['pll']; print('$1 $2 $3', d['value'], d['ms_per_step'], p.get('cycles_per_step'), p.get('shader_clock_mhz'), p.get('timeline',{}).get('pll_idle_ms'), d['config']['pll_cus'])"
done
