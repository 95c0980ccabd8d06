# Round 5 session G: chunk redos by reason and job (SDR_PLL_COUNT diagnosis builds) at the e bracket's
# 2^-44 and 2^-45; where four k_pll waves per CU run (SDR_PLL_HWID builds, tools/diag_pll_place.py)
# beside one-wave f64 microbenchmark workgroups of the same register footprint; then the
# product-build timing A/B of the 2^-45 bracket.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05_g}
mkdir -p $O
for v in cnt cnt45; do
  SDR_AMD_LIB=$PWD/build/variants/$v.so timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-isolated > $O/$v.json 2> $O/$v.err || { tail -5 $O/$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$v.json')); p=d['pll']; print('$v', p.get('cycles_per_step'), json.dumps(p.get('chunk_redo')))"
done
timeout -k 10 120 tools/microbench/bin/ifetch wg1 > $O/wg1.jsonl 2> $O/wg1.err || { tail -5 $O/wg1.err; exit 1; }
cat $O/wg1.jsonl
for ch in 8192 16384 32768; do
  SDR_AMD_LIB=$PWD/build/variants/hwid_notab.so timeout -k 10 120 python tools/diag_pll_place.py --channels $ch --raw $O/place_notab_$ch.rows.json > $O/place_notab_$ch.json 2> $O/place_notab_$ch.err || { tail -5 $O/place_notab_$ch.err; exit 1; }
  cat $O/place_notab_$ch.json
done
for cus in 64 32; do
  SDR_AMD_LIB=$PWD/build/variants/hwid.so timeout -k 10 120 python tools/diag_pll_place.py --channels 2048 --cus $cus > $O/place_tab_cus$cus.json 2> $O/place_tab_cus$cus.err || { tail -5 $O/place_tab_cus$cus.err; exit 1; }
  cat $O/place_tab_cus$cus.json
done
TAG=r05_g/ab VARIANTS="default e45" REPS=3 BENCH_ARGS="--steps 20 --warmup 5" bash tools/gpu/ab_bench.sh
