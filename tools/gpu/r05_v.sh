# Round 5 session V: is the PLL's slowdown at 2 and 4 waves per CU all memory traffic? Timing-only
# builds of the lane-pair chunk without its loads (nm1) or without loads and stores (nm3)
# (tools/patches/pll_nomem_diag.patch) in the persistent bench (no output check: --no-cpu-baseline):
# 1024 channels on 64 CUs (1 wave per CU) and 16 CUs (4, packed workgroups), 2048 on 64 (2).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05_v}
mkdir -p $O
for cfg in "1024 64" "1024 16" "2048 64"; do
  set -- $cfg
  for v in default nm1 nm3; do
    if [ $v = default ]; then unset SDR_AMD_LIB; else export SDR_AMD_LIB=$PWD/build/variants/$v.so; fi
    SDR_BENCH_CUMASK=$2 timeout -k 10 200 python bench.py --channels $1 --steps 10 --warmup 3 --no-cpu-baseline --no-isolated > $O/${v}_$1_$2.json 2> $O/${v}_$1_$2.err || { tail -5 $O/${v}_$1_$2.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/${v}_$1_$2.json')); p=d['pll']; print('$v $1@$2', d['ms_per_step'], p.get('mode'), p.get('cycles_per_step'), p.get('shader_clock_mhz'))"
  done
done
