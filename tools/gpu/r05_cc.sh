# Round 5 session CC: longer runs of the packed groups' LDS-staged PLL loop, outputs verified against
# the oracle over every block: 2048 channels (32-CU mask) and 1024 channels on a 16-CU mask, 100 steps.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05_cc}
mkdir -p $O
for cfg in "2048 32" "1024 16"; do
  set -- $cfg
  SDR_BENCH_CUMASK=$2 timeout -k 10 400 python bench.py --channels $1 --steps 100 --warmup 10 --no-isolated > $O/long_$1_$2.json 2> $O/long_$1_$2.err || { tail -5 $O/long_$1_$2.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/long_$1_$2.json')); p=d['pll']; v=d['cpu_baseline']['verified']; print('$1@$2', d['value'], d['ms_per_step'], p.get('cycles_per_step'), d.get('verified'), v.get('blocks'), v.get('channels'))"
done
