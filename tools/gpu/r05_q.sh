# Round 5 session Q: MFMA front-end tile size (16-output blocks per wave tile: 16, 32 = default, 48,
# 64), isolated (tools/bench_frontend.py, events over 50 launches), 3 interleaved rounds.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05_q}
mkdir -p $O
for r in 1 2 3; do
  for v in default nb16 nb48 nb64; do
    if [ $v = default ]; then unset SDR_AMD_LIB; else export SDR_AMD_LIB=$PWD/build/variants/$v.so; fi
    timeout -k 10 120 python tools/bench_frontend.py > $O/${v}_$r.json 2> $O/${v}_$r.err || { tail -5 $O/${v}_$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/${v}_$r.json')); print('$v', d['frontend']['fast'])"
  done
done
