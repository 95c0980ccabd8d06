# Round 5 session S: MFMA front end with TPW tiles per wave (next window prefetched into registers):
# fast-mode parity under each variant, isolated A/B (3 interleaved rounds), then the driver-shaped
# bench with the per-block timeline maxima.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05_s}
mkdir -p $O
for v in tpw2 tpw3; do
  SDR_AMD_LIB=build/variants/$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_pipeline.py -k "fast_frontend or frontend_timing_stamps" > $O/parity_$v.txt 2>&1 \
    || { echo "parity FAILED for $v"; tail -30 $O/parity_$v.txt; exit 1; }
  echo "$v parity: $(tail -1 $O/parity_$v.txt)"
done
for r in 1 2 3; do
  for v in default tpw2 tpw3 tpw4 tpw2w3; do
    if [ $v = default ]; then unset SDR_AMD_LIB; else export SDR_AMD_LIB=$PWD/build/variants/$v.so; fi
    timeout -k 10 120 python tools/bench_frontend.py > $O/${v}_$r.json 2> $O/${v}_$r.err || { tail -5 $O/${v}_$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/${v}_$r.json')); print('$v', d['frontend']['fast'])"
  done
done
unset SDR_AMD_LIB
TAG=${TAG:-r05_s}/tl VARS="SDR_BENCH_FE_GATE=dsp" REPS=2 bash tools/gpu/env_ab.sh
