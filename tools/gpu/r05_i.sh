# Round 5 session I: what the lane-pair chunk's loads and stores cost the PLL at one wave per CU
# (timing-only builds of a temporary, reverted edit of sdr_pll.hip's lane-pair chunk: 1 no loads, 2 no
# stores, 3 neither; results in profiles/r05/pll_nomem_ab.txt), isolated (tools/bench_pll.py,
# 2048 chains on 64 CUs), 3 interleaved rounds.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05_i}
mkdir -p $O
for r in 1 2 3; do
  for v in default nomem1 nomem2 nomem3; do
    if [ $v = default ]; then unset SDR_AMD_LIB; else export SDR_AMD_LIB=$PWD/build/variants/$v.so; fi
    timeout -k 10 120 python tools/bench_pll.py --iters 10 --channels 2048 --cus 64 > $O/${v}_$r.json 2> $O/${v}_$r.err || { tail -5 $O/${v}_$r.err; exit 1; }
    echo "$v $(cat $O/${v}_$r.json)"
  done
done
