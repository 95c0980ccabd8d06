# Round 5 session C: tests, bench line, kernel trace (roofline cross-check), isolated stages.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05_c}
mkdir -p $O
TAG=${TAG:-r05_c} bash tools/gpu/r05_b.sh || exit 1
timeout -k 10 200 python tools/bench_stages.py --iters 20 > $O/stages.json 2> $O/stages.err || { tail -5 $O/stages.err; exit 1; }
cat $O/stages.json | head -c 3000
