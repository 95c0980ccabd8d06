# rocprofv3 kernel trace of a 20-step bench (no CPU baseline, no isolated runs); the CSV lands under
# gpurun_out/$TAG for tools/timeline.py
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-tr}
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O -o run -- python3 bench.py --steps 20 --no-cpu-baseline --no-isolated > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
f=$(find $O -name "*kernel_trace.csv" | head -1)
cp "$f" $O/kernel_trace.csv
tail -1 $O/prof.log
