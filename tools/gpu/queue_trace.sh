# Kernel trace of the queue-plumbed receiver (bench.py --queue-child) beside the bench's own pipeline
# at the same width, for the per-block kernel budget of each.  TAG=... [BLOCKS=40] bash tools/gpu/queue_trace.sh
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-queue_trace}
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_q -o q -- \
    python3 bench.py --queue-child --channels 1024 --blocks ${BLOCKS:-40} --cus 64 --cap-ch 0 --cap-out /tmp/q.npz \
    > $O/q.log 2>&1 || { tail -20 $O/q.log; exit 1; }
find $O/prof_q -name "*kernel_stats.csv" -exec cp {} $O/q_kernel_stats.csv \;
find $O/prof_q -name "*kernel_trace.csv" -exec cp {} $O/q_kernel_trace.csv \;
rm -rf $O/prof_q
grep '^{' $O/q.log | tail -1
head -25 $O/q_kernel_stats.csv | cut -d, -f1-8 | cut -c1-200
