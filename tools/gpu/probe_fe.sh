# VALU-rate microbenchmark + SQ counter pass over the isolated front end (both numerics modes)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-probe}
mkdir -p $O
timeout -k 10 120 ./tools/microbench/valu_rate > $O/valu_rate.txt 2>&1; rc=$?; cat $O/valu_rate.txt; [ $rc -eq 0 ] || exit $rc
P1=${P1:-SQ_WAVES,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_ACTIVE_INST_VALU,SQ_INSTS_VALU,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY}
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $P1 --output-format csv -d $O/sq1 -o fe -- python3 tools/bench_frontend.py --iters 10 > $O/sq1.log 2>&1; rc=$?
[ $rc -eq 0 ] || { tail -20 $O/sq1.log; exit $rc; }
find $O/sq1 -name "*counter_collection.csv" -exec cp {} $O/sq1.csv \;
echo done
