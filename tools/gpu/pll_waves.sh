# PLL waves per CU without a CU mask (rocprofv3 --pmc does not honour stream CU masks: every mask
# gave the same per-wave counters, profiles/r05/pll_cu/): the isolated lane-pair PLL with 256 / 512 /
# 1024 waves (8192 / 16384 / 32768 chains) on the whole device = 1 / 2 / 4 waves per CU, timed, then
# SQ counter passes per size (one rocprofv3 --pmc run per group, each under its own limit).
#   TAG=r05_pllw bash tools/gpu/pll_waves.sh
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-pllw}
mkdir -p $O
for ch in ${CHAINS:-8192 16384 32768}; do
  timeout -k 10 120 python tools/bench_pll.py --iters 5 --channels $ch > $O/t_$ch.json 2> $O/t_$ch.err || { tail $O/t_$ch.err; exit 1; }
  cat $O/t_$ch.json
done
IFS=";" read -ra G <<< "${PASSES:-SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU;SQ_WAVES SQ_IFETCH SQ_WAIT_ANY SQ_INSTS_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_LDS;SQ_WAVES SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_TC_INST_REQ SQ_ACTIVE_INST_VALU2 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_CVT}"
for ch in ${CHAINS:-8192 16384 32768}; do
  i=0
  for grp in "${G[@]}"; do
    i=$((i+1))
    echo "[chains $ch pass $i] $grp"
    timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $O/c${ch}_p$i -o r -- \
        python3 tools/bench_pll.py --iters 2 --channels $ch > $O/c${ch}_p$i.log 2>&1 || { tail -20 $O/c${ch}_p$i.log; exit 1; }
    f=$(find $O/c${ch}_p$i -name "*counter_collection.csv" | head -1)
    cp "$f" $O/c${ch}_p$i.csv
    python tools/sq_summary.py $O/c${ch}_p$i.csv "k_pll<"
  done
done
