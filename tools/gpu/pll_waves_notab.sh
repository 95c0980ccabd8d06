# As pll_waves.sh with the trigArg LDS table off (a variant build, SDR_PLL_NOTAB=1): no LDS, so 1024
# one-wave workgroups are resident at once (4 per CU, one per SIMD), which the table (59 KB per wave,
# two per CU) prevents in the product build.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-pllwn}
mkdir -p $O
export SDR_AMD_LIB=$PWD/build/variants/notab.so
for ch in ${CHAINS:-8192 16384 32768}; do
  timeout -k 10 120 python tools/bench_pll.py --iters 5 --channels $ch > $O/t_$ch.json 2> $O/t_$ch.err || { tail $O/t_$ch.err; exit 1; }
  cat $O/t_$ch.json
done
IFS=";" read -ra G <<< "${PASSES:-SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU;SQ_WAVES SQ_IFETCH SQ_WAIT_ANY SQ_INSTS_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_IFETCH_LEVEL;SQ_WAVES SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_TC_INST_REQ SQC_ICACHE_BUSY_CYCLES SQC_ICACHE_INPUT_VALID_READYB SQ_INSTS_VALU_CVT}"
for ch in ${CHAINS:-8192 32768}; do
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
