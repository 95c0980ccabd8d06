# PLL waves per CU: the isolated lane-pair PLL (tools/bench_pll.py, 2048 chains = 64 waves) on a
# stream CU-masked to 64 / 32 / 16 CUs (1 / 2 / 4 waves per CU), timed, then SQ counter passes per
# mask (one rocprofv3 --pmc run per group, each under its own limit; first failure ends the script).
#   TAG=r05_pllcu bash tools/gpu/pll_cu.sh
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-pllcu}
mkdir -p $O
timeout -k 10 60 rocprofv3 --list-avail > $O/avail.txt 2>&1 || true
for cu in ${CUS:-64 32 16}; do
  timeout -k 10 120 python tools/bench_pll.py --iters 5 --cus $cu > $O/t_$cu.json 2> $O/t_$cu.err || { tail $O/t_$cu.err; exit 1; }
  cat $O/t_$cu.json
done
IFS=";" read -ra G <<< "${PASSES:-SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU;SQ_WAVES SQ_IFETCH SQ_WAIT_ANY SQ_INSTS_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_LDS}"
for cu in ${CUS:-64 32 16}; do
  i=0
  for grp in "${G[@]}"; do
    i=$((i+1))
    echo "[cus $cu pass $i] $grp"
    timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d $O/c${cu}_p$i -o r -- \
        python3 tools/bench_pll.py --iters 2 --cus $cu > $O/c${cu}_p$i.log 2>&1 || { tail -20 $O/c${cu}_p$i.log; exit 1; }
    f=$(find $O/c${cu}_p$i -name "*counter_collection.csv" | head -1)
    cp "$f" $O/c${cu}_p$i.csv
    python tools/sq_summary.py $O/c${cu}_p$i.csv k_pll
  done
done
