# Round 5 session H: the GPU tests with the e bracket at 2^-45; the PLL's row-strided loads at 1, 2
# and 4 waves per CU (tools/microbench/rowload.hip) and the vector-memory counters of k_pll at 1 and 4
# waves per CU (no-table diagnosis build); two driver-shaped bench lines.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05_h}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 120 tools/microbench/bin/rowload > $O/rowload.jsonl 2> $O/rowload.err || { tail -5 $O/rowload.err; exit 1; }
cat $O/rowload.jsonl
export SDR_AMD_LIB=$PWD/build/variants/hwid_notab.so
IFS=";" read -ra G <<< "${PASSES:-SQ_WAVES TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TCP_PENDING_STALL_CYCLES_sum;SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum TA_TA_BUSY_sum TA_FLAT_READ_WAVEFRONTS_sum}"
for ch in 8192 32768; do
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
unset SDR_AMD_LIB
for r in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench20_$r.json 2> $O/bench20_$r.err || { tail -5 $O/bench20_$r.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/bench20_$r.json')); print(d['value'], d['ms_per_step'], d['pll'].get('cycles_per_step'), d['roofline']['avg_launch_ms'], d['roofline']['frac'], d.get('verified'))"
done
