# Round 5 session U: counters of the two front ends isolated (tools/bench_frontend.py): SQ issue and
# wait, memory instruction mix, MFMA busy, texture addresser / L1 / L2. One counter group per pass,
# each under its own time limit; the first failure ends the script.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05_u}
mkdir -p $O
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_LDS" \
           "SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT" \
           "TA_TA_BUSY_sum TA_FLAT_READ_WAVEFRONTS_sum TCP_PENDING_STALL_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  echo "[pass $i] $grp"
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d /tmp/fepmc$i -o fe -- \
      python3 tools/bench_frontend.py --iters 3 > $O/pmc$i.log 2>&1 || { tail -20 $O/pmc$i.log; exit 1; }
  f=$(find /tmp/fepmc$i -name "*counter_collection.csv" | head -1)
  cp "$f" $O/pmc$i.csv
  python3 tools/sq_summary.py $O/pmc$i.csv k_frontend
done
