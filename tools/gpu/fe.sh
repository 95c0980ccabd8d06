# isolated front end (tools/bench_frontend.py, both numerics modes); PMC=1 adds a kernel trace and one SQ counter pass
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python tools/bench_frontend.py > gpurun_out/fe.json 2> gpurun_out/fe.err; rc=$?
cat gpurun_out/fe.json; tail -3 gpurun_out/fe.err
[ $rc -eq 0 ] || exit $rc
if [ -n "$PMC" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fe_prof -o fe -- python3 tools/bench_frontend.py --iters 10 > gpurun_out/fe_prof.log 2>&1 || exit $?
  timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/fe_pmc1 -o pmc -- python3 tools/bench_frontend.py --iters 10 > gpurun_out/fe_pmc1.log 2>&1 || exit $?
fi
