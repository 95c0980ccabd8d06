# kernel + memory-copy trace of sdr_multi at NCH channels (tools/multi_timeline.py reads it)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-multitrace}
mkdir -p $O
NCH=${NCH:-1024}; NB=${NB:-16}
F=/tmp/multi_in.u8
timeout -k 10 300 python tools/make_multi_input.py $F $NCH $NB > $O/gen.log 2>&1 || { cat $O/gen.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/tr -o m -- \
    real-time-sdr_amd/bin/sdr_multi $NCH --in $F --out /tmp/multi_out ${MULTI_ARGS:-} > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
grep "sdr_multi:" $O/trace.log
find $O/tr -name "*kernel_trace.csv" -exec cp {} $O/kernel_trace.csv \;
find $O/tr -name "*memory_copy_trace.csv" -exec cp {} $O/memcpy_trace.csv \;
rm -rf $O/tr
ls -la $O
