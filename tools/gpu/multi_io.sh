# sdr_multi (the multi-channel receiver with its I/O) at NCH channels from a file of NB blocks in
# the page cache: MS/s, real-time factor; the same file through `cat |` (stdin); the file read alone.
set -o pipefail
O=gpurun_out/${TAG:-multi}
mkdir -p $O
NCH=${NCH:-1024}; NB=${NB:-48}
F=/tmp/multi_in.u8
timeout -k 10 300 python tools/make_multi_input.py $F $NCH $NB > $O/gen.log 2>&1 || { cat $O/gen.log; exit 1; }
ls -la $F
( time cat $F > /dev/null ) 2> $O/read_time.txt; cat $O/read_time.txt
for rd in 8 1 8; do
  SDR_MULTI_READERS=$rd timeout -k 10 300 real-time-sdr_amd/bin/sdr_multi $NCH --in $F --out /tmp/multi_out ${MULTI_ARGS:-} 2> $O/multi_file_r$rd.err > /dev/null || { tail $O/multi_file_r$rd.err; exit 1; }
  echo "readers=$rd $(tail -1 $O/multi_file_r$rd.err)"
done
timeout -k 10 300 bash -c "cat $F | real-time-sdr_amd/bin/sdr_multi $NCH --in - --out /tmp/multi_out2 ${MULTI_ARGS:-}" 2> $O/multi_stdin.err > /dev/null || { tail $O/multi_stdin.err; exit 1; }
echo "stdin $(tail -1 $O/multi_stdin.err)"
cmp /tmp/multi_out.pcm /tmp/multi_out2.pcm && cmp /tmp/multi_out.rds /tmp/multi_out2.rds && echo "file and stdin outputs identical"
ls -la /tmp/multi_out.pcm
