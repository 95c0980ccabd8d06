# kernel trace of tools/microbench/stream_gate.py (does a masked stream start work while another queue waits?)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/gate
mkdir -p $O
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O -o run -- python3 tools/microbench/stream_gate.py > $O/log 2>&1 || { tail -5 $O/log; exit 1; }
f=$(find $O -name "*kernel_trace.csv" | head -1); cp "$f" $O/kernel_trace.csv
python3 - <<'PY'
import csv
rows=sorted(csv.DictReader(open('gpurun_out/gate/kernel_trace.csv')), key=lambda r:int(r['Correlation_Id']))
rows=[r for r in rows if int(r['Correlation_Id'])>2]
t0=int(rows[0]['Start_Timestamp'])
for r in rows:
    s=(int(r['Start_Timestamp'])-t0)/1e3; e=(int(r['End_Timestamp'])-t0)/1e3
    print(f"{int(r['Correlation_Id']):5d} q{r['Queue_Id']:>2} {s:10.1f} {e:10.1f} {r['Kernel_Name'][5:45]}")
PY
