#!/usr/bin/env python3
"""From a rocprofv3 kernel trace of a bench phase (tools/gpu/trace20.sh): how long after the post
stream's flag wait is dispatched the next block's front end (its k_rel_wait) is dispatched, and how
long the front-end queue sat idle before it (profiles/r04/release/gate_gaps.txt).
  python tools/gate_gaps.py gpurun_out/<tag>/kernel_trace.csv"""
import csv,sys
rows=list(csv.DictReader(open(sys.argv[1])))
pll=[r for r in rows if 'k_pll_multi' in r['Kernel_Name']]
t0=int(pll[1]['Start_Timestamp'])
rows.sort(key=lambda r:int(r['Correlation_Id']))
fw=None; prevend=None; gaps=[]
for r in rows:
    s=(int(r['Start_Timestamp'])-t0)/1e3; e=(int(r['End_Timestamp'])-t0)/1e3
    n=r['Kernel_Name']
    if 'k_flag_wait' in n: fw=(s,e)
    if r['Queue_Id']=='2' and ('indexSelect' in n or 'k_flag_store' in n): prevend=e
    if 'k_rel_wait' in n and fw and s>1000:
        gaps.append((s-fw[0], s-prevend))
import statistics as st
print(len(gaps), 'gap after flag_wait dispatch: mean %.1f; q2 idle before: mean %.1f' % (st.mean(g[0] for g in gaps), st.mean(g[1] for g in gaps)))
