# PMC counters (one pass, SQ + GRBM) over the isolated front end; summary per kernel
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-fepmc}
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --pmc ${PMC_LIST:-SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE} --output-format csv -d $O/pmc -o fe -- python3 tools/bench_frontend.py --iters 5 ${FE_ARGS:-} > $O/pmc.log 2>&1 || { tail -20 $O/pmc.log; exit 1; }
python3 - $O <<'PY'
import csv, glob, sys, collections
d = sys.argv[1]
f = glob.glob(d + "/pmc/**/*counter_collection.csv", recursive=True)[0]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(f)):
    n = r["Kernel_Name"]
    if "frontend" not in n and "k_pll" not in n:
        continue
    key = n.split("(")[0][-40:] + n[n.find("<"):n.find(">") + 1]
    agg[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, c in agg.items():
    m = {n: sum(v) / len(v) for n, v in c.items()}
    print(k, {n: round(v) for n, v in m.items()})
    if m.get("SQ_WAVE_CYCLES"):
        w = m["SQ_WAVE_CYCLES"]
        print("   valu/wave-cycle %.3f  wait_any %.3f  wait_inst %.3f  active_any %.3f  waves %d" % (
            m.get("SQ_ACTIVE_INST_VALU", 0) / w, m.get("SQ_WAIT_ANY", 0) / w, m.get("SQ_WAIT_INST_ANY", 0) / w,
            m.get("SQ_ACTIVE_INST_ANY", 0) / w, m.get("SQ_WAVES", 0)))
PY
