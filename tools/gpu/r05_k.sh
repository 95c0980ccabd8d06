# Round 5 session K (default = the library with tools/patches/pll_ci_layout.patch applied): the chunk-interleaved (CI) PLL inputs against the per-channel rows (variant
# build of the previous commit, build/variants/rows.so): the isolated PLL at 1 wave per CU and
# kernel-trace stats of a short pipeline run for each.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05_k}
mkdir -p $O
for r in 1; do
  for v in default rows; do
    if [ $v = default ]; then unset SDR_AMD_LIB; else export SDR_AMD_LIB=$PWD/build/variants/$v.so; fi
    timeout -k 10 120 python tools/bench_pll.py --iters 10 --channels 2048 --cus 64 > $O/pll_${v}_$r.json 2> $O/pll_${v}_$r.err || { tail -5 $O/pll_${v}_$r.err; exit 1; }
    echo "$v $(cat $O/pll_${v}_$r.json)"
  done
done
for v in default rows; do
  if [ $v = default ]; then unset SDR_AMD_LIB; else export SDR_AMD_LIB=$PWD/build/variants/$v.so; fi
  rm -rf /tmp/prof_$v
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_$v -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-isolated > $O/bench_$v.json 2> $O/bench_$v.err || { tail -5 $O/bench_$v.err; exit 1; }
  f=$(find /tmp/prof_$v -name "*kernel_stats.csv" | head -1)
  cp "$f" $O/kstats_$v.csv
  python3 - "$O/kstats_$v.csv" "$v" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:12]:
    print(sys.argv[2], r["Name"][:60].ljust(60), r["Calls"], round(float(r["AverageNs"]) / 1e3, 1))
PY
done
