# packed pilot+band pairs in the 3-filter pass: parity tests, isolated stage A/B (SDR_FRB_PK=1/0), bench
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-frb}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_width.py tests/test_gpu_ranks.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do
for pk in 1 0; do
  SDR_FRB_PK=$pk timeout -k 10 200 python tools/bench_stages.py > $O/st_pk${pk}_$rep.json 2> $O/st_pk${pk}_$rep.err || { tail $O/st_pk${pk}_$rep.err; exit 1; }
  echo "pk=$pk $(cat $O/st_pk${pk}_$rep.json)"
done
done
for rep in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-isolated > $O/b_$rep.json 2> $O/b_$rep.err || { tail -20 $O/b_$rep.err; exit 1; }
  python -c "import json;d=json.load(open('$O/b_$rep.json'));print(d['value'],d['ms_per_step'],d['roofline']['avg_launch_ms'],d['pll']['avg_launch_ms'],d['pll'].get('timeline'))"
done
