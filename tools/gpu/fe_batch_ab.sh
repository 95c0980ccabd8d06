# Exact front-end variants (build/variants/<name>.so, tools/build_variant.sh): front-end parity tests
# under each, then the isolated timing interleaved REPS times (tools/gpu/fe_var_ab.sh).
#   VARIANTS="feb febc" bash tools/gpu/fe_batch_ab.sh
set -o pipefail
O=gpurun_out/${TAG:-febatch}
mkdir -p $O
for v in ${VARIANTS}; do
  SDR_AMD_LIB=build/variants/$v.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_pipeline.py -k "matches_reference_golden or many_channels_vs_oracle or other_modes_vs_oracle" \
    > $O/parity_$v.txt 2>&1 || { echo "parity FAILED for $v"; tail -20 $O/parity_$v.txt; exit 1; }
  echo "$v parity: $(tail -1 $O/parity_$v.txt)"
done
VARIANTS="default ${VARIANTS}" TAG=${TAG:-febatch} REPS=${REPS:-3} bash tools/gpu/fe_var_ab.sh
