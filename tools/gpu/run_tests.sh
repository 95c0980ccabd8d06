# the GPU test suite (PYTEST_ARGS overrides the selection); log in gpurun_out/pytest_gpu1.log
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -m pytest ${PYTEST_ARGS:-tests -x -q -m gpu} > gpurun_out/pytest_gpu1.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -30 gpurun_out/pytest_gpu1.log
exit $rc
