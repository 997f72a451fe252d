set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && echo SMOKE_OK || { echo SMOKE_FAIL; tail -20 gpurun_out/smoke.log; exit 1; }
timeout -k 10 900 python -m pytest tests -x -q -m gpu ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest exit $rc"
tail -30 gpurun_out/pytest_gpu.log
exit $rc
