# smoke + the full GPU suite (one pytest process), per-test time limit
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && echo SMOKE_OK || { echo SMOKE_FAIL; tail -20 gpurun_out/smoke.log; exit 1; }
timeout -k 10 1000 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread --durations 15 ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest exit $rc"
tail -30 gpurun_out/pytest_gpu.log
exit $rc
