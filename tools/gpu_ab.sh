# Parity subset on the new library, then an interleaved A/B of two in-tree
# builds (AB_A = previous, AB_B = current) with AB_CMD, e.g.
#   AB_TESTS='tests/test_gpu_parity.py -k cube' AB_CMD='python tools/tune_cube.py --variants fused --rounds 3' bash tools/gpu_ab.sh
set -o pipefail
mkdir -p gpurun_out
if [ -n "${AB_TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread $AB_TESTS > gpurun_out/ab_tests.log 2>&1; rc=$?
  tail -3 gpurun_out/ab_tests.log; [ $rc -eq 0 ] || exit $rc
fi
bash tools/ab_lib.sh 2>&1 | tee gpurun_out/ab.log
