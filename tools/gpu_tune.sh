set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest exit $rc"; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/tune_cube.py --rounds 5 --variants tile,tile8i,tile32i,tile32j > gpurun_out/tune_cube.log 2>&1; echo "exit $?"; tail -4 gpurun_out/tune_cube.log
