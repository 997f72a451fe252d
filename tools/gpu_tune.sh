set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest exit $rc"; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/tune_pairwise.py --rounds 5 --variants 16:4,16:2 > gpurun_out/tune_c3.log 2>&1; echo "exit $?"; tail -2 gpurun_out/tune_c3.log
timeout -k 10 300 python tools/tune_pairwise.py --rounds 5 --cams 3 --dets 256 --variants 16:4 > gpurun_out/tune_c2.log 2>&1; echo "exit $?"; tail -1 gpurun_out/tune_c2.log
