set -o pipefail
mkdir -p gpurun_out/thr
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_dropin_gpu.py tests/test_batch_match_gpu.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/thr/pytest.log 2>&1; rc=$?; tail -2 gpurun_out/thr/pytest.log; exit $rc
