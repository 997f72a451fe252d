set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; echo "pytest exit $?"; tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 300 python tools/tune_pairwise.py --rounds 5 --variants 4,8,16 > gpurun_out/tune.log 2>&1; echo "exit $?"; tail -3 gpurun_out/tune.log
MVM_PAIRWISE_RG=1 timeout -k 10 300 python tools/tune_pairwise.py --rounds 3 --variants 8,16 > gpurun_out/tune_rg1.log 2>&1; echo "rg1 exit $?"; tail -2 gpurun_out/tune_rg1.log
timeout -k 10 300 python tools/tune_pairwise.py --rounds 3 --variants 8,16 --no-dist > gpurun_out/tune_nodist.log 2>&1; echo "exit $?"; tail -2 gpurun_out/tune_nodist.log
timeout -k 10 300 python tools/tune_pairwise.py --rounds 3 --variants 8,16 --cams 3 --dets 256 > gpurun_out/tune_c2.log 2>&1; echo "c2 exit $?"; tail -2 gpurun_out/tune_c2.log
