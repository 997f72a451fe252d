# pairwise parity on the new build, then same-buffer A/B of libmvmatch_prev.so vs libmvmatch.so (C2, C3)
set -o pipefail
mkdir -p gpurun_out/abpw
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_dropin_gpu.py tests/test_distributed.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/abpw/parity.log 2>&1 || { tail -30 gpurun_out/abpw/parity.log; exit 1; }
tail -2 gpurun_out/abpw/parity.log
L=bpc_baseline_amd/lib/libmvmatch_prev.so,bpc_baseline_amd/lib/libmvmatch.so
timeout -k 10 300 python tools/ab_same_buffers.py --libs $L --workload c2 --buffers 4 --rounds 5 > gpurun_out/abpw/c2.log 2>&1 || { tail -20 gpurun_out/abpw/c2.log; exit 1; }
tail -12 gpurun_out/abpw/c2.log
timeout -k 10 400 python tools/ab_same_buffers.py --libs $L --workload c3 --buffers 6 --rounds 3 > gpurun_out/abpw/c3.log 2>&1 || { tail -20 gpurun_out/abpw/c3.log; exit 1; }
tail -14 gpurun_out/abpw/c3.log
