# same-buffer A/B of libmvmatch_prev.so vs libmvmatch.so on C3 and C2 (pairwise parity first)
set -o pipefail
mkdir -p gpurun_out/abpw
[ -n "$AB_SKIP_TESTS" ] || timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k pairwise --timeout 120 --timeout-method thread > gpurun_out/abpw/parity.log 2>&1 || { tail -30 gpurun_out/abpw/parity.log; exit 1; }
tail -1 gpurun_out/abpw/parity.log
L=bpc_baseline_amd/lib/libmvmatch_prev.so,bpc_baseline_amd/lib/libmvmatch.so
timeout -k 10 400 python tools/ab_same_buffers.py --libs $L --workload c3 --buffers 6 --rounds 3 > gpurun_out/abpw/c3.log 2>&1 || { tail -20 gpurun_out/abpw/c3.log; exit 1; }
tail -9 gpurun_out/abpw/c3.log
timeout -k 10 300 python tools/ab_same_buffers.py --libs $L --workload c2 --buffers 4 --rounds ${C2_ROUNDS:-5} > gpurun_out/abpw/c2.log 2>&1 || { tail -20 gpurun_out/abpw/c2.log; exit 1; }
tail -7 gpurun_out/abpw/c2.log
