# chunked cube (> 256 per view): per-row form (prev) vs per-chunk fast loop (default) vs the same at 3 waves/SIMD
set -o pipefail
mkdir -p gpurun_out/chunked
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "cube" --timeout 200 --timeout-method thread > gpurun_out/chunked/pytest.log 2>&1; rc=$?; tail -2 gpurun_out/chunked/pytest.log; [ $rc -eq 0 ] || exit $rc
L=bpc_baseline_amd/lib
export AB_LIBS="$L/libmvmatch_prev.so $L/libmvmatch.so $L/libmvmatch_lb3.so"
AB_CMD='python tools/tune_cube.py --variants fused --rounds 3 --scenes 20 --dets 512' bash tools/gpu_ab_multi.sh > gpurun_out/chunked/ab512.log 2>&1 || { tail gpurun_out/chunked/ab512.log; exit 1; }
AB_CMD='python tools/tune_cube.py --variants fused --rounds 3 --scenes 40 --dets 384' bash tools/gpu_ab_multi.sh > gpurun_out/chunked/ab384.log 2>&1 || { tail gpurun_out/chunked/ab384.log; exit 1; }
grep -h -E "==|median" gpurun_out/chunked/ab512.log gpurun_out/chunked/ab384.log
