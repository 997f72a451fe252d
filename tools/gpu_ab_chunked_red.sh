# chunked cube: transposed 8-row argmin in the per-chunk fast loop (default build) vs per-row DPP (prev build)
set -o pipefail
mkdir -p gpurun_out/chunkred
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "cube" --timeout 200 --timeout-method thread > gpurun_out/chunkred/pytest.log 2>&1; rc=$?; tail -2 gpurun_out/chunkred/pytest.log; [ $rc -eq 0 ] || exit $rc
export AB_A=bpc_baseline_amd/lib/libmvmatch_prev.so AB_B=bpc_baseline_amd/lib/libmvmatch.so
AB_CMD='python tools/tune_cube.py --variants fused --rounds 3 --scenes 20 --dets 512' bash tools/ab_lib.sh > gpurun_out/chunkred/ab512.log 2>&1 || { tail gpurun_out/chunkred/ab512.log; exit 1; }
AB_CMD='python tools/tune_cube.py --variants fused --rounds 3 --scenes 3 --dets 1024' bash tools/ab_lib.sh > gpurun_out/chunkred/ab1024.log 2>&1 || { tail gpurun_out/chunkred/ab1024.log; exit 1; }
grep -h -E "==|median" gpurun_out/chunkred/ab512.log gpurun_out/chunkred/ab1024.log
