# cube: Markstein RN(s/3) + tile-wide fast loop (default build) vs product + third_fast_ok (-DMVM_CUBE_THIRD_CHECK=1 build)
set -o pipefail
mkdir -p gpurun_out/third
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_dropin_gpu.py tests/test_batch_match_gpu.py -x -q -m gpu -k "cube or triplet or compute_cost or batch or stream" --timeout 200 --timeout-method thread > gpurun_out/third/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/third/pytest.log; [ $rc -eq 0 ] || exit $rc
export AB_A=bpc_baseline_amd/lib/libmvmatch_chk.so AB_B=bpc_baseline_amd/lib/libmvmatch.so
AB_CMD='python tools/tune_cube.py --variants fused --rounds 3 --scenes 250 --dets 256' bash tools/ab_lib.sh > gpurun_out/third/ab256.log 2>&1 || { tail gpurun_out/third/ab256.log; exit 1; }
AB_CMD='python tools/tune_cube.py --variants fused --rounds 3 --scenes 20 --dets 512' bash tools/ab_lib.sh > gpurun_out/third/ab512.log 2>&1 || { tail gpurun_out/third/ab512.log; exit 1; }
AB_CMD='python tools/tune_cube.py --variants fused --rounds 3 --scenes 1000 --dets 64' bash tools/ab_lib.sh > gpurun_out/third/ab64.log 2>&1 || { tail gpurun_out/third/ab64.log; exit 1; }
grep -h -E "==|median" gpurun_out/third/ab256.log gpurun_out/third/ab512.log gpurun_out/third/ab64.log
timeout -k 10 300 python bench.py --workload c2cube --cpu-seconds 0 > gpurun_out/third/bench_c2cube.json 2>/dev/null && cat gpurun_out/third/bench_c2cube.json
