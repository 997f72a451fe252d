# fused cube: transposed 8-row argmin in the fast loop (default build) vs per-row DPP reductions (prev build)
set -o pipefail
mkdir -p gpurun_out/cubered
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_dropin_gpu.py tests/test_batch_match_gpu.py -x -q -m gpu -k "cube or triplet or compute_cost or batch" --timeout 200 --timeout-method thread > gpurun_out/cubered/pytest.log 2>&1; rc=$?; tail -2 gpurun_out/cubered/pytest.log; [ $rc -eq 0 ] || exit $rc
export AB_A=bpc_baseline_amd/lib/libmvmatch_prev.so AB_B=bpc_baseline_amd/lib/libmvmatch.so
AB_CMD='python tools/tune_cube.py --variants fused --rounds 3 --scenes 250 --dets 256' bash tools/ab_lib.sh > gpurun_out/cubered/ab256.log 2>&1 || { tail gpurun_out/cubered/ab256.log; exit 1; }
AB_CMD='python tools/tune_cube.py --variants fused --rounds 3 --scenes 1000 --dets 64' bash tools/ab_lib.sh > gpurun_out/cubered/ab64.log 2>&1 || { tail gpurun_out/cubered/ab64.log; exit 1; }
grep -h -E "==|median" gpurun_out/cubered/ab256.log gpurun_out/cubered/ab64.log
