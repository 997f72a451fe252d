set -o pipefail
mkdir -p gpurun_out/third2
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "cube" --timeout 200 --timeout-method thread > gpurun_out/third2/pytest.log 2>&1; rc=$?; tail -2 gpurun_out/third2/pytest.log; [ $rc -eq 0 ] || exit $rc
L=bpc_baseline_amd/lib
export AB_LIBS="$L/libmvmatch_chk.so $L/libmvmatch.so $L/libmvmatch_lam.so $L/libmvmatch_lam3.so"
AB_CMD='python tools/tune_cube.py --variants fused --rounds 3 --scenes 250 --dets 256' bash tools/gpu_ab_multi.sh > gpurun_out/third2/ab256.log 2>&1 || { tail gpurun_out/third2/ab256.log; exit 1; }
grep -h -E "==|median" gpurun_out/third2/ab256.log
