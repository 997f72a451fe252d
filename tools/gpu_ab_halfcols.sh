# lazy pairwise path with halved columns / row constant (default build) vs per-pair halving (prev build)
set -o pipefail
mkdir -p gpurun_out/halfcols
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_dropin_gpu.py -x -q -m gpu -k "pairwise or epipolar or bench or c3 or c2" --timeout 200 --timeout-method thread > gpurun_out/halfcols/pytest.log 2>&1; rc=$?; tail -2 gpurun_out/halfcols/pytest.log; [ $rc -eq 0 ] || exit $rc
export AB_A=bpc_baseline_amd/lib/libmvmatch_prev.so AB_B=bpc_baseline_amd/lib/libmvmatch.so
AB_CMD='python tools/tune_pairwise.py --rounds 3 --variants 16:4:1:1:1:0:0:2 --scenes 1000 --cams 4 --dets 1024' bash tools/ab_lib.sh > gpurun_out/halfcols/c3.log 2>&1 || { tail gpurun_out/halfcols/c3.log; exit 1; }
AB_CMD='python tools/tune_pairwise.py --rounds 5 --variants 16:4:1:1:1:0:0:2 --scenes 1000 --cams 3 --dets 256' bash tools/ab_lib.sh > gpurun_out/halfcols/c2.log 2>&1 || { tail gpurun_out/halfcols/c2.log; exit 1; }
grep -h -E "==|median" gpurun_out/halfcols/c3.log gpurun_out/halfcols/c2.log
