# small-scene cube kernel: division behind a branch (default build) vs if-converted (prev build)
set -o pipefail
mkdir -p gpurun_out/small
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "cube" --timeout 200 --timeout-method thread > gpurun_out/small/pytest.log 2>&1; rc=$?; tail -2 gpurun_out/small/pytest.log; [ $rc -eq 0 ] || exit $rc
export AB_A=bpc_baseline_amd/lib/libmvmatch_prev.so AB_B=bpc_baseline_amd/lib/libmvmatch.so
AB_CMD='python tools/tune_cube.py --variants small --rounds 5 --scenes 1000 --dets 24' bash tools/ab_lib.sh > gpurun_out/small/ab24.log 2>&1 || { tail gpurun_out/small/ab24.log; exit 1; }
AB_CMD='python tools/tune_cube.py --variants small --rounds 5 --scenes 1000 --dets 48' bash tools/ab_lib.sh > gpurun_out/small/ab48.log 2>&1 || { tail gpurun_out/small/ab48.log; exit 1; }
grep -h -E "==|median" gpurun_out/small/ab24.log gpurun_out/small/ab48.log
