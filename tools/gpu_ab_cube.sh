# cube parity on the new build, then A/B (alternating processes) of libmvmatch_prev.so vs libmvmatch.so at several view sizes
set -o pipefail
mkdir -p gpurun_out/abcube
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_pipeline_gpu.py tests/test_batch_match_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/abcube/parity.log 2>&1 || { tail -30 gpurun_out/abcube/parity.log; exit 1; }
tail -2 gpurun_out/abcube/parity.log
for d in 200 128 64 256; do
  AB_CMD="python tools/tune_cube.py --variants fused --rounds 5 --dets $d --scenes $((250*256*256*256/(d*d*d)))" bash tools/ab_lib.sh > gpurun_out/abcube/d$d.log 2>&1 || { tail gpurun_out/abcube/d$d.log; exit 1; }
  echo "dets $d"; grep -E "==|fused" gpurun_out/abcube/d$d.log
done
