# pairwise parity on the new build, then A/B (alternating processes) of libmvmatch_prev.so vs libmvmatch.so at several view sizes
set -o pipefail
mkdir -p gpurun_out/abalign
[ -n "$AB_SKIP_TESTS" ] || timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_dropin_gpu.py tests/test_distributed.py tests/test_batch_match_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/abalign/parity.log 2>&1 || { tail -30 gpurun_out/abalign/parity.log; exit 1; }
tail -2 gpurun_out/abalign/parity.log
for cfg in ${AB_CFGS:-"4 1000 500" "4 992 500" "4 1020 500" "4 1024 500" "4 300 2000" "3 256 1000"}; do
  set -- ${cfg//_/ }
  AB_CMD="python tools/tune_pairwise.py --variants default --rounds 5 --cams $1 --dets $2 --scenes $3" bash tools/ab_lib.sh > gpurun_out/abalign/d$2.log 2>&1 || { tail gpurun_out/abalign/d$2.log; exit 1; }
  echo "cams $1 dets $2 scenes $3"; grep -E "default" gpurun_out/abalign/d$2.log
done
