# fused cube at views <= 64: four rows per wave instruction (fused) vs two (split2) vs the small-scene kernel
set -o pipefail
mkdir -p gpurun_out/split4
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_dropin_gpu.py tests/test_batch_match_gpu.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/split4/pytest.log 2>&1; rc=$?; tail -2 gpurun_out/split4/pytest.log; [ $rc -eq 0 ] || exit $rc
for n in 24 32 40 48 56 64; do
  echo "n=$n"; timeout -k 10 200 python tools/tune_cube.py --variants small,fused,split2 --rounds 4 --scenes 1000 --dets $n 2>&1 | grep -v amdgpu.ids | tee gpurun_out/split4/t$n.log
done
