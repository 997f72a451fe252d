# fused cube, views <= 128: two rows per wave instruction (default) vs one (MVM_TRIPLET_HALF=0)
set -o pipefail
mkdir -p gpurun_out/half
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_dropin_gpu.py tests/test_batch_match_gpu.py -x -q -m gpu -k "cube or triplet or compute_cost or batch" --timeout 200 --timeout-method thread > gpurun_out/half/pytest.log 2>&1; rc=$?; tail -2 gpurun_out/half/pytest.log; [ $rc -eq 0 ] || exit $rc
for n in 96 128 72; do
  timeout -k 10 200 python tools/tune_cube.py --variants fused,nohalf --rounds 4 --scenes 1000 --dets $n 2>&1 | grep -v amdgpu.ids | tee gpurun_out/half/t$n.log
done
