set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4h; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_random_gpu.py tests/test_dropin_gpu.py tests/test_batch_match_gpu.py tests/test_pipeline_gpu.py -k "cube or batch or pipeline or dropin" -x -q --timeout 120 --timeout-method thread > $O/pytest_cube.log 2>&1 || { tail -30 $O/pytest_cube.log; exit 1; }
tail -1 $O/pytest_cube.log
for spec in "160 490" "150 590" "130 900" "100 2000" "48 18000" "64 7600"; do
  set -- $spec
  timeout -k 10 300 python -u tools/ab_same_buffers.py --workload cube --dets $1 --scenes $2 --buffers 3 --rounds 3 --libs bpc_baseline_amd/lib/libmvmatch.so --opts "default;cube_cols_per_lane=4" > $O/cube_$1.out 2>&1 || { tail -5 $O/cube_$1.out; exit 1; }
  echo "$1: $(tail -1 $O/cube_$1.out)"
done
echo done
