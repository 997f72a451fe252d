set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4k; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_random_gpu.py tests/test_dropin_gpu.py tests/test_batch_match_gpu.py tests/test_pipeline_gpu.py -k "cube or batch or pipeline or dropin" -x -q --timeout 120 --timeout-method thread > $O/pytest_cube.log 2>&1 || { tail -30 $O/pytest_cube.log; exit 1; }
tail -1 $O/pytest_cube.log
L=bpc_baseline_amd/lib/ab
for spec in "50 13000" "101 1900" "126 1000" "250 130" "254 120" "333 55" "64 7600" "256 120"; do
  set -- $spec
  timeout -k 10 300 python -u tools/ab_same_buffers.py --workload cube --dets $1 --scenes $2 --buffers 3 --rounds 3 --libs $L/cube_head.so,$L/cube_new.so > $O/cube_$1.out 2>&1 || { tail -5 $O/cube_$1.out; exit 1; }
  echo "$1: $(tail -1 $O/cube_$1.out)"
done
echo done
