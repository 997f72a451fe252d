# round 4: e13 spread over the workgroup in split cube tiles -- parity, then
# same-buffer timing against the previous prologue at views <= 128
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4s; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_random_gpu.py -k "cube" -x -q --timeout 120 --timeout-method thread > $O/pytest_cube.log 2>&1 || { tail -30 $O/pytest_cube.log; exit 1; }
tail -1 $O/pytest_cube.log
L=bpc_baseline_amd/lib/ab
for spec in "48 18000" "40 26000" "64 7600" "96 2300" "128 950"; do
  set -- $spec
  timeout -k 10 300 python -u tools/ab_same_buffers.py --workload cube --dets $1 --scenes $2 --buffers 3 --rounds 3 --libs $L/nospread.so,$L/spread.so > $O/cube_$1.out 2>&1 || { tail -5 $O/cube_$1.out; exit 1; }
  tail -1 $O/cube_$1.out
done
