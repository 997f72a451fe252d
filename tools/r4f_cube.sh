# round 4: 3-k lanes in the fused cube kernel -- parity, then same-buffer timing
# against 4-k lanes at the mid sizes; plus the pairwise phase A/B (C3, C2)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4f; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_random_gpu.py tests/test_capi.py -k "cube or capi" -x -q --timeout 120 --timeout-method thread > $O/pytest_cube.log 2>&1 || { tail -30 $O/pytest_cube.log; exit 1; }
tail -2 $O/pytest_cube.log
for spec in "48 18000" "96 2300" "160 490" "192 280" "128 950" "64 7600"; do
  set -- $spec
  timeout -k 10 300 python -u tools/ab_same_buffers.py --workload cube --dets $1 --scenes $2 --buffers 3 --rounds 3 --libs bpc_baseline_amd/lib/libmvmatch.so --opts "default;cube_cols_per_lane=4" > $O/cube_$1.out 2>&1 || { tail -5 $O/cube_$1.out; exit 1; }
  tail -1 $O/cube_$1.out
done
L=bpc_baseline_amd/lib/ab
for spec in "300 100" "512 30" "333 80"; do
  set -- $spec
  timeout -k 10 300 python -u tools/ab_same_buffers.py --workload cube --dets $1 --scenes $2 --buffers 3 --rounds 3 --libs $L/cube_head.so,$L/cube_new.so > $O/chunked_$1.out 2>&1 || { tail -5 $O/chunked_$1.out; exit 1; }
  tail -1 $O/chunked_$1.out
done
timeout -k 10 400 python -u tools/ab_same_buffers.py --workload c3 --libs $L/base.so,$L/cheaplines.so,$L/noassoc.so,$L/cheap_noassoc.so,$L/noarith.so,$L/noarith_cheap_noassoc.so --buffers 6 --rounds 3 --no-check > $O/c3_phases.out 2>&1 || { tail -5 $O/c3_phases.out; exit 1; }
timeout -k 10 300 python -u tools/ab_same_buffers.py --workload c2 --libs $L/base.so,$L/noarith.so,$L/noarith_cheap_noassoc.so --buffers 4 --rounds 3 --no-check > $O/c2_phases.out 2>&1 || { tail -5 $O/c2_phases.out; exit 1; }
echo done
