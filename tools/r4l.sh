set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4l; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_random_gpu.py tests/test_dropin_gpu.py tests/test_distributed.py -k "pairwise or dropin or ranks or rccl" -x -q --timeout 120 --timeout-method thread > $O/pytest_pairwise.log 2>&1 || { tail -30 $O/pytest_pairwise.log; exit 1; }
tail -1 $O/pytest_pairwise.log
MVM_LIB_PATH=bpc_baseline_amd/lib/ab/cube_head.so timeout -k 10 300 python -u tools/bench_ragged.py --scenes 500 --rounds 4 --out $O/ragged_before.json > $O/ragged_before.out 2>&1 || { tail -5 $O/ragged_before.out; exit 1; }
tail -12 $O/ragged_before.out
timeout -k 10 300 python -u tools/bench_ragged.py --scenes 500 --rounds 4 --out $O/ragged_after.json > $O/ragged_after.out 2>&1 || { tail -5 $O/ragged_after.out; exit 1; }
tail -12 $O/ragged_after.out
timeout -k 10 400 python -u tools/ab_same_buffers.py --workload c3 --libs bpc_baseline_amd/lib/ab/cube_head.so,bpc_baseline_amd/lib/libmvmatch.so --buffers 6 --rounds 3 > $O/c3_ab.out 2>&1 || { tail -5 $O/c3_ab.out; exit 1; }
tail -8 $O/c3_ab.out
timeout -k 10 300 python -u tools/ab_same_buffers.py --workload c2 --libs bpc_baseline_amd/lib/ab/cube_head.so,bpc_baseline_amd/lib/libmvmatch.so --buffers 4 --rounds 3 > $O/c2_ab.out 2>&1 || { tail -5 $O/c2_ab.out; exit 1; }
tail -6 $O/c2_ab.out
echo done
