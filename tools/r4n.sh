# round 4, C3 at 128-row blocks: pairwise/drop-in/distributed parity, then the
# bench line under the kernel trace and the two PMC passes
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4n; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_random_gpu.py tests/test_dropin_gpu.py tests/test_distributed.py -k "pairwise or dropin or ranks or rccl or bench" -x -q --timeout 120 --timeout-method thread > $O/pytest_pairwise.log 2>&1 || { tail -30 $O/pytest_pairwise.log; exit 1; }
tail -1 $O/pytest_pairwise.log
RUN=r4n bash tools/gpu.sh trace c3 || exit 1
RUN=r4n bash tools/gpu.sh pmc c3 || exit 1
echo done
