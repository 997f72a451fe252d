# parity of the pairwise paths + A/B of the lazy argmin reductions (1: per-row DPP, 2: transposed)
set -o pipefail
mkdir -p gpurun_out/lazy2
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k pairwise --timeout 120 --timeout-method thread > gpurun_out/lazy2/pytest.log 2>&1; rc=$?; tail -5 gpurun_out/lazy2/pytest.log; [ $rc -eq 0 ] || exit $rc
V="16:4:1:1:1:0:0:1,16:4:1:1:1:0:0:2"
timeout -k 10 120 python tools/tune_pairwise.py --rounds 7 --variants $V --scenes 1000 --cams 3 --dets 256 2>&1 | tee gpurun_out/lazy2/c2.log
timeout -k 10 200 python tools/tune_pairwise.py --rounds 5 --variants $V --scenes 1000 --cams 4 --dets 1024 2>&1 | tee gpurun_out/lazy2/c3.log
timeout -k 10 120 python tools/tune_pairwise.py --rounds 5 --variants $V --scenes 2000 --cams 4 --dets 512 2>&1 | tee gpurun_out/lazy2/c512.log
