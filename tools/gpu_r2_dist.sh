# Round 2: the 2-rank real-kernel test + a C3 bench line with the clock sampler.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 500 --timeout-method thread tests/test_distributed.py -m gpu > gpurun_out/r2_dist.log 2>&1 || { tail -40 gpurun_out/r2_dist.log; exit 1; }
tail -8 gpurun_out/r2_dist.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-seconds 0 > gpurun_out/r2_c3.json 2> gpurun_out/r2_c3.err || { tail -20 gpurun_out/r2_c3.err; exit 1; }
cat gpurun_out/r2_c3.json
