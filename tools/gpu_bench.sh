# Bench + rocprofv3 kernel-trace summary + PMC (FETCH_SIZE / WRITE_SIZE in separate passes).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
W=${W:-c3}
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -20 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 400 python bench.py --workload $W > gpurun_out/bench_$W.json 2> gpurun_out/bench_$W.err || { echo "bench failed"; tail -20 gpurun_out/bench_$W.err; exit 1; }
cat gpurun_out/bench_$W.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$W -o run -- python bench.py --workload $W --steps 3 --warmup 1 --cpu-seconds 0 > gpurun_out/prof_$W.log 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/prof_$W.log; exit 1; }
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch_$W -o run -- python bench.py --workload $W --steps 1 --warmup 0 --cpu-seconds 0 > gpurun_out/pmc_fetch_$W.log 2>&1 || { echo "pmc fetch failed"; tail -20 gpurun_out/pmc_fetch_$W.log; exit 1; }
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write_$W -o run -- python bench.py --workload $W --steps 1 --warmup 0 --cpu-seconds 0 > gpurun_out/pmc_write_$W.log 2>&1 || { echo "pmc write failed"; tail -20 gpurun_out/pmc_write_$W.log; exit 1; }
echo ok
