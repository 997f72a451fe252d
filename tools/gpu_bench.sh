# Bench lines + rocprofv3 kernel-trace summaries + PMC FETCH/WRITE (separate passes) per workload.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for W in ${WORKLOADS:-c3 c2 c2cube}; do
  timeout -k 10 400 python bench.py --workload $W > gpurun_out/bench_$W.json 2> gpurun_out/bench_$W.err || { echo "bench $W failed"; tail -20 gpurun_out/bench_$W.err; exit 1; }
  cat gpurun_out/bench_$W.json
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$W -o run -- python bench.py --workload $W --steps 3 --warmup 1 --cpu-seconds 0 > gpurun_out/prof_$W.log 2>&1 || { echo "rocprof $W failed"; tail -20 gpurun_out/prof_$W.log; exit 1; }
  timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch_$W -o run -- python bench.py --workload $W --steps 1 --warmup 0 --cpu-seconds 0 > gpurun_out/pmc_fetch_$W.log 2>&1 || { echo "pmc fetch $W failed"; exit 1; }
  timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write_$W -o run -- python bench.py --workload $W --steps 1 --warmup 0 --cpu-seconds 0 > gpurun_out/pmc_write_$W.log 2>&1 || { echo "pmc write $W failed"; exit 1; }
done
echo ok
