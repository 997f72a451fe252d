set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for W in c2 c2cube; do
  timeout -k 10 400 python bench.py --workload $W --cpu-seconds 8 > gpurun_out/bench_$W.json 2> gpurun_out/bench_$W.err || { echo "bench $W failed"; tail -20 gpurun_out/bench_$W.err; exit 1; }
  cat gpurun_out/bench_$W.json
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c2cube -o run -- python bench.py --workload c2cube --steps 2 --warmup 1 --cpu-seconds 0 > gpurun_out/prof_c2cube.log 2>&1 || { echo "rocprof failed"; exit 1; }
cat gpurun_out/prof_c2cube/run_kernel_stats.csv
