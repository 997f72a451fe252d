# Batched capture pipeline timings + kernel breakdown (run via gpurun).
set -o pipefail
mkdir -p gpurun_out/pipeline
export TMPDIR=/tmp
for cfg in ${PIPE_CFGS:-"1000 24" "1000 64" "100 256"}; do
  set -- $cfg
  timeout -k 10 300 python tools/bench_pipeline.py --captures $1 --dets $2 > gpurun_out/pipeline/bench_$1_$2.json 2> gpurun_out/pipeline/bench_$1_$2.err || { echo "bench $1 $2 failed"; tail -20 gpurun_out/pipeline/bench_$1_$2.err; exit 1; }
  cat gpurun_out/pipeline/bench_$1_$2.json
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pipeline/prof -o run -- python tools/bench_pipeline.py --captures 1000 --dets 24 --cpu-sample 1 > gpurun_out/pipeline/prof.log 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/pipeline/prof.log; exit 1; }
find gpurun_out/pipeline/prof -name "*kernel_stats.csv" | head -1 | xargs cut -d, -f1-8 | head -20
