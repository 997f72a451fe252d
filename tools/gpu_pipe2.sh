# full GPU suite + pipeline timings (plans with one pinned H2D copy)
set -o pipefail
mkdir -p gpurun_out/pipe2
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/pipe2/pytest.log 2>&1; rc=$?; tail -2 gpurun_out/pipe2/pytest.log; [ $rc -eq 0 ] || exit $rc
for cfg in "1000 24" "1000 64"; do
  set -- $cfg
  timeout -k 10 300 python tools/bench_pipeline.py --captures $1 --dets $2 --steps 10 --cpu-sample 5 > gpurun_out/pipe2/bench_$1_$2.json 2> gpurun_out/pipe2/bench_$1_$2.err || { tail -20 gpurun_out/pipe2/bench_$1_$2.err; exit 1; }
  python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[1],'seq %.3f ms'%d['ms_per_batch'],'stream %.3f ms'%d['stream']['ms_per_batch'],'static %.3f ms'%d['static_rig']['ms_per_batch'],d['stage_ms_synchronised'])" gpurun_out/pipe2/bench_$1_$2.json
done
