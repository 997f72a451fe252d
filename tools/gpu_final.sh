# end-of-session check: smoke + full GPU suite, default bench line, pipeline timings
set -o pipefail
mkdir -p gpurun_out/final
bash tools/gpu_check.sh || exit 1
timeout -k 10 300 python bench.py > gpurun_out/final/bench_c3.json 2> gpurun_out/final/bench_c3.err || { tail gpurun_out/final/bench_c3.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/final/bench_c3.json'));r=d['roofline'];print('c3 %.4g pairs/s frac %.3f probe %.3f launch %.3f ms'%(d['value'],r['frac'],r['frac_of_write_probe'],r['avg_launch_ms']), d['parity'])"
for cfg in "1000 24" "1000 64" "100 256"; do
  set -- $cfg
  timeout -k 10 300 python tools/bench_pipeline.py --captures $1 --dets $2 --steps 10 --cpu-sample 3 > gpurun_out/final/pipe_$1_$2.json 2> gpurun_out/final/pipe_$1_$2.err || { tail -20 gpurun_out/final/pipe_$1_$2.err; exit 1; }
  python -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[1],'seq %.3f ms'%d['ms_per_batch'],'stream %.3f ms'%d['stream']['ms_per_batch'],'static %.3f ms'%d['static_rig']['ms_per_batch'],d['stage_ms_synchronised'])" gpurun_out/final/pipe_$1_$2.json
done
