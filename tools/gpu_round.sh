# smoke + full GPU suite, then the default bench line of each workload
set -o pipefail
mkdir -p gpurun_out/round
bash tools/gpu_check.sh || exit 1
for W in ${WORKLOADS:-c3 c2 c2cube}; do
  timeout -k 10 300 python bench.py --workload $W --cpu-seconds ${CPU_SECONDS:-0} > gpurun_out/round/bench_$W.json 2> gpurun_out/round/bench_$W.err || { tail gpurun_out/round/bench_$W.err; exit 1; }
  python -c "import json,sys;d=json.load(open(sys.argv[1]));r=d['roofline'];print(sys.argv[2],'%.4g'%d['value'],'frac %.3f'%r['frac'],'probe %.0f'%r['write_probe_gbs'],'of-probe %.3f'%r['frac_of_write_probe'],'launch %.3f ms'%r['avg_launch_ms'],d['parity'])" gpurun_out/round/bench_$W.json $W
done
