# the three workload lines (no CPU baseline), compact summary
set -o pipefail
mkdir -p gpurun_out/b3
for W in ${WORKLOADS:-c3 c2 c2cube}; do
  timeout -k 10 300 python bench.py --workload $W --cpu-seconds 0 ${BENCH_ARGS:-} > gpurun_out/b3/$W.json 2> gpurun_out/b3/$W.err || { tail -20 gpurun_out/b3/$W.err; exit 1; }
  python -c "import json,sys;d=json.load(open(sys.argv[1]));r=d['roofline'];print(sys.argv[2],'%.4g'%d['value'],'ms/step %.4f'%d['ms_per_step'],'launch %.4f ms'%r['avg_launch_ms'],'frac %.3f'%r['frac'],'probe %.0f'%r['write_probe_gbs'],'of-probe %.3f'%r['frac_of_write_probe'],'sclk %s'%(d.get('sclk') or {}).get('mean_mhz'),d['parity'][:30])" gpurun_out/b3/$W.json $W
done
