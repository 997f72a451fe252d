# bench lines with resident outputs (default) vs one ring buffer, twice each
set -o pipefail
mkdir -p gpurun_out/resident
for rnd in 1 2; do
  for W in ${WORKLOADS:-c3 c2cube}; do
    for O in resident ring; do
      timeout -k 10 300 python bench.py --workload $W --output $O --cpu-seconds 0 > gpurun_out/resident/${W}_${O}_$rnd.json 2> gpurun_out/resident/${W}_${O}_$rnd.err || { tail gpurun_out/resident/${W}_${O}_$rnd.err; exit 1; }
      python -c "import json,sys;d=json.load(open(sys.argv[1]));r=d['roofline'];c=d['config'];print(sys.argv[2],'%.4g'%d['value'],'frac %.3f'%r['frac'],'probe %.0f'%r['write_probe_gbs'],'of-probe %.3f'%r['frac_of_write_probe'],'launch %.3f ms'%r['avg_launch_ms'],'slots',c['output_allocations'],'%.0f GB'%c['output_gb'],d['parity'])" gpurun_out/resident/${W}_${O}_$rnd.json "$W $O"
    done
  done
done
