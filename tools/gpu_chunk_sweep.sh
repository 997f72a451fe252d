# C3 bench at several scenes-per-launch (--chunk), interleaved, one box
set -o pipefail
mkdir -p gpurun_out/chunk
for rnd in 1 2; do
  for c in ${CHUNKS:-1000 2500 5000}; do
    timeout -k 10 240 python bench.py --workload c3 --chunk $c --steps 5 --warmup 2 --cpu-seconds 0 > gpurun_out/chunk/c${c}_r${rnd}.json 2> gpurun_out/chunk/c${c}_r${rnd}.err || { tail -5 gpurun_out/chunk/c${c}_r${rnd}.err; exit 1; }
    python -c "import json,sys;d=json.load(open(sys.argv[1]));r=d['roofline'];print(sys.argv[2],'%.4g pairs/s'%d['value'],'step %.2f ms'%d['ms_per_step'],'launch %.3f ms'%r['avg_launch_ms'],'probe %.0f'%r['write_probe_gbs'],'of-probe %.3f'%r['frac_of_write_probe'])" gpurun_out/chunk/c${c}_r${rnd}.json $c
  done
done
