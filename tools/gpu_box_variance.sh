# default bench line + write probe on whatever box this call gets (box-to-box spread)
set -o pipefail
mkdir -p gpurun_out/var
tag=$(date +%s)
timeout -k 10 300 python bench.py --cpu-seconds 2 > gpurun_out/var/c3_$tag.json 2>/dev/null || exit 1
timeout -k 10 300 python bench.py --workload c2cube --cpu-seconds 2 > gpurun_out/var/c2cube_$tag.json 2>/dev/null || exit 1
for f in gpurun_out/var/*_$tag.json; do python -c "import json,sys;d=json.load(open(sys.argv[1]));r=d['roofline'];print(sys.argv[1],'%.4g'%d['value'],'launch %.3f ms'%r['avg_launch_ms'],'probe %.0f GB/s'%r['write_probe_gbs'],'frac %.3f'%r['frac'],'of probe %.3f'%r['frac_of_write_probe'])" $f; done
