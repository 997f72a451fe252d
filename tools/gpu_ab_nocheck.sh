set -o pipefail
mkdir -p gpurun_out/nc
export AB_A=bpc_baseline_amd/lib/libmvmatch.so AB_B=bpc_baseline_amd/lib/libmvmatch_nc.so
AB_CMD='python tools/tune_cube.py --variants fused --rounds 5 --scenes 250 --dets 256' bash tools/ab_lib.sh > gpurun_out/nc/ab.log 2>&1 || { tail gpurun_out/nc/ab.log; exit 1; }
grep -vi "warn" gpurun_out/nc/ab.log | tail -20
