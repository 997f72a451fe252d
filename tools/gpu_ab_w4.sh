# A/B: RPW-16 pairwise at 3 vs 4 waves/SIMD (-DMVM_PAIRWISE_WAVES16=4 build), plus RPW 8 in-process
set -o pipefail
mkdir -p gpurun_out/w4
export AB_A=bpc_baseline_amd/lib/libmvmatch.so AB_B=bpc_baseline_amd/lib/libmvmatch_w4.so
AB_CMD='python tools/tune_pairwise.py --rounds 5 --variants 16:4:1:1:1:0:0:2,8:8:1:1:1:0:0:2 --scenes 1000 --cams 3 --dets 256' bash tools/ab_lib.sh > gpurun_out/w4/c2.log 2>&1 || exit 1
AB_CMD='python tools/tune_pairwise.py --rounds 3 --variants 16:4:1:1:1:0:0:2,8:8:1:1:1:0:0:2 --scenes 1000 --cams 4 --dets 1024' bash tools/ab_lib.sh > gpurun_out/w4/c3.log 2>&1 || exit 1
grep -E "==|RPW" gpurun_out/w4/c2.log gpurun_out/w4/c3.log
