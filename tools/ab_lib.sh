# A/B of two in-tree builds (MVM_LIB_PATH), alternating processes:
#   AB_CMD='python tools/tune_cube.py --variants fused --rounds 3' bash tools/ab_lib.sh
set -o pipefail
mkdir -p gpurun_out
A=${AB_A:-bpc_baseline_amd/lib/libmvmatch_prev.so}
B=${AB_B:-bpc_baseline_amd/lib/libmvmatch.so}
for rnd in 1 2 3; do
  for lib in "$A" "$B"; do
    echo "== $lib (round $rnd)"
    MVM_LIB_PATH=$lib timeout -k 10 200 $AB_CMD 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
