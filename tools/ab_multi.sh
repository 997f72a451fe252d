# Interleaved timing of several in-tree builds (AB_LIBS, space separated) with
# AB_CMD, alternating processes, AB_ROUNDS rounds:
#   AB_LIBS='bpc_baseline_amd/lib/libmvmatch_prev.so bpc_baseline_amd/lib/libmvmatch.so' \
#   AB_CMD='python tools/tune_cube.py --variants fused --rounds 3' bash tools/ab_multi.sh
set -o pipefail
mkdir -p gpurun_out
for rnd in $(seq 1 ${AB_ROUNDS:-3}); do
  for lib in $AB_LIBS; do
    echo "== $lib (round $rnd)"
    MVM_LIB_PATH=$lib timeout -k 10 200 $AB_CMD 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
