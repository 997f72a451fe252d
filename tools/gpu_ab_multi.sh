# A/B/C/... of several in-tree builds (AB_LIBS), alternating processes: AB_CMD='...' AB_LIBS='a.so b.so' bash tools/gpu_ab_multi.sh
set -o pipefail
for rnd in 1 2 3; do
  for lib in $AB_LIBS; do
    echo "== $lib (round $rnd)"
    MVM_LIB_PATH=$lib timeout -k 10 200 $AB_CMD 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
