# small-scene cube kernel vs the two-rows-per-wave fused kernel around the 64 threshold
set -o pipefail
mkdir -p gpurun_out/svh
for n in 32 40 48 56 63; do
  echo "n=$n"; timeout -k 10 200 python tools/tune_cube.py --variants small,fused --rounds 4 --scenes 1000 --dets $n 2>&1 | grep -v amdgpu.ids | tee gpurun_out/svh/t$n.log
done
