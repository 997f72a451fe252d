# Small-scene cube variants (run via gpurun): tiled vs one-scene-per-workgroup blocks
set -o pipefail
mkdir -p gpurun_out
for n in 16 24 32 48 64; do
  sc=$(( 250000000 / (n * n * n) ))
  [ $sc -gt 60000 ] && sc=60000
  echo "== n=$n scenes=$sc"
  timeout -k 10 200 python tools/tune_cube.py --scenes $sc --dets $n --rounds 4 --variants tile,small,small4,small8,small32,small64 2>&1 | grep -v amdgpu.ids || exit 1
done
