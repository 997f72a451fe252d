# cube tile shapes after the fast-loop changes (in-process interleaved A/B)
set -o pipefail
mkdir -p gpurun_out/tiles
timeout -k 10 300 python tools/tune_cube.py --variants fused,f8x32,f32x32,f16x16 --rounds 4 --scenes 250 --dets 256 2>&1 | grep -v amdgpu.ids | tee gpurun_out/tiles/t256.log
timeout -k 10 300 python tools/tune_cube.py --variants fused,f8x32 --rounds 4 --scenes 1000 --dets 96 2>&1 | grep -v amdgpu.ids | tee gpurun_out/tiles/t96.log
