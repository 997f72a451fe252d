# round 4: GPU suite on the current tree (3-k lane cube, chunked-kernel loads),
# then same-buffer timing of the cube changes and the default C3 line
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4g; mkdir -p $O
RUN=r4g bash tools/gpu.sh check || exit 1
for spec in "48 18000" "96 2300" "160 490" "192 280"; do
  set -- $spec
  timeout -k 10 300 python -u tools/ab_same_buffers.py --workload cube --dets $1 --scenes $2 --buffers 3 --rounds 3 --libs bpc_baseline_amd/lib/libmvmatch.so --opts "default;cube_cols_per_lane=4" > $O/cube_$1.out 2>&1 || { tail -5 $O/cube_$1.out; exit 1; }
  tail -1 $O/cube_$1.out
done
L=bpc_baseline_amd/lib/ab
for spec in "300 100" "512 30"; do
  set -- $spec
  timeout -k 10 300 python -u tools/ab_same_buffers.py --workload cube --dets $1 --scenes $2 --buffers 3 --rounds 3 --libs $L/cube_head.so,$L/cube_new.so > $O/chunked_$1.out 2>&1 || { tail -5 $O/chunked_$1.out; exit 1; }
  tail -1 $O/chunked_$1.out
done
RUN=r4g bash tools/gpu.sh bench c3 || exit 1
echo done
