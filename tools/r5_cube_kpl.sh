# round 5: 5-8 k per lane in the split cube forms -- parity on every cube
# suite, then same-buffer timing of the new default lane shape against the
# round-4 shape (forced) at the sizes where they differ, and tiles of 32 i
# rows, ~8 GB per launch
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5m; mkdir -p $O
[ -n "$SKIP_PYTEST" ] || timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_random_gpu.py tests/test_lsap_bmin8_gpu.py -x -q -k "cube or bmin8" --timeout 240 --timeout-method thread > $O/pytest_cube.log 2>&1 || { tail -15 $O/pytest_cube.log; exit 1; }
[ -n "$SKIP_PYTEST" ] || tail -2 $O/pytest_cube.log
LIB=bpc_baseline_amd/lib/libmvmatch.so
# size : the round-4 shape (rows per instruction, k per lane)
for spec in 48:4:3 100:2:4 130:1:3 150:1:3 64:4:4 96:2:3 68:2:3 200:1:4 140:1:3 110:2:4; do
  N=${spec%%:*}; rest=${spec#*:}; R=${rest%%:*}; K=${rest#*:}
  SC=$(python -c "print(max(1, int(8e9 / (4 * $N ** 3))))")
  timeout -k 10 300 python -u tools/ab_same_buffers.py --libs $LIB --workload cube --dets $N --scenes $SC --buffers 3 --rounds 2 --opts "default;cube_rows_per_instr=$R,cube_cols_per_lane=$K;cube_tile_rows=32" > $O/ab_$N.log 2>&1 || { tail -5 $O/ab_$N.log; exit 1; }
  echo "N=$N ($SC scenes) $(tail -1 $O/ab_$N.log)"
done
