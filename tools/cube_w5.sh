# 2 x 4 split form at five waves per SIMD (w5) against the kept build, at
# views where the default is the 4 x 7 form; same buffers, results compared.
set -o pipefail
O=gpurun_out/${RUN:-w5}; mkdir -p $O
for D in ${SIZES:-100 110 120 128 104}; do
  SC=$(python -c "print(max(1,int(8e9/(4*$D**3))))")
  timeout -k 10 300 python -u tools/ab_same_buffers.py --libs bpc_baseline_amd/lib/ab/kept.so,bpc_baseline_amd/lib/ab/w5.so \
    --opts "default;cube_rows_per_instr=2,cube_cols_per_lane=4" --workload cube --dets $D --scenes $SC --buffers 3 --rounds 2 \
    > $O/w5_$D.log 2>&1 || { tail -20 $O/w5_$D.log; exit 1; }
  echo "$D: $(grep -A1 '^buffer' $O/w5_$D.log | head -1)"; echo "$D: $(tail -1 $O/w5_$D.log)"
done
