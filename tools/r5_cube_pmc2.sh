# round 5: SQ issue/wait breakdown of the cube kernel at views where the lane
# shapes differ (64: 4 rows x 4 k; 100: 4 x 7 in panels; 96: 2 x 3; 256: full tiles)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5v; mkdir -p $O
LIB=bpc_baseline_amd/lib/libmvmatch.so
for D in 64 100 96 256; do
  SC=$(python -c "print(max(1,int(8e9/(4*$D**3))))")
  U=$((SC*D*D*D))
  i=0
  for P in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU" \
           "SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVES" \
           "GRBM_GUI_ACTIVE GRBM_COUNT"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $O/pmc_${D}_$i -o run -- python tools/ab_same_buffers.py --libs $LIB --workload cube --dets $D --scenes $SC --buffers 1 --rounds 1 > $O/pmc_${D}_$i.log 2>&1 || { echo "pmc $D $i failed"; tail -3 $O/pmc_${D}_$i.log; exit 1; }
    python tools/summarise_sq.py $O/pmc_${D}_$i/run_counter_collection.csv triplet_fused $U --what "$D pass $i" > $O/sum_${D}_$i.json 2>&1 || true
  done
  echo "pmc $D ok"
done
