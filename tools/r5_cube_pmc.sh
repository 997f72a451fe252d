# round 5: counters of the cube kernel at views where the same tile shape runs
# at different fractions of the write probe (96x96x256 vs 256^3: the same
# 16 x 32 x 256 tiles), one --pmc pass per counter group
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5p; mkdir -p $O
LIB=bpc_baseline_amd/lib/libmvmatch.so
sc() { python -c "import math;d=[int(x) for x in '$1'.split(',')];print(max(1,int(8e9/(4*math.prod(d)))))"; }
for D in 96,96,256 256,256,256 256,96,256 96,256,256 96,96,96 96,96,128; do
  SC=$(sc $D)
  timeout -k 10 300 python -u tools/ab_same_buffers.py --libs $LIB --workload cube --dets $D --scenes $SC --buffers 2 --rounds 2 > $O/t_$D.log 2>&1 || { tail -5 $O/t_$D.log; exit 1; }
  echo "time $D ($SC scenes): $(tail -1 $O/t_$D.log)"
done
for D in 96,96,256 256,256,256 256,96,256 96,96,96 96,96,128; do
  SC=$(sc $D)
  U=$(python -c "import math;print($SC*math.prod([int(x) for x in '$D'.split(',')]))")
  i=0
  for P in "SQ_WAVES SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVE_CYCLES" \
           "TCC_EA0_WRREQ_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum TCC_TOO_MANY_EA_WRREQS_STALL_sum TCC_EA0_WRREQ_LEVEL_sum" \
           "GRBM_GUI_ACTIVE TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $O/pmc_${D}_$i -o run -- python tools/ab_same_buffers.py --libs $LIB --workload cube --dets $D --scenes $SC --buffers 1 --rounds 1 > $O/pmc_${D}_$i.log 2>&1 || { echo "pmc $D $i failed"; tail -3 $O/pmc_${D}_$i.log; exit 1; }
    python tools/summarise_sq.py $O/pmc_${D}_$i/run_counter_collection.csv triplet_fused $U --what "$D pass $i" > $O/sum_${D}_$i.json 2>&1 || true
  done
  echo "pmc $D ok"
done
echo done
