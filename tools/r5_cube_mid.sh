# round 5: the cube at mid sizes, aligned (P % 32 == 0) vs not -- timing on the
# same buffers, then HBM read / write bytes and L2->DRAM write requests per
# launch (one --pmc pass each)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5l; mkdir -p $O
LIB=bpc_baseline_amd/lib/libmvmatch.so
for N in 128 130 100 96 150 160 48 64; do
  timeout -k 10 200 python -u tools/ab_same_buffers.py --libs $LIB --workload cube --dets $N --buffers 3 --rounds 2 > $O/t_$N.log 2>&1 || { tail -5 $O/t_$N.log; exit 1; }
  echo "N=$N $(grep -E 'mean|probe' $O/t_$N.log | tail -2 | tr '\n' ' ' | cut -c1-200)"
done
for N in 128 130; do
  for P in "FETCH_SIZE" "WRITE_SIZE" "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"; do
    tag=$(echo $P | cut -d' ' -f1)
    timeout -s KILL 200 rocprofv3 --pmc $P --output-format csv -d $O/pmc_${N}_$tag -o run -- python tools/ab_same_buffers.py --libs $LIB --workload cube --dets $N --buffers 2 --rounds 1 > $O/pmc_${N}_$tag.log 2>&1 || { echo "pmc $N $tag failed"; tail -3 $O/pmc_${N}_$tag.log; exit 1; }
  done
done
echo done
