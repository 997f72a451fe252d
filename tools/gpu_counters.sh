set -o pipefail
mkdir -p gpurun_out/ctr2
export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU"
P2="GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_WAVES SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_WR"
P3="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $P --output-format csv -d gpurun_out/ctr2/p$i -o run -- python tools/tune_cube.py --rounds 1 --variants rpw4 > gpurun_out/ctr2/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/ctr2/p$i.log; }
done
echo done
