set -o pipefail
mkdir -p gpurun_out/ctr
export TMPDIR=/tmp
rocprofv3 -L > gpurun_out/ctr/counters_list.txt 2>&1 || true
grep -o "SQ_[A-Z0-9_]*\|GRBM_[A-Z0-9_]*\|TA_[A-Z0-9_]*BUSY[A-Z0-9_]*\|TCP_[A-Z0-9_]*" gpurun_out/ctr/counters_list.txt | sort -u > gpurun_out/ctr/names.txt || true
export MVM_PAIRWISE_RPW=16
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU"
P2="GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_WAVES SQ_ACTIVE_INST_LDS"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $P --output-format csv -d gpurun_out/ctr/p$i -o run -- python tools/tune_pairwise.py --rounds 1 --variants 16 > gpurun_out/ctr/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/ctr/p$i.log; }
done
echo done
