# VALU issue-rate probe + SQ counters of the C2 pairwise launch (tools/probes/valu_rate.hip)
set -o pipefail
mkdir -p gpurun_out/valu
export TMPDIR=/tmp
timeout -k 10 60 ./tools/probes/valu_rate > gpurun_out/valu/rate.log 2>&1 || { echo "probe failed"; cat gpurun_out/valu/rate.log; exit 1; }
cat gpurun_out/valu/rate.log
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU"
P2="GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_WAVES SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_WR"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  for W in "--scenes 1000 --cams 3 --dets 256" "--scenes 1000 --cams 4 --dets 1024"; do
    tag=$(echo $W | tr -d ' -')
    timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d gpurun_out/valu/p${i}_$tag -o run -- python tools/tune_pairwise.py --rounds 1 --variants 16 $W > gpurun_out/valu/p${i}_$tag.log 2>&1 || { echo "pass $i $tag failed"; tail -5 gpurun_out/valu/p${i}_$tag.log; exit 1; }
  done
done
echo done
