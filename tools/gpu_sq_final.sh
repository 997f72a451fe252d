# SQ instruction counters of the final kernels: C3 / C2 pairwise launches and the 256^3 cube
set -o pipefail
mkdir -p gpurun_out/sqf
export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES"
i=0
for W in "tune_pairwise.py --variants default --scenes 1000 --cams 4 --dets 1024" "tune_pairwise.py --variants default --scenes 1000 --cams 3 --dets 256" "tune_cube.py --variants fused --scenes 250 --dets 256"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $P1 --output-format csv -d gpurun_out/sqf/w$i -o run -- python tools/$W --rounds 1 > gpurun_out/sqf/w$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/sqf/w$i.log; exit 1; }
done
echo done
