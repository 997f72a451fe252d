# C2 pairwise launch split into its parts (no distances / no association) + the
# write probe at C2's byte count (805 MB) and at 4 GiB
set -o pipefail
mkdir -p gpurun_out/c2parts
W="--scenes 1000 --cams 3 --dets 256"
V="16:4:1:1:1:0:0:2"
timeout -k 10 120 python tools/tune_pairwise.py --rounds 7 --variants $V $W 2>&1 | grep RPW | tee gpurun_out/c2parts/full.log
timeout -k 10 120 python tools/tune_pairwise.py --rounds 7 --variants $V $W --no-dist 2>&1 | grep RPW | tee gpurun_out/c2parts/nodist.log
timeout -k 10 120 python tools/tune_pairwise.py --rounds 7 --variants $V $W --no-argmin 2>&1 | grep RPW | tee gpurun_out/c2parts/noargmin.log
for E in 201270000 1073741824; do
  MVM_PROBE_ELEMS=$E timeout -k 10 60 python tools/probe_write.py one 2>&1 | grep TB | tee -a gpurun_out/c2parts/probe.log
  MVM_PROBE_ELEMS=$E MVM_PROBE_MODE=12 timeout -k 10 60 python tools/probe_write.py one 2>&1 | grep TB | tee -a gpurun_out/c2parts/probe.log
done
