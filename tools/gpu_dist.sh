# Distributed-path rehearsals on a 1-GPU box: RCCL process group forced at
# world 1 (device-bound group, async chunked gathers, barriers), torchrun at
# world 1, and two gloo ranks sharing the GPU (host-staged gathers).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
MVM_DIST_FORCE=1 timeout -k 10 300 python bench.py --scenes 300 --chunk 150 --steps 2 --warmup 1 --cpu-seconds 0 > gpurun_out/dist_rccl1.json 2> gpurun_out/dist_rccl1.err || { echo "rccl1 failed"; tail -20 gpurun_out/dist_rccl1.err; exit 1; }
cat gpurun_out/dist_rccl1.json
MVM_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --scenes 300 --chunk 150 --steps 2 --warmup 1 > gpurun_out/dist_gloo.json 2> gpurun_out/dist_gloo.err || { echo "gloo failed"; tail -20 gpurun_out/dist_gloo.err; exit 1; }
cat gpurun_out/dist_gloo.json
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 1 --scenes 300 --chunk 150 --steps 2 --warmup 1 --cpu-seconds 0 > gpurun_out/dist_torchrun1.json 2> gpurun_out/dist_torchrun1.err || { echo "torchrun1 failed"; tail -20 gpurun_out/dist_torchrun1.err; exit 1; }
cut -c1-300 gpurun_out/dist_torchrun1.json
