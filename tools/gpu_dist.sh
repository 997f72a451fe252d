set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
MVM_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --scenes 300 --chunk 150 --steps 2 --warmup 1 > gpurun_out/dist_gloo.json 2> gpurun_out/dist_gloo.err; echo "gloo exit $?"; cat gpurun_out/dist_gloo.json; tail -3 gpurun_out/dist_gloo.err
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 1 --scenes 300 --chunk 150 --steps 2 --warmup 1 --cpu-seconds 0 > gpurun_out/dist_torchrun1.json 2> gpurun_out/dist_torchrun1.err; echo "torchrun1 exit $?"; cat gpurun_out/dist_torchrun1.json | cut -c1-200
