set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python tools/tune_pairwise.py --rounds 6 --variants 16:4:1,16:4:0 > gpurun_out/tune_c3.log 2>&1; echo "exit $?"; tail -2 gpurun_out/tune_c3.log
timeout -k 10 300 python tools/tune_pairwise.py --rounds 6 --cams 3 --dets 256 --variants 16:4:1,16:4:0 > gpurun_out/tune_c2.log 2>&1; echo "exit $?"; tail -2 gpurun_out/tune_c2.log
