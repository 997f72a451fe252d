set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python tools/tune_pairwise.py --rounds 7 --cams 3 --dets 256 --variants 16:1:1:1:1,16:2:1:1:1,16:4:1:1:1,8:2:1:1:1,8:4:1:1:1,8:8:1:1:1,4:4:1:1:1 > gpurun_out/tune_c2.log 2>&1; echo "exit $?"; cat gpurun_out/tune_c2.log
timeout -k 10 300 python tools/tune_pairwise.py --rounds 5 --variants 16:4:1:1:1,16:2:1:1:1,8:8:1:1:1 > gpurun_out/tune_c3.log 2>&1; echo "exit $?"; cat gpurun_out/tune_c3.log
