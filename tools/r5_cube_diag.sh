# round 5: where the mid-size cube loses its time -- views N,M,P varied one
# at a time (j tiles left part-empty by M, lane shape / alignment by P), each
# ~8 GB per launch on the same buffers as the write probe
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5d; mkdir -p $O
LIB=bpc_baseline_amd/lib/libmvmatch.so
run() {   # name dets opts
  SC=$(python -c "import math;d=[int(x) for x in '$2'.split(',')];print(max(1,int(8e9/(4*math.prod(d)))))")
  timeout -k 10 300 python -u tools/ab_same_buffers.py --libs $LIB --workload cube --dets $2 --scenes $SC --buffers 2 --rounds 2 --opts "$3" > $O/$1.log 2>&1 || { tail -5 $O/$1.log; exit 1; }
  echo "$1 dets=$2 ($SC scenes) $(tail -1 $O/$1.log)"
}
run m100 100,100,100 "default;cube_rows_per_instr=2,cube_cols_per_lane=4"
run m96 100,96,100 "default;cube_rows_per_instr=2,cube_cols_per_lane=4"
run p96 96,96,96 "default;cube_rows_per_instr=2,cube_cols_per_lane=4"
run p112 96,96,112 "default;cube_rows_per_instr=2,cube_cols_per_lane=4"
run p128 96,96,128 "default;cube_rows_per_instr=1,cube_cols_per_lane=3"
run p64 96,96,64 "default;cube_rows_per_instr=2,cube_cols_per_lane=4"
run m68 68,68,68 "default;cube_rows_per_instr=2,cube_cols_per_lane=3"
run m64p68 68,64,68 "default;cube_rows_per_instr=2,cube_cols_per_lane=3"
run m130 130,130,130 "default"
run m128p130 130,128,130 "default"
run p256 96,96,256 "default"
echo done
