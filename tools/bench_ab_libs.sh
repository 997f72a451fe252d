# A/B of library builds on the bench line itself, alternating on one box:
#   bash tools/bench_ab_libs.sh WORKLOAD ROUNDS lib1.so lib2.so ...   ("default" = the in-tree build)
set -o pipefail
export TMPDIR=/tmp
W=$1; R=$2; shift 2
O=gpurun_out/bench_ablib_$W; mkdir -p $O
for r in $(seq 1 $R); do
  i=0
  for lib in "$@"; do
    i=$((i+1))
    if [ "$lib" = "default" ]; then unset MVM_LIB_PATH; else export MVM_LIB_PATH=$lib; fi
    timeout -k 10 300 python bench.py --workload $W --steps 10 --warmup 3 --cpu-seconds 0 --parity scene > $O/v${i}_r$r.json 2> $O/v${i}_r$r.err || { tail -5 $O/v${i}_r$r.err; exit 1; }
    echo "[$(basename $lib)] $(python tools/summarise_line.py $O/v${i}_r$r.json | cut -c1-150)"
  done
done
unset MVM_LIB_PATH
