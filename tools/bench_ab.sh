# A/B of kernel-path options on the bench line itself, alternating on one box:
#   bash tools/bench_ab.sh WORKLOAD ROUNDS "opts1" "opts2" ...   ("default" = no options)
# (same-buffer A/Bs -- tools/ab_same_buffers.py -- rewrite one buffer back to back,
# which the bench does not; round 4 found them to disagree by 4% on C3 row blocks)
set -o pipefail
export TMPDIR=/tmp
W=$1; R=$2; shift 2
O=gpurun_out/bench_ab_$W; mkdir -p $O
for r in $(seq 1 $R); do
  i=0
  for opt in "$@"; do
    i=$((i+1))
    a=(); [ "$opt" != "default" ] && a=(--options "$opt")
    timeout -k 10 300 python bench.py --workload $W --steps 10 --warmup 3 --cpu-seconds 0 --parity scene "${a[@]}" > $O/v${i}_r$r.json 2> $O/v${i}_r$r.err || { tail -5 $O/v${i}_r$r.err; exit 1; }
    echo "[$opt] $(python tools/summarise_line.py $O/v${i}_r$r.json | cut -c1-150)"
  done
done
