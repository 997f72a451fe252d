# A/B of bench.py arguments on the bench line itself, alternating on one box:
#   bash tools/bench_ab_args.sh WORKLOAD ROUNDS "args1" "args2" ...   ("default" = none)
set -o pipefail
export TMPDIR=/tmp
W=$1; R=$2; shift 2
O=gpurun_out/bench_abargs_$W; mkdir -p $O
for r in $(seq 1 $R); do
  i=0
  for a in "$@"; do
    i=$((i+1))
    x=(); [ "$a" != "default" ] && x=($a)
    timeout -k 10 300 python bench.py --workload $W --steps 10 --warmup 3 --cpu-seconds 0 --parity scene "${x[@]}" > $O/v${i}_r$r.json 2> $O/v${i}_r$r.err || { tail -5 $O/v${i}_r$r.err; exit 1; }
    echo "[$a] $(python tools/summarise_line.py $O/v${i}_r$r.json | cut -c1-150)"
  done
done
