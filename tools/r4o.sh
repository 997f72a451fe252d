# round 4: the C3 bench line itself with 256- vs 128-row blocks on ONE box,
# alternating (MVM_LIB_PATH selects the 256-row build)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4o; mkdir -p $O
for r in 1 2; do
  MVM_LIB_PATH=bpc_baseline_amd/lib/ab/rg4.so timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-seconds 0 --parity scene > $O/rg4_$r.json 2> $O/rg4_$r.err || { tail -5 $O/rg4_$r.err; exit 1; }
  python tools/summarise_line.py $O/rg4_$r.json | sed "s/^/rg4 /"
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-seconds 0 --parity scene > $O/rg2_$r.json 2> $O/rg2_$r.err || { tail -5 $O/rg2_$r.err; exit 1; }
  python tools/summarise_line.py $O/rg2_$r.json | sed "s/^/rg2 /"
done
echo done
