# round 4: nontemporal cube rows when a wave's rows cover whole 128-byte lines
# (P = 48 at four rows per instruction) -- same-buffer timing against the shipped rule
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4n; mkdir -p $O
L=bpc_baseline_amd/lib/ab
for spec in "48 18000" "56 11000" "64 7600"; do
  set -- $spec
  timeout -k 10 300 python -u tools/ab_same_buffers.py --workload cube --dets $1 --scenes $2 --buffers 3 --rounds 3 --libs $L/base.so,$L/ntw.so > $O/cube_$1.out 2>&1 || { tail -5 $O/cube_$1.out; exit 1; }
  tail -1 $O/cube_$1.out
done
