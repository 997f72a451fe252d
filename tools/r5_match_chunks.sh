# round 5: the c2match line with the step in chunks on two streams
# (assignment of chunk k overlapping the cube of chunk k+1) vs serial
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5x; mkdir -p $O
for C in ${CHUNKS:-1 4 8 2}; do
  timeout -k 10 300 python -u bench.py --workload c2match --steps 5 --warmup 2 --match-chunks $C > $O/c2match_c$C.json 2> $O/c2match_c$C.err || { tail -5 $O/c2match_c$C.err; exit 1; }
  python -c "import json;d=json.load(open('$O/c2match_c$C.json'));print($C, round(d['value']), round(d['ms_per_step'],2), {k:round(v,2) for k,v in d['stages_ms'].items() if k!='note'}, d['parity'])"
done
