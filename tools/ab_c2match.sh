# c2match line A/B over kernel option sets, interleaved in alternating processes.
#   bash tools/ab_c2match.sh "default;lsap_sparse_blocks=8" [ROUNDS]
# A set is `default` or bench.py --options FIELD=VALUE,... (include/mvmatch.h);
# MVM_LIB_PATH picks the library build for every set.  Prints per run:
# set, captures/s, cube ms, assignment ms, parity.  Output: gpurun_out/$RUN/.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${RUN:-c2ab}; mkdir -p "$O"
IFS=';' read -r -a SETS <<< "${1:-default}"
for r in $(seq 1 "${2:-2}"); do
  for v in "${SETS[@]}"; do
    tag=$(echo "$v" | tr ',=' '_-')
    opt=(); [ "$v" != default ] && opt=(--options "$v")
    timeout -k 10 400 python -u bench.py --workload c2match --steps 3 --warmup 1 --cpu-seconds 0 "${opt[@]}" \
      > "$O/$tag.$r.json" 2> "$O/$tag.$r.err" || { tail -5 "$O/$tag.$r.err"; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(sys.argv[2], round(d['value']), round(d['stages_ms'].get('cube', d['stages_ms'].get('minima', 0)),3), round(d['stages_ms']['lsap'],3), d['parity'])" "$O/$tag.$r.json" "$v"
  done
done
