set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5i; mkdir -p $O
for r in 1 2 3; do
  for v in default bm8occ4; do
    if [ $v = default ]; then unset MVM_LIB_PATH; else export MVM_LIB_PATH=bpc_baseline_amd/lib/ab/$v.so; fi
    timeout -k 10 400 python -u bench.py --workload c2match --steps 3 --warmup 1 --cpu-seconds 0 > $O/$v.$r.json 2> $O/$v.$r.err || { tail -5 $O/$v.$r.err; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(sys.argv[2], round(d['value']), round(d['stages_ms']['cube'],3), round(d['stages_ms']['lsap'],3), d['parity'])" $O/$v.$r.json $v
  done
done
