# round 5: assignment suites, then the c2match line twice and its trace
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_lsap_bmin8_gpu.py tests/test_lsap_gpu.py tests/test_batch_match_gpu.py -x -q --timeout 240 --timeout-method thread > $O/pytest_lsap.log 2>&1 || { tail -15 $O/pytest_lsap.log; exit 1; }
tail -1 $O/pytest_lsap.log
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --workload c2match --steps 5 --warmup 2 > $O/c2match.$r.json 2> $O/c2match.$r.err || { tail -5 $O/c2match.$r.err; exit 1; }
  python -c "import json;d=json.load(open('$O/c2match.$r.json'));print(round(d['value']),{k:round(v,3) for k,v in d['stages_ms'].items() if k!='note'},d['parity'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python bench.py --workload c2match --steps 5 --warmup 2 > $O/c2match_traced.json 2> $O/c2match_traced.err || { tail -5 $O/c2match_traced.err; exit 1; }
find $O/trace -name "*kernel_stats.csv" | head -1 | xargs -I{} sh -c 'cut -d, -f1-5 {} | head -12'
