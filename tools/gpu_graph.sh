# bench.py step as one hipGraph replay vs eager op calls (C2 is a 0.14-ms kernel)
set -o pipefail
mkdir -p gpurun_out/graph
timeout -k 10 300 python -u -m pytest tests/test_distributed.py -x -q -m gpu -k graph --timeout 200 --timeout-method thread > gpurun_out/graph/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/graph/pytest.log; [ $rc -eq 0 ] || exit $rc
show() { python -c "import json,sys;d=json.load(open(sys.argv[1]));r=d['roofline'];print(sys.argv[2],'%.4g'%d['value'],'ms/step %.4f'%d['ms_per_step'],'launch %.4f'%r['avg_launch_ms'],'frac %.3f'%r['frac'],d['parity'])" $1 $2; }
for G in on off; do for ST in 5 50; do
  timeout -k 10 300 python bench.py --workload c2 --cpu-seconds 0 --graph $G --steps $ST > gpurun_out/graph/c2_${G}_$ST.json 2>/dev/null || exit 1
  show gpurun_out/graph/c2_${G}_$ST.json "c2 graph=$G steps=$ST"
done; done
timeout -k 10 300 python bench.py --workload c3 --cpu-seconds 0 > gpurun_out/graph/c3.json 2>/dev/null && show gpurun_out/graph/c3.json "c3 graph=auto"
