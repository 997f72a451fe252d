# round 5: 16-bit 8-row minima + NaN key 0 (assignment suites, c2match line),
# then the cube lane shapes (tools/r5_cube_kpl.sh)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5k; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_lsap_bmin8_gpu.py tests/test_lsap_gpu.py tests/test_batch_match_gpu.py -x -q --timeout 240 --timeout-method thread > $O/pytest_lsap.log 2>&1 || { tail -15 $O/pytest_lsap.log; exit 1; }
tail -2 $O/pytest_lsap.log
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --workload c2match --steps 5 --warmup 2 > $O/c2match.$r.json 2> $O/c2match.$r.err || { tail -5 $O/c2match.$r.err; exit 1; }
  python -c "import json;d=json.load(open('$O/c2match.$r.json'));print(d['value'],d['stages_ms'],d['lsap'].get('stages_ms'),d['parity'])"
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_random_gpu.py -x -q -k "cube" --timeout 240 --timeout-method thread > $O/pytest_cube.log 2>&1 || { tail -15 $O/pytest_cube.log; exit 1; }
tail -2 $O/pytest_cube.log
