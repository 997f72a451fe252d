set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest exit $rc"; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --workload c2cube --cpu-seconds 0 > gpurun_out/bench_c2cube.json 2> gpurun_out/bench_c2cube.err || { tail gpurun_out/bench_c2cube.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_c2cube.json')); print('NEW', d['value'], d['roofline']['achieved'], d['roofline']['avg_launch_ms'])"
MVM_TRIPLET_GENERIC=1 timeout -k 10 400 python bench.py --workload c2cube --cpu-seconds 0 > gpurun_out/bench_c2cube_generic.json 2> gpurun_out/bench_c2cube_g.err || { tail gpurun_out/bench_c2cube_g.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_c2cube_generic.json')); print('GENERIC', d['value'], d['roofline']['achieved'], d['roofline']['avg_launch_ms'])"
