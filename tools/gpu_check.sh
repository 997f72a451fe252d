set -o pipefail
mkdir -p gpurun_out
rocminfo | grep -m3 -i "gfx\|Marketing" > gpurun_out/gpuinfo.txt 2>&1 || true
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && echo SMOKE_OK
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; echo "pytest exit $?"
tail -30 gpurun_out/pytest_gpu.log
