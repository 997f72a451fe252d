# round 5: cube parity suites (every cube path, the 8-row minima, the random
# sweep), then the A/B of tools/r5_cube_ab.sh
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_random_gpu.py tests/test_lsap_bmin8_gpu.py -x -q -k "cube or bmin8" --timeout 240 --timeout-method thread > $O/pytest_cube.log 2>&1 || { tail -15 $O/pytest_cube.log; exit 1; }
tail -1 $O/pytest_cube.log
bash tools/r5_cube_ab.sh "$@"
