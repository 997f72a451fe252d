# round 5: the 8-row minima from the split forms -- bmin8 + assignment suites,
# cube suites, then the block-minima source A/B by view size
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_lsap_bmin8_gpu.py tests/test_lsap_gpu.py tests/test_batch_match_gpu.py tests/test_gpu_parity.py tests/test_random_gpu.py -x -q -k "bmin8 or lsap or batch or cube or assignment" --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { tail -25 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for spec in 1000:64 1000:100 1000:128 300:150 300:256 2000:48; do
  S=${spec%%:*}; D=${spec#*:}
  echo "== $D x $S"
  timeout -k 10 200 python tools/ab_bmin8_input.py --scenes $S --dets $D 2>&1 | grep -v amdgpu.ids || exit 1
done
