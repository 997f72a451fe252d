# Cube builds on the same buffers (results compared across builds), then the
# cube parity suites under the candidate builds.
set -o pipefail
O=gpurun_out/${RUN:-e13row}; mkdir -p $O
LIBS=${LIBS:-kept v1 v2 v3}
L=$(for x in $LIBS; do echo -n "bpc_baseline_amd/lib/ab/$x.so,"; done); L=${L%,}
for D in ${SIZES:-100 110 128 256 200 150 88 70 120}; do
  SC=$(python -c "print(max(1,int(8e9/(4*$D**3))))")
  timeout -k 10 300 python -u tools/ab_same_buffers.py --libs $L --workload cube --dets $D --scenes $SC --buffers 3 --rounds 2 \
    > $O/ab_$D.log 2>&1 || { tail -20 $O/ab_$D.log; exit 1; }
  echo "$D: $(tail -1 $O/ab_$D.log)"
done
for x in ${CHECK:-v2 v3}; do
  MVM_LIB_PATH=bpc_baseline_amd/lib/ab/$x.so timeout -k 10 600 python -u -m pytest tests/test_dropin_gpu.py tests/test_gpu_parity.py \
    tests/test_random_gpu.py tests/test_cubefree_gpu.py tests/test_lsap_bmin8_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread \
    > $O/pytest_$x.log 2>&1 || { tail -20 $O/pytest_$x.log; exit 1; }
  echo "$x: $(tail -1 $O/pytest_$x.log)"
done
