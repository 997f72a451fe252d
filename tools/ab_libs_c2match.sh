# c2match line A/B over in-tree library builds (lib/ab/NAME.so), alternating
# processes, then the assignment suites under each build.
#   bash tools/ab_libs_c2match.sh "kept pf" [ROUNDS] [TESTS]
set -o pipefail
export TMPDIR=/tmp
for r in $(seq 1 "${2:-3}"); do
  for L in $1; do
    echo -n "$L: "
    MVM_LIB_PATH=bpc_baseline_amd/lib/ab/$L.so RUN=${RUN:-libab}_$L bash tools/ab_c2match.sh default 1 || exit 1
  done
done
for L in $1; do
  MVM_LIB_PATH=bpc_baseline_amd/lib/ab/$L.so timeout -k 10 600 python -u -m pytest ${3:-tests/test_cubefree_gpu.py tests/test_lsap_bmin8_gpu.py} \
    -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/${RUN:-libab}_pytest_$L.log 2>&1 \
    || { tail -20 gpurun_out/${RUN:-libab}_pytest_$L.log; exit 1; }
  echo "$L: $(tail -1 gpurun_out/${RUN:-libab}_pytest_$L.log)"
done
