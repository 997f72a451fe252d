# round 4 final tree: smoke + GPU suite, then per workload the bench line under
# rocprofv3 --kernel-trace --stats (same process, reconciled by
# tools/profile_window.py) and the FETCH_SIZE / WRITE_SIZE passes
set -o pipefail
export TMPDIR=/tmp
R=${RUN:-r4final}
RUN=$R bash tools/gpu.sh check || exit 1
for W in c3 c2 c2cube; do
  RUN=$R bash tools/gpu.sh trace $W || exit 1
  RUN=$R bash tools/gpu.sh pmc $W || exit 1
done
echo done
