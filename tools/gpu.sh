# One runner for every GPU-box task (run it through gpurun).  Chain tasks with &&.
#
#   bash tools/gpu.sh check [pytest args]     smoke + the -m gpu suite (one pytest process)
#   bash tools/gpu.sh bench W [bench args]    one bench.py line of workload W
#   bash tools/gpu.sh trace W [bench args]    the bench line under rocprofv3 --kernel-trace
#                                             --stats (same process), reconciled with
#                                             tools/profile_window.py
#   bash tools/gpu.sh pmc W [bench args]      FETCH_SIZE and WRITE_SIZE, one pass each
#   bash tools/gpu.sh sq "PMC LIST" TOOL [args]  one --pmc pass over a tools/ script
#   bash tools/gpu.sh py TOOL [args]          a tools/ script (or bench.py) under a time limit
#   bash tools/gpu.sh final [W ...]           check, then per workload (default c3 c2 c2cube)
#                                             trace + pmc: the end-of-round evidence
#   bash tools/gpu.sh slots [OPTIONS]         the C3 launch on eleven 25 GB buffers as the
#                                             bench allocates them (tools/slot_counters.py):
#                                             timing, then the TLB and L2->DRAM write-path
#                                             counters, one --pmc pass each
#   bash tools/gpu.sh match [bench args]      the c2match line (cube + assignment + select)
#                                             and its kernel trace
#   bash tools/gpu.sh cubeab LIBS "SIZES" [OPTS]  cube builds / option sets on the same output
#                                             buffers (tools/ab_same_buffers.py), ~CUBE_BYTES
#                                             (8e9) per launch; a size is N or N,M,P
#   bash tools/gpu.sh cubecheck LIBS "SIZES" [OPTS]  the cube parity suites, then cubeab
#   bash tools/gpu.sh lsapcheck               the assignment suites, the c2match line twice
#                                             and its kernel trace
#   bash tools/gpu.sh bm8ab                   the 8-row-minima and assignment suites, then
#                                             the assignment's block-minima source by view
#                                             size (tools/ab_bmin8_input.py)
#   bash tools/gpu.sh cubefree [bench args]  the cube-free association's suites, the
#                                             c2match line without / with the cube, its trace
#   AB_LIBS="a.so b.so" bash tools/gpu.sh ab CMD...
#                                             in-tree library builds (MVM_LIB_PATH) timed by
#                                             CMD in alternating processes, AB_ROUNDS rounds
#                                             (same-buffer A/B in one process:
#                                             tools/ab_same_buffers.py)
#
# Output goes to gpurun_out/$RUN/ (default gpurun_out/run).  Every GPU step has
# its own time limit; a failing step ends the script with its status.
set -o pipefail
export TMPDIR=/tmp
RUN=${RUN:-run}
O=gpurun_out/$RUN
mkdir -p "$O"
LIMIT=${LIMIT:-420}
task=$1; shift || true

fail() { echo "FAIL: $1"; [ -f "$2" ] && tail -n 25 "$2"; exit 1; }

case "$task" in
check)
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 \
    || fail smoke "$O/smoke.log"
  echo SMOKE_OK
  timeout -k 10 1000 python -u -m pytest ${@:-tests} -x -q -m gpu --timeout 300 \
    --timeout-method thread --durations 15 > "$O/pytest_gpu.log" 2>&1
  rc=$?; tail -22 "$O/pytest_gpu.log"; exit $rc ;;
bench)
  W=$1; shift
  timeout -k 10 "$LIMIT" python bench.py --workload "$W" "$@" > "$O/bench_$W.json" \
    2> "$O/bench_$W.err" || fail "bench $W" "$O/bench_$W.err"
  python tools/summarise_line.py "$O/bench_$W.json" ;;
trace)
  W=$1; shift
  timeout -k 10 "$LIMIT" rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace_$W" \
    -o run -- python bench.py --workload "$W" "$@" > "$O/bench_$W.json" 2> "$O/trace_$W.err" \
    || fail "trace $W" "$O/trace_$W.err"
  python tools/summarise_line.py "$O/bench_$W.json" &&
  python tools/profile_window.py "$O/bench_$W.json" "$O/trace_$W/run_kernel_trace.csv" \
    --out "$O/window_$W.json" ;;
pmc)
  W=$1; shift
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 300 rocprofv3 --pmc $C --output-format csv -d "$O/pmc_${C}_$W" -o run -- \
      python bench.py --workload "$W" --steps 1 --warmup 0 --cpu-seconds 0 --c2match off "$@" \
      > "$O/pmc_${C}_$W.log" 2>&1 || fail "pmc $C $W" "$O/pmc_${C}_$W.log"
  done
  echo "pmc $W ok" ;;
sq)
  P=$1; T=$2; shift 2
  N=$(basename "$T" .py)
  timeout -s KILL 200 rocprofv3 --pmc $P --output-format csv -d "$O/sq_$N" -o run -- \
    python "$T" "$@" > "$O/sq_$N.log" 2>&1 || fail "sq $N" "$O/sq_$N.log"
  echo "sq $N ok" ;;
py)
  T=$1; shift
  N=$(basename "$T" .py)
  timeout -k 10 "$LIMIT" python -u "$T" "$@" > "$O/$N.out" 2> "$O/$N.err" \
    || fail "$T" "$O/$N.err"
  tail -40 "$O/$N.out" ;;
final)
  bash "$0" check || exit 1
  for W in ${@:-c3 c2 c2cube}; do
    bash "$0" trace "$W" || exit 1
    bash "$0" pmc "$W" || exit 1
  done
  bash "$0" trace c2match || echo "c2match trace: see $O/trace_c2match.err"
  echo final ok ;;
slots)
  OPT=${1:+--options $1}
  timeout -k 10 300 python -u tools/slot_counters.py --buffers 11 --rounds 3 $OPT > "$O/slots.log" 2>&1 \
    || fail slots "$O/slots.log"
  i=0
  for P in "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum" \
           "TCC_EA0_WRREQ_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum TCC_TOO_MANY_EA_WRREQS_STALL_sum TCC_EA0_WRREQ_LEVEL_sum" \
           "GRBM_UTCL2_BUSY GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    timeout -s KILL 240 rocprofv3 --pmc $P --output-format csv -d "$O/slots_pmc_$i" -o run -- \
      python tools/slot_counters.py --buffers 11 --rounds 2 $OPT > "$O/slots_pmc_$i.log" 2>&1 \
      || fail "slots pmc $i" "$O/slots_pmc_$i.log"
    python tools/slot_counters.py --summarise "$O/slots_pmc_$i/run_counter_collection.csv" --buffers 11 \
      > "$O/slots_pmc_$i.summary.txt" 2>&1 || true
  done
  echo slots ok ;;
match)
  timeout -k 10 "$LIMIT" python -u bench.py --workload c2match "$@" > "$O/bench_c2match.json" \
    2> "$O/bench_c2match.err" || fail "bench c2match" "$O/bench_c2match.err"
  # last: the profiler's teardown has crashed after writing its files
  timeout -k 10 "$LIMIT" rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace_c2match" \
    -o run -- python -u bench.py --workload c2match --cpu-seconds 0 "$@" > "$O/trace_c2match.json" \
    2> "$O/trace_c2match.err"
  rc=$?; echo "match trace rc=$rc (run it last: nothing after a crashed process)"; exit $rc ;;
cubeab)
  for D in $2; do
    SC=$(python -c "import math,os;d=[int(x) for x in '$D'.split(',')];d=d*3 if len(d)==1 else d;print(max(1,int(float(os.environ.get('CUBE_BYTES','8e9'))/(4*math.prod(d)))))")
    timeout -k 10 300 python -u tools/ab_same_buffers.py --libs "$1" --workload cube --dets "$D" \
      --scenes "$SC" --buffers 3 --rounds 2 --opts "${3:-default}" > "$O/ab_$D.log" 2>&1 \
      || fail "cubeab $D" "$O/ab_$D.log"
    echo "$D ($SC scenes): $(tail -1 "$O/ab_$D.log")"
  done ;;
cubecheck)
  timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_random_gpu.py \
    tests/test_lsap_bmin8_gpu.py -x -q -k "cube or bmin8" --timeout 240 --timeout-method thread \
    > "$O/pytest_cube.log" 2>&1 || fail "cube suites" "$O/pytest_cube.log"
  tail -1 "$O/pytest_cube.log"
  bash "$0" cubeab "$@" ;;
lsapcheck)
  timeout -k 10 600 python -u -m pytest tests/test_lsap_bmin8_gpu.py tests/test_lsap_gpu.py \
    tests/test_batch_match_gpu.py -x -q --timeout 240 --timeout-method thread \
    > "$O/pytest_lsap.log" 2>&1 || fail "assignment suites" "$O/pytest_lsap.log"
  tail -1 "$O/pytest_lsap.log"
  bash "$0" match ;;
bm8ab)
  timeout -k 10 600 python -u -m pytest tests/test_lsap_bmin8_gpu.py tests/test_lsap_gpu.py \
    tests/test_batch_match_gpu.py -x -q --timeout 240 --timeout-method thread \
    > "$O/pytest_bm8.log" 2>&1 || fail "bmin8 suites" "$O/pytest_bm8.log"
  tail -1 "$O/pytest_bm8.log"
  for spec in 1000:64 1000:100 1000:128 300:150 300:256 2000:48; do
    echo "== ${spec#*:} x ${spec%%:*}"
    timeout -k 10 200 python tools/ab_bmin8_input.py --scenes "${spec%%:*}" --dets "${spec#*:}" \
      > "$O/bm8ab_${spec#*:}.log" 2>&1 || fail "bm8ab $spec" "$O/bm8ab_${spec#*:}.log"
    grep -E "minima|itself" "$O/bm8ab_${spec#*:}.log"
  done ;;
cubefree)
  # the cube-free association (ABI 7): its suite and the assignment / pipeline
  # suites, then the c2match line without and with the cube, and its trace
  timeout -k 10 900 python -u -m pytest tests/test_cubefree_gpu.py tests/test_lsap_bmin8_gpu.py \
    tests/test_lsap_gpu.py tests/test_batch_match_gpu.py -x -q --timeout 240 --timeout-method thread \
    > "$O/pytest_cubefree.log" 2>&1 || fail "cube-free suites" "$O/pytest_cubefree.log"
  tail -1 "$O/pytest_cubefree.log"
  for M in free keep free keep; do
    timeout -k 10 "$LIMIT" python -u bench.py --workload c2match --cube $M --cpu-seconds 0 "$@" \
      >> "$O/bench_c2match_$M.json" 2>> "$O/bench_c2match_$M.err" || fail "c2match $M" "$O/bench_c2match_$M.err"
    python tools/summarise_line.py <(tail -1 "$O/bench_c2match_$M.json")
  done
  timeout -k 10 "$LIMIT" rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace_c2match_free" \
    -o run -- python -u bench.py --workload c2match --cube free --cpu-seconds 0 "$@" \
    > "$O/trace_c2match_free.json" 2> "$O/trace_c2match_free.err"
  rc=$?; echo "cubefree trace rc=$rc"; exit $rc ;;
cfab)
  # the cube-free chain's options A/B on the c2match line (alternating), then
  # one SQ counter pass over it
  timeout -k 10 600 python -u -m pytest tests/test_cubefree_gpu.py -x -q --timeout 240 \
    --timeout-method thread > "$O/pytest_cfab.log" 2>&1 || fail "cube-free suite" "$O/pytest_cfab.log"
  tail -1 "$O/pytest_cfab.log"
  for rnd in 1 2; do
    for V in ${CF_VARIANTS:-default cube_tile_rows=32}; do
      OPT=""; [ "$V" != default ] && OPT="--options $V"
      timeout -k 10 "$LIMIT" python -u bench.py --workload c2match --cube free --cpu-seconds 0 $OPT "$@" \
        > "$O/cf_${V}_$rnd.json" 2> "$O/cf_${V}_$rnd.err" || fail "c2match $V" "$O/cf_${V}_$rnd.err"
      echo "== $V round $rnd"; python tools/summarise_line.py "$O/cf_${V}_$rnd.json" | tail -1
    done
  done
  for C in ${CF_CHUNKS:-2 4}; do
    timeout -k 10 "$LIMIT" python -u bench.py --workload c2match --cube free --cpu-seconds 0 --match-chunks $C "$@" \
      > "$O/cf_chunks$C.json" 2> "$O/cf_chunks$C.err" || fail "c2match chunks $C" "$O/cf_chunks$C.err"
    echo "== $C chunks"; python tools/summarise_line.py "$O/cf_chunks$C.json"
  done
  timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY \
    SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_LDS --output-format csv -d "$O/sq_cf" -o run -- \
    python bench.py --workload c2match --cube free --steps 2 --warmup 1 --cpu-seconds 0 > "$O/sq_cf.log" 2>&1 \
    || fail "sq c2match" "$O/sq_cf.log"
  for K in triplet_minima sp_solve sp_lists sp_bmin8_reduce; do
    python tools/summarise_sq.py "$O/sq_cf/run_counter_collection.csv" $K 16777216000 --what "c2match free $K" \
      --out "$O/sq_cf_$K.json" | grep -E "valu_|wait_over|SQ_" | tr -d '\n'; echo
  done ;;
cubepin)
  # the mid-size cube, kept build against the store-only
  # diagnostic (tools/diag/cube_storeonly.patch) on the same buffers, then
  # SQ and L2->DRAM write-path counters per build at the sizes named
  K=bpc_baseline_amd/lib/ab/kept.so; SO=bpc_baseline_amd/lib/ab/cube_storeonly.so
  for D in ${CP_SIZES:-100 130 150 256}; do
    SC=$(python -c "print(max(1,int(8e9/(4*$D**3))))")
    timeout -k 10 300 python -u tools/ab_same_buffers.py --libs "$K,$SO" --workload cube --dets "$D" \
      --scenes "$SC" --buffers 3 --rounds 2 --no-check > "$O/pin_ab_$D.log" 2>&1 || fail "pin ab $D" "$O/pin_ab_$D.log"
    echo "$D^3 ($SC scenes): $(tail -1 "$O/pin_ab_$D.log")"
  done
  for D in ${CP_PMC_SIZES:-100 130}; do
    SC=$(python -c "print(max(1,int(8e9/(4*$D**3))))")
    for L in kept cube_storeonly; do
      i=0
      for PM in "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT" \
                "TCC_EA0_WRREQ_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum TCC_TOO_MANY_EA_WRREQS_STALL_sum TCC_EA0_WRREQ_LEVEL_sum" \
                "SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"; do
        i=$((i+1))
        timeout -s KILL 150 rocprofv3 --pmc $PM --output-format csv -d "$O/pin_pmc_${L}_${D}_$i" -o run -- \
          python tools/ab_same_buffers.py --libs "bpc_baseline_amd/lib/ab/$L.so" --workload cube --dets "$D" \
          --scenes "$SC" --buffers 1 --rounds 1 --no-check > "$O/pin_pmc_${L}_${D}_$i.log" 2>&1 \
          || fail "pin pmc $L $D $i" "$O/pin_pmc_${L}_${D}_$i.log"
        python tools/summarise_sq.py "$O/pin_pmc_${L}_${D}_$i/run_counter_collection.csv" triplet_ \
          $((SC * D * D * D)) --what "$L $D^3 pass $i" --out "$O/pin_pmc_${L}_${D}_$i.json" > /dev/null
      done
      echo "pmc $L $D^3 ok"
    done
  done ;;
ab)
  for rnd in $(seq 1 "${AB_ROUNDS:-3}"); do
    for lib in $AB_LIBS; do
      echo "== $lib (round $rnd)"
      MVM_LIB_PATH=$lib timeout -k 10 200 "$@" 2>&1 | grep -v amdgpu.ids || exit 1
    done
  done ;;
*)
  echo "unknown task '$task'"; exit 2 ;;
esac
