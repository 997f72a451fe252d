# round 4: C2 accounting (SQ counters of the phase-variant builds), events
# inside a captured graph, and the C2 line with a reused output buffer
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4d; mkdir -p $O
timeout -k 10 120 python -u tools/probes/graph_events.py > $O/graph_events.log 2>&1 || { tail -5 $O/graph_events.log; exit 1; }
SQ="SQ_INSTS_VALU SQ_WAVES SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_WAVE_CYCLES"
for v in base cheaplines noassoc cheap_noassoc; do
  MVM_LIB_PATH=bpc_baseline_amd/lib/ab/$v.so timeout -s KILL 200 rocprofv3 --pmc $SQ --output-format csv -d $O/sq_$v -o run -- python tools/tune_pairwise.py --cams 3 --dets 256 --rounds 2 > $O/sq_$v.log 2>&1 || { echo "sq $v failed"; tail -5 $O/sq_$v.log; exit 1; }
  python tools/summarise_sq.py $O/sq_$v/run_counter_collection.csv pairwise_lazy_kernel 196608000 --what "C2 $v" --out $O/sq_$v.json > /dev/null || exit 1
done
RUN=r4d bash tools/gpu.sh bench c2 --steps 20 --output ring || exit 1
cp $O/bench_c2.json $O/bench_c2_ring_launch.json
RUN=r4d bash tools/gpu.sh bench c2 --steps 20 --output ring --graph steps || exit 1
cp $O/bench_c2.json $O/bench_c2_ring_steps.json
echo done
