# round 5: the C2 launch on the bench's twenty fresh 0.8 GB allocations vs a
# buffer just written (first write vs back-to-back repeats), the TLB and
# DRAM write-path counters of the same, the line resident vs ring; then the
# batched pipeline at 100 x 256 and 1000 x 64
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r5k; mkdir -p $O
A="--cams 3 --dets 256 --scenes 1000 --buffers 20 --rounds 3 --repeat 3"
timeout -k 10 300 python -u tools/slot_counters.py $A > $O/c2_slots.log 2>&1 || { tail -5 $O/c2_slots.log; exit 1; }
grep -E "repeat|slowest" $O/c2_slots.log | cut -c1-200
i=0
for P in "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_REQUEST_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum GRBM_GUI_ACTIVE" \
         "TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_STALL_sum TCC_EA0_WRREQ_LEVEL_sum GRBM_UTCL2_BUSY"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $P --output-format csv -d $O/c2_pmc_$i -o run -- python tools/slot_counters.py --cams 3 --dets 256 --scenes 1000 --buffers 20 --rounds 2 --repeat 3 > $O/c2_pmc_$i.log 2>&1 || { echo "pmc $i failed"; tail -5 $O/c2_pmc_$i.log; exit 1; }
done
for mode in resident ring resident ring; do
  timeout -k 10 300 python -u bench.py --workload c2 --steps 20 --warmup 3 --cpu-seconds 0 --parity scene --output $mode > $O/c2_$mode.json 2> $O/c2_$mode.err || { tail -5 $O/c2_$mode.err; exit 1; }
  python tools/summarise_line.py $O/c2_$mode.json | cut -c1-200
done
timeout -k 10 300 python -u tools/bench_pipeline.py --captures 100 --dets 256 --cpu-sample 3 > $O/pipeline_100x256.txt 2>&1 || { tail -5 $O/pipeline_100x256.txt; exit 1; }
tail -4 $O/pipeline_100x256.txt
timeout -k 10 300 python -u tools/bench_pipeline.py --captures 1000 --dets 64 --cpu-sample 10 > $O/pipeline_1000x64.txt 2>&1 || { tail -5 $O/pipeline_1000x64.txt; exit 1; }
tail -4 $O/pipeline_1000x64.txt
