# round 4: what the write fronts change in the L2 -> DRAM write path (C3, eleven
# 25 GB buffers as the bench allocates them): timing, then one PMC pass each with
# one and four fronts per XCD
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4p; mkdir -p $O
P="TCC_EA0_WRREQ_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum TCC_TOO_MANY_EA_WRREQS_STALL_sum TCC_EA0_WRREQ_LEVEL_sum GRBM_GUI_ACTIVE"
for F in 1 4; do
  timeout -k 10 300 python -u tools/slot_counters.py --buffers 11 --rounds 3 --options pairwise_xcd_fronts=$F > $O/slots_f$F.log 2>&1 || { tail -5 $O/slots_f$F.log; exit 1; }
  tail -1 $O/slots_f$F.log | cut -c1-300
done
for F in 1 4; do
  timeout -s KILL 240 rocprofv3 --pmc $P --output-format csv -d $O/pmc_f$F -o run -- python tools/slot_counters.py --buffers 11 --rounds 2 --options pairwise_xcd_fronts=$F > $O/pmc_f$F.log 2>&1 || { echo "pmc F=$F failed"; tail -5 $O/pmc_f$F.log; exit 1; }
  python tools/slot_counters.py --summarise $O/pmc_f$F/run_counter_collection.csv --buffers 11 > $O/pmc_f$F.summary.txt 2>&1 || true
done
echo done
