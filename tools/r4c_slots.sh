set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4c; mkdir -p $O
RUN=r4c bash tools/gpu.sh bench c2 --steps 20 || exit 1
timeout -k 10 300 python -u tools/slot_counters.py --buffers 11 --rounds 3 > $O/slots_plain.log 2>&1 || exit 1
P1="TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_STALL_UTCL2_REQ_OUT_OF_CREDITS_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum"
P2="TCC_EA0_WRREQ_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum TCC_TOO_MANY_EA_WRREQS_STALL_sum TCC_EA0_WRREQ_LEVEL_sum"
P3="TCP_UTCL1_TRANSLATION_MISS_UNDER_MISS_sum TCP_UTCL1_STALL_MULTI_MISS_sum TCP_UTCL1_THRASHING_STALL_sum TCP_UTCL1_REQUEST_sum GRBM_UTCL2_BUSY GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $P --output-format csv -d $O/pmc_$i -o run -- python tools/slot_counters.py --buffers 11 --rounds 2 > $O/pmc_$i.log 2>&1 || { echo "pmc pass $i failed"; tail -5 $O/pmc_$i.log; exit 1; }
  python tools/slot_counters.py --summarise $O/pmc_$i/run_counter_collection.csv --buffers 11 > $O/pmc_$i.summary.txt 2>&1 || true
done
echo done
