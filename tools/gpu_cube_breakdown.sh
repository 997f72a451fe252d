set -o pipefail
mkdir -p gpurun_out/cube2
export TMPDIR=/tmp
AB_LIBS='bpc_baseline_amd/lib/libmvmatch_prev.so bpc_baseline_amd/lib/libmvmatch_cur.so bpc_baseline_amd/lib/libmvmatch_nostore.so' AB_CMD='python tools/tune_cube.py --variants fused --rounds 3' bash tools/ab_multi.sh > gpurun_out/cube2/ab.log 2>&1 || { tail -20 gpurun_out/cube2/ab.log; exit 1; }
cat gpurun_out/cube2/ab.log
timeout -k 10 300 python bench.py --workload c2cube --steps 5 --cpu-seconds 0 > gpurun_out/cube2/bench.json 2> gpurun_out/cube2/bench.err || { tail gpurun_out/cube2/bench.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/cube2/bench.json'));r=d['roofline'];print('c2cube %.4g triples/s frac %.3f probe %.0f GB/s of-probe %.3f launch %.3f ms'%(d['value'],r['frac'],r['write_probe_gbs'],r['frac_of_write_probe'],r['avg_launch_ms']), d['parity'])"
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES"
timeout -s KILL 150 rocprofv3 --pmc $P1 --output-format csv -d gpurun_out/cube2/sq -o run -- python tools/tune_cube.py --variants fused --rounds 1 > gpurun_out/cube2/sq.log 2>&1 || { echo "sq failed"; tail -5 gpurun_out/cube2/sq.log; exit 1; }
echo ok
