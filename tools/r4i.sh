set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4i; mkdir -p $O
L=bpc_baseline_amd/lib/ab
timeout -k 10 400 python -u tools/ab_same_buffers.py --workload c3 --libs $L/base.so,$L/cheaplines.so,$L/noassoc.so,$L/cheap_noassoc.so,$L/noarith.so,$L/noarith_cheap_noassoc.so --buffers 6 --rounds 3 --no-check > $O/c3_phases.out 2>&1 || { tail -5 $O/c3_phases.out; exit 1; }
tail -8 $O/c3_phases.out
timeout -k 10 400 python -u tools/ab_same_buffers.py --workload c3 --libs bpc_baseline_amd/lib/libmvmatch.so --opts "default;pairwise_row_groups=2;pairwise_row_interleave=-1" --buffers 10 --rounds 3 > $O/c3_rowgroups.out 2>&1 || { tail -5 $O/c3_rowgroups.out; exit 1; }
tail -12 $O/c3_rowgroups.out
echo done
