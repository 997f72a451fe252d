set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r4j; mkdir -p $O
timeout -k 10 500 python -u tools/ab_same_buffers.py --workload c3 --libs bpc_baseline_amd/lib/libmvmatch.so --opts "default;pairwise_row_groups=2;pairwise_row_groups=2,pairwise_row_interleave=-1" --buffers 11 --rounds 4 > $O/c3_rowgroups11.out 2>&1 || { tail -5 $O/c3_rowgroups11.out; exit 1; }
tail -14 $O/c3_rowgroups11.out
echo done
