# The mid-size cube's j tail: views N x M x P with the same N and P (so the
# same lane shape) and M a multiple of 32 or not, on the same kind of buffers.
set -o pipefail
O=gpurun_out/${RUN:-tail}; mkdir -p $O
for V in ${SIZES:-100,96,100 100,100,100 100,97,100 100,128,100 130,128,130 130,130,130}; do
  SC=$(python -c "n,m,p=map(int,'$V'.split(',')); print(max(1,int(8e9/(4*n*m*p))))")
  timeout -k 10 240 python -u tools/ab_same_buffers.py --libs bpc_baseline_amd/lib/libmvmatch.so --workload cube \
    --dets $V --scenes $SC --buffers 3 --rounds 2 --no-check > $O/tail_$V.log 2>&1 || { tail -20 $O/tail_$V.log; exit 1; }
  python -c "
import sys; n,m,p=map(int,'$V'.split(',')); sc=$SC
pr,k=[float(x) for x in open('$O/tail_$V.log').read().splitlines()[-1].split()[1:3]]
gb=sc*n*m*p*4/1e9
print(f'{n}x{m}x{p} scenes {sc}: kernel {k:.3f} ms {gb/k:.0f} GB/s, probe {pr:.3f} ms on the buffer')"
done
