# round 5: cube builds A/B'd on the same buffers, ~8 GB per launch
#   bash tools/r5_cube_ab.sh OUTDIR LIB1,LIB2,... "48 96 100,96,100 ..." [OPTS]
# a size is one view count (N = M = P) or N,M,P
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/$1; mkdir -p $O
for D in $3; do
  SC=$(python -c "import math,os;d=[int(x) for x in '$D'.split(',')];d=d*3 if len(d)==1 else d;print(max(1,int(float(os.environ.get('CUBE_BYTES','8e9'))/(4*math.prod(d)))))")
  timeout -k 10 300 python -u tools/ab_same_buffers.py --libs $2 --workload cube --dets $D --scenes $SC --buffers 3 --rounds 2 --opts "${4:-default}" > $O/ab_$D.log 2>&1 || { tail -5 $O/ab_$D.log; exit 1; }
  echo "$D ($SC scenes): $(tail -1 $O/ab_$D.log)"
done
