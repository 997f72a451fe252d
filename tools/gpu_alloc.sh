mkdir -p gpurun_out
for a in "--buffers 6" "--buffers 3 --contiguous --first contiguous" "--buffers 3 --pad-gb 30"; do
  echo "## $a"; timeout -k 10 300 python tools/probe_alloc.py $a --rounds 3 2>&1 | grep -v amdgpu.ids || exit 1
done
