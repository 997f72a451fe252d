set -o pipefail
for rnd in 1 2 3; do
for lib in bpc_baseline_amd/lib/libmvmatch.so bpc_baseline_amd/lib/libmvmatch_storeonly.so; do
  echo "== $lib"; MVM_LIB_PATH=$lib timeout -k 10 200 python tools/tune_cube.py --variants fused --rounds 3 2>&1 | grep -v amdgpu.ids || exit 1
done; done
for lib in bpc_baseline_amd/lib/libmvmatch.so; do
  echo "== probe"; python - <<'PY'
import torch, sys
sys.path.insert(0,'.')
from bpc_baseline_amd import ops
buf=torch.empty(16_900_000_000//4, dtype=torch.float32, device='cuda')
ops.hbm_write_probe(buf); torch.cuda.synchronize()
e0,e1=torch.cuda.Event(enable_timing=True),torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(5): ops.hbm_write_probe(buf)
e1.record(); torch.cuda.synchronize()
t=e0.elapsed_time(e1)/5
print('probe %.3f ms for 16.9 GB = %.0f GB/s'%(t, 16.9e9/t/1e6))
PY
done
