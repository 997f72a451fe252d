"""Where does the small-problem LSAP time go?  1000 problems of 576 x 24
(tall: transposed inside the kernel) vs the same problems pre-transposed to
24 x 576 (no in-kernel transpose)."""
import os, sys
import numpy as np, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bpc_baseline_amd import ops  # noqa: E402
from bpc_baseline_amd.synth import make_scenes  # noqa: E402
from oracle import oracle as O  # noqa: E402

dev = torch.device("cuda", 0)
S, n = 1000, 24
b = make_scenes(S, 3, n, seed=1)
cube, *_ = O.cube(b.pts, b.cam_offs, b.F, S)
tall = cube.reshape(S, n * n, n)
wide = np.ascontiguousarray(tall.transpose(0, 2, 1))
res = {}
for name, arr, rows, cols in (("tall 576x24", tall, n * n, n), ("wide 24x576", wide, n, n * n)):
    plan = ops.LsapPlan(np.full(S, rows), np.full(S, cols), device=dev)
    d = torch.from_numpy(arr.reshape(-1).copy()).to(dev)
    offs = torch.arange(S, dtype=torch.int64, device=dev) * (rows * cols)
    for rep in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        r, c, st = ops.linear_sum_assignment_batched(d, offs, plan)
        e1.record()
        torch.cuda.synchronize()
    res[name] = (e0.elapsed_time(e1), r.cpu().numpy(), c.cpu().numpy())
    print(f"{name}: {res[name][0]:.3f} ms")
rt, ct = res["tall 576x24"][1:]
rw, cw = res["wide 24x576"][1:]
# same assignment with the roles swapped (tall output is sorted by its rows)
a = set(zip((np.repeat(np.arange(S), n) * 10**6 + rt).tolist(), ct.tolist()))
b2 = set(zip((np.repeat(np.arange(S), n) * 10**6 + cw).tolist(), rw.tolist()))
assert a == b2
print("same assignments")
