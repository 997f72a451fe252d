"""Assignment timing: GPU LSAP vs scipy on this host, single scene and batched
(device cube -> LSAP).  python tools/bench_lsap.py [--scenes 100 --dets 256]"""
import argparse, os, sys, time
import numpy as np, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scipy.optimize import linear_sum_assignment as scipy_lsa  # noqa: E402
from bpc_baseline_amd import ops  # noqa: E402
from bpc_baseline_amd.synth import make_scenes  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--scenes", type=int, default=100)
ap.add_argument("--dets", type=int, default=256)
args = ap.parse_args()
dev = torch.device("cuda", 0)
n = args.dets
b = make_scenes(args.scenes, 3, n, seed=1)
tp = ops.TripletPlan(b.cam_offs, b.n_scenes, device=dev)
cube, _, _ = ops.triplet_cost_argmin(*(torch.from_numpy(x).to(dev) for x in (b.pts, b.cam_offs, b.F)), tp)
rows = np.full(b.n_scenes, n * n, np.int64)
cols = np.full(b.n_scenes, n, np.int64)
offs = torch.from_numpy(tp.cube_offs_host[:-1].copy()).to(dev)

def gpu_run(k, options=None):
    plan = ops.LsapPlan(rows[:k], cols[:k], device=dev)
    ops.linear_sum_assignment_batched(cube, offs[:k], plan, options=options)        # warm
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    r, c, st = ops.linear_sum_assignment_batched(cube, offs[:k], plan, options=options)
    e1.record()
    torch.cuda.synchronize()
    assert int(st.max()) == 0
    return e0.elapsed_time(e1) * 1e-3, r.cpu().numpy(), c.cpu().numpy()

t1w, _, _ = gpu_run(1, {"lsap_multi_g": -1})   # one workgroup per problem
t1, r1, c1 = gpu_run(1)
host0 = cube[: n * n * n].cpu().numpy().reshape(n * n, n)
ts = time.perf_counter(); r0, c0 = scipy_lsa(host0); ts = time.perf_counter() - ts
assert np.array_equal(r0, r1) and np.array_equal(c0, c1)
tb, rb, cb = gpu_run(b.n_scenes)
# the batch through each class, interleaved: candidate lists (the default for
# long sides > 4096) vs the split register-state kernel (round 3/4 default)
for rnd in range(3):
    for name, opt in (("default", None), ("candidate lists from 1025", {"lsap_sparse_min_cols": 1025}),
                      ("no candidate lists", {"lsap_sparse_min_cols": -1})):
        tt, rr, cc = gpu_run(b.n_scenes, opt)
        assert np.array_equal(rr, rb) and np.array_equal(cc, cb)
        print(f"round {rnd} {name}: {b.n_scenes} x {n}^3 in {tt * 1e3:.2f} ms", flush=True)
# spot-check the last scene of the batch
last = cube[tp.cube_offs_host[-2]:tp.cube_offs_host[-1]].cpu().numpy().reshape(n * n, n)
rl, cl = scipy_lsa(last)
assert np.array_equal(rb[-n:], rl) and np.array_equal(cb[-n:], cl)
print(f"{n}^3 single scene: GPU {t1 * 1e3:.2f} ms (one workgroup: {t1w * 1e3:.2f} ms), scipy {ts * 1e3:.1f} ms on this host "
      f"({ts / t1:.0f}x); batch of {b.n_scenes}: {tb * 1e3:.1f} ms = {b.n_scenes / tb:.0f} scenes/s "
      f"(scipy {1 / ts:.1f} scenes/s on one core)")
