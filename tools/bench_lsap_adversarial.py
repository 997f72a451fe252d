"""The candidate-list assignment on adversarial C2-sized batches (VERDICT r5
item 4): timing, the solver's dense fallbacks, and exactness against scipy.

    python tools/bench_lsap_adversarial.py [--scenes 1000 --dets 256 --reps 3]

Cases (1,000 captures x 3 x 256 detections unless --scenes/--dets say
otherwise; the generator is bpc_baseline_amd.synth.make_scenes):
  default     the bench's generator (half true objects, half clutter)
  dup10/dup30 10% / 30% of every view's detections replaced by exact copies of
              other detections of the same view (duplicated detections: equal
              cost rows and columns)
  clutter     every detection uniform in the image (no true correspondences)
  objects     every detection a projection of a shared object (low costs
              everywhere: many near-equal candidates per row)
  quant1/quant8  the default cube with every cost rounded down to a multiple
              of 1 / 8 px (blocks of exactly equal costs)
The cube-free chain (triplet_minima -> linear_sum_assignment_resid; block
minima only unless --bmin8) runs the first five, the cube form (the quantised cube and its 8-row minima ->
linear_sum_assignment_batched) the last two.  Per case: the assignment's ms
(HIP events, best and median of --reps), and the solver's counters per batch
(ops.lsap_sparse_stats: dense free-minimum scans, dense tie scans, overflowed
lists, Dijkstra steps); two scenes are compared with scipy on the same costs.
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scipy.optimize import linear_sum_assignment as scipy_lsa  # noqa: E402

from bpc_baseline_amd import ops  # noqa: E402
from bpc_baseline_amd.synth import IMAGE_SIZE, make_scenes  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--scenes", type=int, default=1000)
ap.add_argument("--dets", type=int, default=256)
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--cases", default="default,dup10,dup30,clutter,objects,quant1,quant8")
ap.add_argument("--json", default=None, help="also write the table here")
ap.add_argument("--bmin8", action="store_true",
                help="cube-free cases with the 8-row minima (default: block minima only, "
                     "what match_captures runs)")
args = ap.parse_args()
dev = torch.device("cuda", 0)
S, n = args.scenes, args.dets
rng = np.random.default_rng(12345)


def batch_for(case):
    b = make_scenes(S, 3, n, seed=1)
    pts = b.pts.copy()
    co = b.cam_offs
    if case.startswith("dup"):
        frac = int(case[3:]) / 100.0
        for v in range(3 * S):
            a, e = int(co[v]), int(co[v + 1])
            k = int(round(frac * (e - a)))
            dst = rng.choice(np.arange(a, e), size=k, replace=False)
            src = rng.choice(np.setdiff1d(np.arange(a, e), dst), size=k)
            pts[dst] = pts[src]
    elif case == "clutter":
        pts = np.floor(rng.uniform(0.0, IMAGE_SIZE, size=pts.shape) * 2.0) / 2.0
    elif case == "objects":
        pts = _objects_only(b)
    b.pts = pts
    return b


def _objects_only(b):
    """Every detection a noisy projection of one of n shared 3-D objects, on
    each scene's own rig (b.meta's Ks / RTs, so b.F still holds)."""
    from bpc_baseline_amd.synth import _project
    out = np.empty_like(b.pts)
    co = b.cam_offs
    for s_ in range(S):
        X = np.stack([rng.uniform(-250, 250, n), rng.uniform(-250, 250, n), rng.uniform(-80, 80, n)], axis=1)
        for c_ in range(3):
            v = 3 * s_ + c_
            uv = _project(b.meta["Ks"][s_, c_], b.meta["RTs"][s_, c_], X) + rng.normal(0.0, 1.5, (n, 2))
            out[co[v]:co[v + 1]] = (np.round(uv * 2.0) / 2.0)[rng.permutation(n)]
    return out


def time_it(fn, reps):
    ts, out = [], None
    for _ in range(reps + 1):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        out = fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    ts = ts[1:]
    return min(ts), float(np.median(ts)), out


rows = []
for case in args.cases.split(","):
    b = batch_for(case)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    P, C, F = t(b.pts), t(b.cam_offs), t(b.F)
    tp = ops.TripletPlan(b.cam_offs, S, device=dev)
    c3 = tp.counts
    if case.startswith("quant"):
        q = float(case[5:])
        cube, _, _ = ops.triplet_cost_argmin(P, C, F, tp)
        cube.div_(q).floor_().mul_(q)
        # the quantised cube's 8-row minima, as the cube kernel writes them
        v = cube.view(S, n, n // 8, 8, n).amin(dim=3).reshape(-1)
        keys = ((v.view(torch.int32) | int(np.int32(-2 ** 31))) >> 16).to(torch.int16)
        bm8 = keys.contiguous()
        lp = ops.LsapPlan(c3[:, 0] * c3[:, 1], c3[:, 2], device=dev)
        offs = tp.cube_offs[:-1].contiguous()
        fn = lambda: ops.linear_sum_assignment_batched(cube, offs, lp, bmin8=(bm8, tp.bmin8_offs, tp.segs))
        costs_host = lambda s: cube[tp.cube_offs_host[s]:tp.cube_offs_host[s + 1]].cpu().numpy()
    else:
        bm8 = ops.triplet_minima(P, C, F, tp, with_bmin8=args.bmin8)   # (8-row minima, block minima)
        lp = ops.LsapPlan(c3[:, 0] * c3[:, 1], c3[:, 2], device=dev, resid=True)
        fn = lambda: ops.linear_sum_assignment_resid(lp, tp, bm8)

        def costs_host(s):
            from oracle import oracle as O
            co1 = b.cam_offs[3 * s:3 * s + 4]
            return O.cube(b.pts[int(co1[0]):int(co1[3])], co1 - co1[0], b.F[3 * s:3 * s + 3], 1)[0]
    best, med, (r, c, st) = time_it(fn, args.reps)
    st = st.cpu().numpy()
    stats = ops.lsap_sparse_stats(lp)
    ok = bool((st == 0).all())
    r, c = r.cpu().numpy(), c.cpu().numpy()
    o = lp.out_offs_host
    for s in (0, S - 1):
        rr, cc = scipy_lsa(costs_host(s).reshape(n * n, n))
        ok &= bool(np.array_equal(r[o[s]:o[s + 1]], rr) and np.array_equal(c[o[s]:o[s + 1]], cc))
    row = {"case": case, "ms_best": best, "ms_median": med, "status_ok": bool((st == 0).all()),
           "equal_scipy_2_scenes": ok,
           "dense_min_scans": int(stats[:, 0].sum()), "dense_tie_scans": int(stats[:, 1].sum()),
           "overflowed_lists": int(stats[:, 2].sum()), "dijkstra_steps": int(stats[:, 3].sum()),
           "problems_with_fallback": int(((stats[:, 0] + stats[:, 1]) > 0).sum()),
           "max_steps_per_problem": int(stats[:, 3].max())}
    rows.append(row)
    print(json.dumps(row), flush=True)
    del b, P, C, F, tp, bm8, lp, fn
    if case.startswith("quant"):
        del cube
    torch.cuda.empty_cache()

print(f"\n{'case':10s} {'ms best':>8s} {'median':>8s} {'dense min':>10s} {'dense tie':>10s} "
      f"{'overflow':>9s} {'steps':>9s} {'max steps':>9s} exact")
for w in rows:
    print(f"{w['case']:10s} {w['ms_best']:8.2f} {w['ms_median']:8.2f} {w['dense_min_scans']:10d} "
          f"{w['dense_tie_scans']:10d} {w['overflowed_lists']:9d} {w['dijkstra_steps']:9d} "
          f"{w['max_steps_per_problem']:9d} {w['equal_scipy_2_scenes']}")
if args.json:
    with open(args.json, "w") as fh:
        json.dump(rows, fh, indent=1)
