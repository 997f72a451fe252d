"""Per-launch time of the pairwise launch against its size, with the host out
of the way (each size's launches captured in one hipGraph and replayed), next
to the write probe over the same bytes: separates a launch's fixed cost
(start-up, the last partial round of workgroups) from its per-byte cost.

python tools/launch_scaling.py [--cams 3] [--dets 256] [--scenes 250,500,1000,2000,4000]
                               [--reps 20] [--variants default,16:1,16:4]
"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bpc_baseline_amd import ops  # noqa: E402
from bpc_baseline_amd.synth import make_scenes  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--cams", type=int, default=3)
ap.add_argument("--dets", type=int, default=256)
ap.add_argument("--scenes", default="250,500,1000,2000,4000")
ap.add_argument("--reps", type=int, default=20)
ap.add_argument("--rounds", type=int, default=3)
ap.add_argument("--variants", default="default")
args = ap.parse_args()


def options_of(v):
    if v == "default":
        return {}
    rpw, _, rg = v.partition(":")
    o = {"pairwise_rows_per_wave": int(rpw)}
    if rg:
        o["pairwise_row_groups"] = int(rg)
    return o


dev = torch.device("cuda", 0)
sizes = [int(x) for x in args.scenes.split(",")]
variants = args.variants.split(",")
b = make_scenes(max(sizes), args.cams, args.dets, seed=0)
rows = []
for n in sizes:
    C, P = b.n_cams, b.n_pairs
    co = b.cam_offs[:n * C + 1]
    plan = ops.PairwisePlan(co, n, C, b.pairs, device=dev, row_align="auto")
    pts = torch.from_numpy(b.pts[:int(co[-1])]).to(dev)
    cot = torch.from_numpy(co).to(dev)
    F = torch.from_numpy(b.F[:n * P]).to(dev)
    dist = torch.empty(plan.dist_size, dtype=torch.float32, device=dev)
    am = torch.empty(plan.n_rows, dtype=torch.int32, device=dev)
    mv = torch.empty(plan.n_rows, dtype=torch.float32, device=dev)
    graphs = {}
    for v in variants:
        opt = options_of(v)
        ops.pairwise_residual_argmin(pts, cot, F, plan, out=(dist, am, mv), options=opt)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(args.reps):
                ops.pairwise_residual_argmin(pts, cot, F, plan, out=(dist, am, mv), options=opt)
        g.replay()
        graphs[v] = g
    pg = torch.cuda.CUDAGraph()
    with torch.cuda.graph(pg):
        for _ in range(args.reps):
            ops.hbm_write_probe(dist)
    pg.replay()
    torch.cuda.synchronize()
    t = {v: [] for v in variants + ["probe"]}
    for _ in range(args.rounds):
        for v, g in list(graphs.items()) + [("probe", pg)]:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            g.replay()
            e1.record()
            torch.cuda.synchronize()
            t[v].append(e0.elapsed_time(e1) / args.reps)
    med = {v: float(np.median(x)) for v, x in t.items()}
    rows.append((n, plan.dist_size * 4 / 1e9, med))
    print(f"{n:>6} scenes {plan.dist_size * 4 / 1e9:7.3f} GB  probe {med['probe']:.4f} ms  " +
          "  ".join(f"{v} {med[v]:.4f} ms ({med[v] / med['probe']:.3f}x)" for v in variants),
          flush=True)
    del dist, graphs, pg
    torch.cuda.empty_cache()
# least-squares fixed + per-GB cost per variant
gb = np.array([r[1] for r in rows])
for v in variants + ["probe"]:
    ms = np.array([r[2][v] for r in rows])
    A = np.vstack([np.ones_like(gb), gb]).T
    (c0, c1), *_ = np.linalg.lstsq(A, ms, rcond=None)
    print(f"{v:>10}: fixed {c0 * 1e3:.1f} us per launch + {c1:.4f} ms/GB ({1 / c1:.2f} TB/s marginal)")
