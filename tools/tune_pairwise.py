"""Interleaved A/B of pairwise-kernel paths in ONE process (perf deltas from
interleaved rounds), selected with explicit mvm_options.  Every variant's
association and first matrix bytes must equal the first variant's.

python tools/tune_pairwise.py [--scenes 1000] [--cams 4] [--dets 1024] [--rounds 5]
                              [--variants default,eager,rpw8]
Variants: a name below, or RPW[:RG[:ARGMIN]] (e.g. 16:4:lazy_rows).
"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bpc_baseline_amd import ops  # noqa: E402
from bpc_baseline_amd.synth import make_scenes  # noqa: E402

NAMED = {"default": {}, "eager": {"pairwise_argmin": "eager"},
         "lazy_rows": {"pairwise_argmin": "lazy_rows"},
         "rpw8": {"pairwise_rows_per_wave": 8}, "rpw4": {"pairwise_rows_per_wave": 4}}


def options_of(v: str) -> dict:
    if v in NAMED:
        return NAMED[v]
    rpw, _, rest = v.partition(":")
    rg, _, argmin = rest.partition(":")
    o = {"pairwise_rows_per_wave": int(rpw)}
    if rg:
        o["pairwise_row_groups"] = int(rg)
    if argmin:
        o["pairwise_argmin"] = argmin
    return o


ap = argparse.ArgumentParser()
ap.add_argument("--scenes", type=int, default=1000)
ap.add_argument("--cams", type=int, default=4)
ap.add_argument("--dets", type=int, default=1024)
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--variants", default="default")
ap.add_argument("--no-dist", action="store_true", help="association only (no matrix output)")
ap.add_argument("--no-argmin", action="store_true", help="matrices only (no association)")
args = ap.parse_args()

dev = torch.device("cuda", 0)
b = make_scenes(args.scenes, args.cams, args.dets, seed=0)
plan = ops.PairwisePlan(b.cam_offs, b.n_scenes, b.n_cams, b.pairs, device=dev, row_align="auto")
pts = torch.from_numpy(b.pts).to(dev)
co = torch.from_numpy(b.cam_offs).to(dev)
F = torch.from_numpy(b.F).to(dev)
dist = torch.empty(0 if args.no_dist else plan.dist_size, dtype=torch.float32, device=dev)
am = torch.empty(0 if args.no_argmin else plan.n_rows, dtype=torch.int32, device=dev)
mv = torch.empty(0 if args.no_argmin else plan.n_rows, dtype=torch.float32, device=dev)
nbytes = (16.0 * b.pts.shape[0] + 72.0 * b.F.shape[0] + (0 if args.no_dist else 4.0 * plan.n_dist)
          + 8.0 * plan.n_rows)
variants = [v.strip() for v in args.variants.split(",")]
times = {v: [] for v in variants}
ref = None
for rnd in range(args.rounds + 1):
    for v in variants:
        opt = options_of(v)
        ops.pairwise_residual_argmin(pts, co, F, plan, out=(dist, am, mv), options=opt)   # warm
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(3):
            ops.pairwise_residual_argmin(pts, co, F, plan, out=(dist, am, mv), options=opt)
        e1.record()
        torch.cuda.synchronize()
        if rnd > 0:
            times[v].append(e0.elapsed_time(e1) / 3)
        chk = (am.cpu().numpy().tobytes(), dist[:1 << 20].cpu().numpy().tobytes())
        if ref is None:
            ref = chk
        assert chk == ref, f"variant {v} differs"
for v in variants:
    t = np.array(times[v])
    print(f"{v:>12}: median {np.median(t):.3f} ms  min {t.min():.3f} ms  "
          f"{nbytes / (np.median(t) * 1e-3) / 1e9:.0f} GB/s  "
          f"{plan.n_dist / (np.median(t) * 1e-3):.3e} pairs/s")
