"""Interleaved A/B of cube-kernel paths in one process, selected with explicit
mvm_options; every variant's association and first cube bytes must equal the
first variant's.

python tools/tune_cube.py [--scenes 250] [--dets 256] [--rounds 5] [--variants fused,workspace]
"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bpc_baseline_amd import ops  # noqa: E402
from bpc_baseline_amd.synth import make_scenes  # noqa: E402

VARIANTS = {"default": {}, "small": {"cube_kernel": "small"}, "fused": {"cube_kernel": "fused"},
            "fused1": {"cube_kernel": "fused", "cube_rows_per_instr": 1},
            "fused2": {"cube_kernel": "fused", "cube_rows_per_instr": 2},
            "workspace": {"cube_kernel": "workspace"}, "generic": {"cube_kernel": "generic"}}

ap = argparse.ArgumentParser()
ap.add_argument("--scenes", type=int, default=250)
ap.add_argument("--dets", type=int, default=256)
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--variants", default="fused,workspace")
args = ap.parse_args()
dev = torch.device("cuda", 0)
b = make_scenes(args.scenes, 3, args.dets, seed=0)
plan = ops.TripletPlan(b.cam_offs, b.n_scenes, device=dev)
pts, co, F = (torch.from_numpy(x).to(dev) for x in (b.pts, b.cam_offs, b.F))
out = (torch.empty(plan.n_cube, dtype=torch.float32, device=dev),
       torch.empty(plan.n_rows, dtype=torch.int32, device=dev),
       torch.empty(plan.n_rows, dtype=torch.float32, device=dev))
nbytes = 4.0 * plan.n_cube + 8.0 * plan.n_rows + 16.0 * b.pts.shape[0] + 72.0 * b.F.shape[0]
times = {v: [] for v in args.variants.split(",")}
ref = None
for rnd in range(args.rounds + 1):
    for v in times:
        opt = VARIANTS[v]
        ops.triplet_cost_argmin(pts, co, F, plan, out=out, options=opt)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(3):
            ops.triplet_cost_argmin(pts, co, F, plan, out=out, options=opt)
        e1.record()
        torch.cuda.synchronize()
        if rnd:
            times[v].append(e0.elapsed_time(e1) / 3)
        chk = (out[1].cpu().numpy().tobytes(), out[0][:1 << 22].cpu().numpy().tobytes())
        ref = ref or chk
        assert chk == ref, v
for v, t in times.items():
    t = np.array(t)
    print(f"{v:>10}: median {np.median(t):.3f} ms  {nbytes / np.median(t) / 1e6:.0f} GB/s  "
          f"{plan.n_cube / np.median(t) / 1e-3:.3e} triples/s")
