"""The assignment's block minima at a given view size: from the cube kernel's
8-row minima (requested from the cube launch: written by the kernel itself on
its one-row-per-instruction forms, else read back from the cube by
bmin8_from_cube_kernel) vs the assignment reading the cost itself
(sp_blockmin_kernel).  Same batch, HIP events, alternating.

python tools/ab_bmin8_input.py --scenes 1000 --dets 64 [--rounds 5]
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
ap.add_argument("--scenes", type=int, default=1000)
ap.add_argument("--dets", type=int, default=64)
ap.add_argument("--rounds", type=int, default=5)
args = ap.parse_args()
dev = torch.device("cuda", 0)
b = make_scenes(args.scenes, 3, args.dets, seed=0)
pts, co, F = (torch.from_numpy(x).to(dev) for x in (b.pts, b.cam_offs, b.F))
tp = ops.TripletPlan(b.cam_offs, b.n_scenes, device=dev)
c3 = tp.counts
lp = ops.LsapPlan(c3[:, 0] * c3[:, 1], c3[:, 2], device=dev)
cube = torch.empty(tp.n_cube, dtype=torch.float32, device=dev)
am = torch.empty(tp.n_rows, dtype=torch.int32, device=dev)
mv = torch.empty(tp.n_rows, dtype=torch.float32, device=dev)
bm8 = torch.empty(max(tp.n_bmin8, 1), dtype=torch.int16, device=dev)
offs = tp.cube_offs[:-1].contiguous()


def run(use):
    e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    e[0].record()
    ops.triplet_cost_argmin(pts, co, F, tp, out=(cube, am, mv), bmin8=bm8 if use else None)
    e[1].record()
    r, c, st = ops.linear_sum_assignment_batched(cube, offs, lp,
                                                 bmin8=(bm8, tp.bmin8_offs, tp.segs) if use else None)
    e[2].record()
    torch.cuda.synchronize()
    return e[0].elapsed_time(e[1]), e[1].elapsed_time(e[2]), r.cpu().numpy(), c.cpu().numpy()


t = {True: [], False: []}
ref = None
for k in range(args.rounds + 1):
    for use in (True, False) if k % 2 else (False, True):
        a, l, r, c = run(use)
        if ref is None:
            ref = (r, c)
        assert np.array_equal(r, ref[0]) and np.array_equal(c, ref[1]), "assignments differ"
        if k:
            t[use].append((a, l))
for use in (True, False):
    a = np.median(np.array(t[use]), axis=0)
    print(f"{'8-row minima' if use else 'cost itself ':>13}: cube {a[0]:.3f} ms  assignment {a[1]:.3f} ms  "
          f"total {a.sum():.3f} ms")
