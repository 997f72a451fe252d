"""Dijkstra steps per problem of the candidate-list assignment on C2-like
cubes (the restatement oracle/lsap_sparse.py counts them), for the solver's
latency model: the batch runs every problem at once, so the solve kernel's
time over the mean step count is the time of one step.

python tools/lsap_step_model.py [--scenes 3] [--dets 256] [--solve-ms 1.76]
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bpc_baseline_amd.synth import make_scenes  # noqa: E402
from oracle import oracle as O  # noqa: E402
from oracle import lsap_sparse as LS  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--scenes", type=int, default=3)
ap.add_argument("--dets", type=int, default=256)
ap.add_argument("--solve-ms", type=float, default=None,
                help="sp_solve_kernel's traced time for a batch (all problems at once)")
args = ap.parse_args()
b = make_scenes(args.scenes, 3, args.dets, seed=0)
cubes, _, _, _, _ = O.cube(b.pts, b.cam_offs, b.F, b.n_scenes, nthreads=os.cpu_count() or 1)
n = args.dets
per = []
for s in range(args.scenes):
    c = cubes[s * n ** 3:(s + 1) * n ** 3].reshape(n * n, n)
    st = {}
    LS.linear_sum_assignment(c, stats=st, key16=True)
    per.append(st)
steps = [p["steps"] for p in per]
out = {"dets": n, "scenes": args.scenes, "steps_per_problem": steps,
       "mean_steps": float(np.mean(steps)), "searches": [p["searches"] for p in per],
       "dense_rows": [p["dense_rows"] for p in per]}
if args.solve_ms:
    out["solve_ms"] = args.solve_ms
    out["us_per_step"] = args.solve_ms * 1e3 / out["mean_steps"]
print(json.dumps(out))
