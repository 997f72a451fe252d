"""Do back-to-back C3 launches gain from alternating two HIP streams (the next
launch's workgroups filling the CUs left idle by the previous launch's tail)?
Ten launches into ten of the bench's 25 GB allocations, one stream vs two,
interleaved, same buffers.

python tools/probes/two_streams.py [--rounds 4]
"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from bpc_baseline_amd import ops  # noqa: E402
from bpc_baseline_amd.synth import make_scenes  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--rounds", type=int, default=4)
ap.add_argument("--launches", type=int, default=10)
args = ap.parse_args()

dev = torch.device("cuda", 0)
b = make_scenes(1000, 4, 1024, seed=0)
plan = ops.PairwisePlan(b.cam_offs, b.n_scenes, b.n_cams, b.pairs, device=dev, row_align="auto")
pts, co, F = (torch.from_numpy(x).to(dev) for x in (b.pts, b.cam_offs, b.F))
n = args.launches
bufs = [torch.empty(plan.dist_size, dtype=torch.float32, device=dev) for _ in range(n)]
ams = [torch.empty(plan.n_rows, dtype=torch.int32, device=dev) for _ in range(n)]
mvs = [torch.empty(plan.n_rows, dtype=torch.float32, device=dev) for _ in range(n)]
main = torch.cuda.current_stream(dev)
side = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]


def run(k_streams):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(main)
    for s in side:
        s.wait_stream(main)
    for i in range(n):
        s = main if k_streams == 1 else side[i % 2]
        with torch.cuda.stream(s):
            ops.pairwise_residual_argmin(pts, co, F, plan, out=(bufs[i], ams[i], mvs[i]))
    for s in side:
        main.wait_stream(s)
    e1.record(main)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1)


run(1)
run(2)   # warm-up: every buffer written once
ref = [a.clone() for a in ams]
t = {1: [], 2: []}
for r in range(args.rounds):
    for k in ((1, 2) if r % 2 == 0 else (2, 1)):
        t[k].append(run(k))
    assert all(torch.equal(a, b) for a, b in zip(ams, ref)), "results differ"
for k in (1, 2):
    print(f"{k} stream(s): {n} launches {np.median(t[k]):.3f} ms median "
          f"({' '.join(f'{x:.3f}' for x in t[k])}), {np.median(t[k]) / n:.4f} ms per launch")
print(f"two streams / one: {np.median(t[2]) / np.median(t[1]):.4f}")
