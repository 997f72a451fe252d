"""The cube-free minima kernel (mvm_triplet_minima) alone on a C2-sized batch:
HIP-event time per launch, best and median of --reps, with the same output
buffers every launch.  For A/B of in-tree builds (MVM_LIB_PATH, tools/gpu.sh
ab) and SQ counter passes (tools/gpu.sh sq).

    python tools/bench_minima.py [--scenes 1000 --dets 256 --reps 10]
"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bpc_baseline_amd import _native, ops  # noqa: E402
from bpc_baseline_amd.synth import make_scenes  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--scenes", type=int, default=1000)
ap.add_argument("--dets", type=int, default=256)
ap.add_argument("--reps", type=int, default=10)
ap.add_argument("--no-bmin8", action="store_true", help="no 8-row minima (with_bmin8=False)")
args = ap.parse_args()
dev = torch.device("cuda", 0)
b = make_scenes(args.scenes, 3, args.dets, seed=1)
t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
P, C, F = t(b.pts), t(b.cam_offs), t(b.F)
tp = ops.TripletPlan(b.cam_offs, args.scenes, device=dev)
bm8, bm32 = ops.triplet_minima(P, C, F, tp, with_bmin8=not args.no_bmin8)
ts = []
for _ in range(args.reps):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    ops.triplet_minima(P, C, F, tp, bmin8=bm8, bm32=bm32, with_bmin8=not args.no_bmin8)
    e1.record()
    torch.cuda.synchronize()
    ts.append(e0.elapsed_time(e1))
triples = float(tp.n_cube)
print(f"{_native.version()}{' (no bmin8)' if args.no_bmin8 else ''}: minima best {min(ts):.3f} ms median "
      f"{float(np.median(ts)):.3f} ms  ({triples / min(ts) / 1e9:.1f} G triples/s)", flush=True)
