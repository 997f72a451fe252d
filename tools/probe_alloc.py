"""Does the C3 launch time depend on WHICH allocation the distance matrices go
to?  One process, several 25 GB output buffers (torch allocations and one
hipExtMallocWithFlags(hipDeviceMallocContiguous) allocation), the same
1000-scene C3 launch and the write probe timed on each, interleaved.

python tools/probe_alloc.py [--buffers 3] [--rounds 3] [--contiguous]
"""
import argparse
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bpc_baseline_amd import ops  # noqa: E402
from bpc_baseline_amd.synth import make_scenes  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--buffers", type=int, default=3)
ap.add_argument("--rounds", type=int, default=3)
ap.add_argument("--contiguous", action="store_true")
ap.add_argument("--scenes", type=int, default=1000)
ap.add_argument("--first", default="torch", choices=["torch", "contiguous"],
                help="which kind of allocation is made first")
ap.add_argument("--cube", action="store_true", help="the C2 cube launch (250 x 256^3) instead of C3")
ap.add_argument("--variants", default="default",
                help="comma list: default or RPW:RG pairwise options (e.g. 16:1)")
ap.add_argument("--pad-gb", type=float, default=0.0,
                help="allocate (and keep) this many GB before the output buffers")
args = ap.parse_args()

dev = torch.device("cuda", 0)
if args.cube:
    b = make_scenes(250 if args.scenes == 1000 else args.scenes, 3, 256, seed=0)
    plan = ops.TripletPlan(b.cam_offs, b.n_scenes, device=dev)
    plan.n_dist = plan.n_cube
else:
    b = make_scenes(args.scenes, 4, 1024, seed=0)
    plan = ops.PairwisePlan(b.cam_offs, b.n_scenes, b.n_cams, b.pairs, device=dev, row_align="auto")
pts, co, F = (torch.from_numpy(x).to(dev) for x in (b.pts, b.cam_offs, b.F))
am = torch.empty(plan.n_rows, dtype=torch.int32, device=dev)
mv = torch.empty(plan.n_rows, dtype=torch.float32, device=dev)
nbytes = 4.0 * plan.n_dist + 8.0 * plan.n_rows + 16.0 * b.pts.shape[0] + 72.0 * b.F.shape[0]


def run(dist, options):
    if args.cube:
        ops.triplet_cost_argmin(pts, co, F, plan, out=(dist, am, mv), options=options)
    else:
        ops.pairwise_residual_argmin(pts, co, F, plan, out=(dist, am, mv), options=options)


class DevPtr:
    """A raw device allocation exposed to torch via __cuda_array_interface__."""

    def __init__(self, ptr, n):
        self.__cuda_array_interface__ = {"shape": (n,), "typestr": "<f4", "data": (ptr, False),
                                         "version": 2}


pad = torch.empty(int(args.pad_gb * 1e9) // 4, dtype=torch.float32, device=dev) if args.pad_gb else None
bufs = {}


def add_contiguous():
    hip = ctypes.CDLL("libamdhip64.so")
    p = ctypes.c_void_p()
    st = hip.hipExtMallocWithFlags(ctypes.byref(p), ctypes.c_size_t(4 * plan.n_dist), 0x4)
    if st == 0:
        bufs["contiguous"] = torch.as_tensor(DevPtr(p.value, plan.n_dist), device=dev)
    else:
        print(f"hipExtMallocWithFlags(contiguous) failed: {st}")


if args.contiguous and args.first == "contiguous":
    add_contiguous()
for i in range(args.buffers):
    bufs[f"torch{i}"] = torch.empty(plan.dist_size if hasattr(plan, "dist_size") else plan.n_dist, dtype=torch.float32, device=dev)
if args.contiguous and args.first == "torch":
    add_contiguous()
for name, t in bufs.items():
    print(f"{name}: base 0x{t.data_ptr():x}")

variants = args.variants.split(",")


def opts(v):
    if v == "default":
        return None
    if args.cube:
        return {"cube_kernel": v}
    rpw, rg = v.split(":")
    return {"pairwise_rows_per_wave": int(rpw), "pairwise_row_groups": int(rg)}


times = {(n, v): [] for n in bufs for v in variants}
ptimes = {n: [] for n in bufs}
ev = lambda: torch.cuda.Event(enable_timing=True)   # noqa: E731
for rnd in range(args.rounds + 1):
    for name, dist in bufs.items():
      for v in variants:
        run(dist, opts(v))
        e0, e1 = ev(), ev()
        e0.record()
        for _ in range(3):
            run(dist, opts(v))
        e1.record()
        torch.cuda.synchronize()
        if rnd:
            times[(name, v)].append(e0.elapsed_time(e1) / 3)
      if True:
        q0, q1 = ev(), ev()
        q0.record()
        for _ in range(3):
            ops.hbm_write_probe(dist)
        q1.record()
        torch.cuda.synchronize()
        if rnd:
            ptimes[name].append(q0.elapsed_time(q1) / 3)
for name in bufs:
    q = np.array(ptimes[name])
    line = f"{name:>11}: probe {np.median(q):.3f} ms ({4.0 * plan.n_dist / np.median(q) / 1e6:.0f} GB/s)"
    for v in variants:
        t = np.array(times[(name, v)])
        line += f" | {v} {np.median(t):.3f} ms"
    print(line)
