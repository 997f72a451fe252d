"""Interleaved A/B of cube-kernel variants in one process (env knobs)."""
import argparse, os, sys
import numpy as np, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bpc_baseline_amd import ops  # noqa: E402
from bpc_baseline_amd.synth import make_scenes  # noqa: E402
ap = argparse.ArgumentParser()
ap.add_argument("--scenes", type=int, default=250)
ap.add_argument("--dets", type=int, default=256)
ap.add_argument("--rounds", type=int, default=5)
ap.add_argument("--variants", default="fused,tile,generic")
args = ap.parse_args()
dev = torch.device("cuda", 0)
b = make_scenes(args.scenes, 3, args.dets, seed=0)
plan = ops.TripletPlan(b.cam_offs, b.n_scenes, device=dev)
pts, co, F = (torch.from_numpy(x).to(dev) for x in (b.pts, b.cam_offs, b.F))
out = (torch.empty(plan.n_cube, dtype=torch.float32, device=dev),
       torch.empty(plan.n_rows, dtype=torch.int32, device=dev),
       torch.empty(plan.n_rows, dtype=torch.float32, device=dev))
nbytes = 4.0 * plan.n_cube + 8.0 * plan.n_rows + 16.0 * b.pts.shape[0] + 72.0 * b.F.shape[0]
env = {"tile": {"MVM_TRIPLET_VARIANT": "3", "MVM_TRIPLET_SMALL": "0", "MVM_TRIPLET_FUSED": "0"},
       "fused": {"MVM_TRIPLET_VARIANT": "3", "MVM_TRIPLET_SMALL": "0", "MVM_TRIPLET_FUSED": "1"},
       "fusedx": {"MVM_TRIPLET_VARIANT": "3", "MVM_TRIPLET_SMALL": "0", "MVM_TRIPLET_FUSED": "1", "MVM_TRIPLET_XCD": "1"},
       "f32x32": {"MVM_TRIPLET_SMALL": "0", "MVM_TRIPLET_FUSED": "1", "MVM_TRIPLET_TILE": "4"},
       "f8x32": {"MVM_TRIPLET_SMALL": "0", "MVM_TRIPLET_FUSED": "1", "MVM_TRIPLET_TILE": "2"},
       "f16x16": {"MVM_TRIPLET_SMALL": "0", "MVM_TRIPLET_FUSED": "1", "MVM_TRIPLET_TILE": "0"},
       "small": {"MVM_TRIPLET_SMALL": "1"},
       "small4": {"MVM_TRIPLET_SMALL": "1", "MVM_TRIPLET_SMALL_IB": "4"},
       "small8": {"MVM_TRIPLET_SMALL": "1", "MVM_TRIPLET_SMALL_IB": "8"},
       "small32": {"MVM_TRIPLET_SMALL": "1", "MVM_TRIPLET_SMALL_IB": "32"},
       "small64": {"MVM_TRIPLET_SMALL": "1", "MVM_TRIPLET_SMALL_IB": "64"},
       "t16x16": {"MVM_TRIPLET_VARIANT": "3", "MVM_TRIPLET_TILE": "0"},
       "t8x16": {"MVM_TRIPLET_VARIANT": "3", "MVM_TRIPLET_TILE": "1"},
       "t8x32": {"MVM_TRIPLET_VARIANT": "3", "MVM_TRIPLET_TILE": "2"},
       "t16x32": {"MVM_TRIPLET_VARIANT": "3", "MVM_TRIPLET_TILE": "3"},
       "generic": {"MVM_TRIPLET_VARIANT": "1"},
       "chunked": {"MVM_TRIPLET_CHUNKED": "1"},
       "nochunk": {"MVM_TRIPLET_CHUNKED": "0"},
       "nohalf": {"MVM_TRIPLET_VARIANT": "3", "MVM_TRIPLET_SMALL": "0", "MVM_TRIPLET_FUSED": "1", "MVM_TRIPLET_HALF": "0"},
       "split2": {"MVM_TRIPLET_VARIANT": "3", "MVM_TRIPLET_SMALL": "0", "MVM_TRIPLET_FUSED": "1", "MVM_TRIPLET_HALF": "2"}}
times = {v: [] for v in args.variants.split(",")}
ref = None
for rnd in range(args.rounds + 1):
    for v in times:
        for k in ("MVM_TRIPLET_RPW", "MVM_TRIPLET_VARIANT", "MVM_TRIPLET_TILE", "MVM_TRIPLET_SMALL",
                  "MVM_TRIPLET_SMALL_IB", "MVM_TRIPLET_FUSED", "MVM_TRIPLET_XCD", "MVM_TRIPLET_CHUNKED",
                  "MVM_TRIPLET_HALF"):
            os.environ.pop(k, None)
        os.environ.update(env[v])
        ops.triplet_cost_argmin(pts, co, F, plan, out=out)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(3):
            ops.triplet_cost_argmin(pts, co, F, plan, out=out)
        e1.record()
        torch.cuda.synchronize()
        if rnd:
            times[v].append(e0.elapsed_time(e1) / 3)
        chk = (out[1].cpu().numpy().tobytes(), out[0][:1 << 22].cpu().numpy().tobytes())
        ref = ref or chk
        assert chk == ref, v
for v, t in times.items():
    t = np.array(t)
    print(f"{v:>8}: median {np.median(t):.3f} ms  {nbytes / np.median(t) / 1e6:.0f} GB/s  "
          f"{plan.n_cube / np.median(t) / 1e-3:.3e} triples/s (incl. fp64 prologue)")
