"""Interleaved A/B of LSAP kernel classes (explicit mvm_options) on a batch of
flattened cubes.  python tools/tune_lsap.py --scenes 1000 --dets 64 --variants wg256,wg1024"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bpc_baseline_amd import ops  # noqa: E402
from bpc_baseline_amd.synth import make_scenes  # noqa: E402

OFF = {"lsap_wave_max_cols": -1, "lsap_multi_g": -1, "lsap_reg_max_cols": -1}
VARIANTS = {"default": {},
            "wave": {"lsap_multi_g": -1},
            "multi": {"lsap_wave_max_cols": -1},
            "reg": {"lsap_wave_max_cols": -1, "lsap_multi_g": -1},
            "reg1024": {"lsap_wave_max_cols": -1, "lsap_multi_g": -1, "lsap_reg_threads": 1024},
            "lds": OFF,
            "lds1024": dict(OFF, lsap_lds_small_cols=-1),
            "lds256": dict(OFF, lsap_lds_small_cols=4096),
            "wg256": dict(OFF, lsap_lds_max_cols=-1, lsap_mid_max_cols=1000000),
            "wg1024": dict(OFF, lsap_lds_max_cols=-1, lsap_mid_max_cols=-1),
            "nomreg": {"lsap_mreg_max_cols": -1},
            "mreg": {"lsap_wave_max_cols": -1, "lsap_reg_max_cols": -1, "lsap_multi_g": -1},
            "wave512": {"lsap_wave_max_cols": 512, "lsap_multi_g": -1},
            "wave256": {"lsap_wave_max_cols": 256, "lsap_multi_g": -1}}

ap = argparse.ArgumentParser()
ap.add_argument("--scenes", type=int, default=1000)
ap.add_argument("--dets", type=int, default=64)
ap.add_argument("--rounds", type=int, default=3)
ap.add_argument("--variants", default="default,reg,reg1024,lds")
args = ap.parse_args()
dev = torch.device("cuda", 0)
b = make_scenes(args.scenes, 3, args.dets, seed=1)
tp = ops.TripletPlan(b.cam_offs, b.n_scenes, device=dev)
cube, _, _ = ops.triplet_cost_argmin(*(torch.from_numpy(x).to(dev) for x in (b.pts, b.cam_offs, b.F)), tp)
n = args.dets
plan = ops.LsapPlan(np.full(b.n_scenes, n * n), np.full(b.n_scenes, n), device=dev)
offs = tp.cube_offs[:-1].contiguous()
times = {v: [] for v in args.variants.split(",")}
ref = None
for rnd in range(args.rounds + 1):
    for v in times:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        r, c, st = ops.linear_sum_assignment_batched(cube, offs, plan, options=VARIANTS[v])
        e1.record()
        torch.cuda.synchronize()
        assert int(st.max()) == 0, v
        if rnd:
            times[v].append(e0.elapsed_time(e1))
        chk = (r.cpu().numpy().tobytes(), c.cpu().numpy().tobytes())
        ref = ref or chk
        assert chk == ref, v
for v, t in times.items():
    print(f"{v:>8}: median {np.median(t):.3f} ms  ({args.scenes} problems of {n * n} x {n})")
