"""Interleaved A/B of LSAP kernel choices (env knobs) on a batch of flattened
cubes.  python tools/tune_lsap.py --scenes 1000 --dets 64 --variants wg256,wg1024"""
import argparse, os, sys
import numpy as np, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bpc_baseline_amd import ops  # noqa: E402
from bpc_baseline_amd.synth import make_scenes  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--scenes", type=int, default=1000)
ap.add_argument("--dets", type=int, default=64)
ap.add_argument("--rounds", type=int, default=3)
ap.add_argument("--variants", default="wg256,wg1024")
args = ap.parse_args()
ENV = {"wg256": {"MVM_LSAP_MULTI_G": "0", "MVM_LSAP_MID_MAX_COLS": "1000000"},
       "wg1024": {"MVM_LSAP_MULTI_G": "0", "MVM_LSAP_MID_MAX_COLS": "0"},
       "multi": {"MVM_LSAP_MULTI_G": "-1"},
       "wave": {"MVM_LSAP_WAVE_MAX_COLS": "1024"},
       "wave_dpp": {"MVM_LSAP_WAVE_MAX_COLS": "1024", "MVM_LSAP_DPP": "1"},
       "wave_shfl": {"MVM_LSAP_WAVE_MAX_COLS": "1024", "MVM_LSAP_DPP": "0"},
       "wg256_shfl": {"MVM_LSAP_MULTI_G": "0", "MVM_LSAP_MID_MAX_COLS": "1000000", "MVM_LSAP_DPP": "0"},
       "wg1024_shfl": {"MVM_LSAP_MULTI_G": "0", "MVM_LSAP_MID_MAX_COLS": "0", "MVM_LSAP_DPP": "0"},
       "wave_wg256": {"MVM_LSAP_WAVE_MAX_COLS": "0", "MVM_LSAP_MULTI_G": "0", "MVM_LSAP_MID_MAX_COLS": "1000000"},
       "nowave": {"MVM_LSAP_WAVE_MAX_COLS": "0", "MVM_LSAP_MULTI_G": "0", "MVM_LSAP_MID_MAX_COLS": "0"},
       "lds": {"MVM_LSAP_MULTI_G": "0"},
       "nolds": {"MVM_LSAP_MULTI_G": "0", "MVM_LSAP_LDS_MAX_COLS": "0"},
       "lds1024": {"MVM_LSAP_MULTI_G": "0", "MVM_LSAP_LDS_SMALL_COLS": "0"},
       "lds256": {"MVM_LSAP_MULTI_G": "0", "MVM_LSAP_LDS_SMALL_COLS": "4096"}}
KEYS = ("MVM_LSAP_MULTI_G", "MVM_LSAP_MID_MAX_COLS", "MVM_LSAP_WAVE_MAX_COLS", "MVM_LSAP_DPP",
        "MVM_LSAP_LDS_MAX_COLS", "MVM_LSAP_LDS_SMALL_COLS")
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
        for k in KEYS:
            os.environ.pop(k, None)
        os.environ.update(ENV[v])
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        r, c, st = ops.linear_sum_assignment_batched(cube, offs, plan)
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
