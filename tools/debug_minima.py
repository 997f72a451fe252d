"""Where mvm_triplet_minima's 8-row minima differ from the oracle's (debug aid):
counts, key differences and positions on one 256^3 scene."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bpc_baseline_amd import ops  # noqa: E402
from bpc_baseline_amd.synth import make_scenes  # noqa: E402
from oracle import oracle as O  # noqa: E402

dev = torch.device("cuda", 0)
b = make_scenes(2, 3, 256, seed=5)
t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
tp = ops.TripletPlan(b.cam_offs, 2, device=dev)
bm8, bm32 = ops.triplet_minima(t(b.pts), t(b.cam_offs), t(b.F), tp)
got = bm8.cpu().numpy().view(np.uint16)[:256 * 32 * 256].reshape(256, 32, 256)
cube = O.cube(b.pts, b.cam_offs, b.F, 2)[0][:256 ** 3].reshape(256, 256, 256)
want = O.bmin8_keys(cube)
bad = got != want
print("mismatches", int(bad.sum()), "of", bad.size)
if bad.any():
    idx = np.argwhere(bad)
    d = got[bad].astype(np.int64) - want[bad].astype(np.int64)
    print("diff histogram", dict(zip(*np.unique(d, return_counts=True))) if len(np.unique(d)) < 30 else
          (d.min(), d.max()))
    print("by g:", np.bincount(idx[:, 1], minlength=32))
    print("by k mod 64:", np.bincount(idx[:, 2] % 64, minlength=64))
    print("by i mod 16:", np.bincount(idx[:, 0] % 16, minlength=16))
    for i, g, k in idx[:8]:
        print(i, g, k, hex(got[i, g, k]), hex(want[i, g, k]), cube[i, 8 * g:8 * g + 8, k])
