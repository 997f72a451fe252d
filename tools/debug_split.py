"""Where a mixed match_captures batch spends its assignment time (debug aid):
the cube-free part and the dense part of a detector batch, timed apart."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bpc_baseline_amd import ops  # noqa: E402
from bpc_baseline_amd.inference.batch_match import match_captures  # noqa: E402
from bpc_baseline_amd.synth import make_detector_batch  # noqa: E402

dets = int(sys.argv[1]) if len(sys.argv) > 1 else 64
dev = torch.device("cuda", 0)
b = make_detector_batch(1000, dets, seed=5)
t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
boxes, conf, cls, offs = t(b.boxes), t(b.conf), t(b.cls), t(b.img_offs)
r = match_captures(boxes, conf, cls, offs, b.Ks, b.RTs)
c3 = np.diff(r.cam_offs).reshape(-1, 3)
free = ops.cube_free_scenes(c3)
nm = c3[:, 0] * c3[:, 1]
print("scenes", len(c3), "free", int(free.sum()), "N*M range free", nm[free].min() if free.any() else None,
      nm[free].max() if free.any() else None, "P free max", c3[free, 2].max() if free.any() else None)
for keep in (False, True):
    st = {}
    for _ in range(3):
        match_captures(boxes, conf, cls, offs, b.Ks, b.RTs, keep_cube=keep, timings=st)
    print("keep_cube", keep, {k: round(v / 3 * 1e3, 3) for k, v in st.items()})
