"""Where the candidate-list solver's time goes (diagnostic build only):
MVM_LIB_PATH=bpc_baseline_amd/lib/ab/solve_phases.so python tools/solve_phases.py

The build (tools/build_variant.py solve_phases --patch solve_phases) records
thread 0's s_memtime cycles per phase of every problem's searches:
  0 the step's row data in registers (waits for its loads), 1 the slot scan
  and the free entry, 2 the wave reductions and records, 3 the step barrier,
  4 the combine / free minimum / rb, 5 the tie scan (general sink), 6 the
  rest of a search, 7 the tail, 8 a removal step's tail up to the next step;
  9 counts the searches whose sink came from the first step.
"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bpc_baseline_amd import _native, ops  # noqa: E402
from bpc_baseline_amd.synth import make_scenes  # noqa: E402

dev = torch.device("cuda", 0)
S, n = 1000, 256
b = make_scenes(S, 3, n, seed=1)
t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
P, C, F = t(b.pts), t(b.cam_offs), t(b.F)
tp = ops.TripletPlan(b.cam_offs, S, device=dev)
mn = ops.triplet_minima(P, C, F, tp, with_bmin8=False)
c3 = tp.counts
lp = ops.LsapPlan(c3[:, 0] * c3[:, 1], c3[:, 2], device=dev, resid=True)
for _ in range(2):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    ops.linear_sum_assignment_resid(lp, tp, mn)
    e1.record()
    torch.cuda.synchronize()
    print("assignment ms", e0.elapsed_time(e1))
lib = _native.load()
buf = (ctypes.c_ulonglong * (S * 10))()
assert lib.mvm_diag_solve_phases(buf, S) == 0
ph = np.frombuffer(buf, dtype=np.uint64).reshape(S, 10).astype(np.float64)
st = ops.lsap_sparse_stats(lp)
tot = ph[:, :9].sum(axis=1)
print("cycles per problem (mean / max):", tot.mean(), tot.max())
for k, name in enumerate(["row data (load waits)", "slot scan + free entry", "wave records",
                          "step barrier", "combine + free min", "tie scan", "search rest", "tail",
                          "removal step tail"]):
    print(f"  {name:26s} mean {ph[:, k].mean():12.0f}  ({ph[:, k].mean() / tot.mean():.1%})")
print("searches with a first-step sink per problem:", ph[:, 9].mean(), " steps per problem:",
      st[:, 3].mean())
