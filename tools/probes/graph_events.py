"""Can HIP events recorded INSIDE a captured hipGraph time the kernels between
them on replay?  (bench.py --graph steps would then keep per-launch times.)

python tools/probes/graph_events.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from bpc_baseline_amd import ops  # noqa: E402

dev = torch.device("cuda", 0)
buf = torch.empty(1 << 28, dtype=torch.float32, device=dev)   # 1 GiB
ops.hbm_write_probe(buf)
torch.cuda.synchronize()
n = 4
evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g, capture_error_mode="thread_local"):
    for e0, e1 in evs:
        e0.record()
        ops.hbm_write_probe(buf)
        e1.record()
outer0, outer1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for rep in range(3):
    outer0.record()
    g.replay()
    outer1.record()
    torch.cuda.synchronize()
    try:
        inner = [e0.elapsed_time(e1) for e0, e1 in evs]
    except RuntimeError as ex:
        inner = f"error: {ex}"
    print(f"replay {rep}: outer {outer0.elapsed_time(outer1):.4f} ms, inner {inner}")
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(n):
    ops.hbm_write_probe(buf)
e1.record()
torch.cuda.synchronize()
print(f"eager {n} launches: {e0.elapsed_time(e1):.4f} ms")
