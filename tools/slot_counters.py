"""Per-output-allocation timing of the C3 launch, for PMC passes over the same
allocations ("the same launch runs up to ~18% apart on
different allocations -- which hardware counter moves with it?").

Allocates the output buffers in the order bench.py does (inputs first, then
--buffers launch-sized float32 allocations), then runs --rounds rounds of one
launch per buffer, buffer 0 first, timing each with HIP events.  Under
``rocprofv3 --pmc ...`` the dispatches of the pairwise kernel come in the
order printed here (warm-up launch first), so the counter CSV maps to buffers
by dispatch index: tools/slot_counters.py --summarise CSV.

python tools/slot_counters.py [--buffers 11] [--rounds 2] [--scenes 1000] [--cams 4 --dets 1024]
                              [--repeat R]   (R launches per buffer back to back: the
                                              first after another buffer, the rest on a
                                              buffer just written -- C2's same-buffer gap)
python tools/slot_counters.py --summarise run_counter_collection.csv [--buffers 11]
"""
import argparse
import csv
import json
import os
import sys
from collections import defaultdict

ap = argparse.ArgumentParser()
ap.add_argument("--buffers", type=int, default=11)
ap.add_argument("--rounds", type=int, default=2)
ap.add_argument("--scenes", type=int, default=1000)
ap.add_argument("--summarise", default=None, metavar="CSV")
ap.add_argument("--kernel", default="pairwise_lazy_kernel")
ap.add_argument("--cams", type=int, default=4)
ap.add_argument("--dets", type=int, default=1024)
ap.add_argument("--repeat", type=int, default=1)
ap.add_argument("--options", default=None,
                help="comma list of mvm_options fields for the launches (e.g. "
                     "pairwise_row_interleave=-1)")
args = ap.parse_args()

if args.summarise:
    # dispatch order of the kernel: warm-up, then rounds x buffers
    per = defaultdict(lambda: defaultdict(float))
    order = []
    for r in csv.DictReader(open(args.summarise)):
        if args.kernel not in r["Kernel_Name"]:
            continue
        d = int(r["Dispatch_Id"])
        if d not in per:
            order.append(d)
        per[d][r["Counter_Name"]] += float(r["Counter_Value"])
    order.sort()
    launches = order[1:]                      # the first is the warm-up launch
    by_buf = defaultdict(lambda: defaultdict(list))
    for k, d in enumerate(launches):
        for c, v in per[d].items():
            by_buf[k % args.buffers][c].append(v)
    names = sorted({c for d in per.values() for c in d})
    out = {b: {c: sum(v) / len(v) for c, v in cs.items()} for b, cs in sorted(by_buf.items())}
    print("buffer " + " ".join(f"{c:>28}" for c in names))
    for b, cs in out.items():
        print(f"{b:>6} " + " ".join(f"{cs.get(c, 0):>28.4g}" for c in names))
    print(json.dumps({"per_buffer": out}))
    sys.exit(0)

import numpy as np  # noqa: E402
import torch  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bpc_baseline_amd import ops  # noqa: E402
from bpc_baseline_amd.synth import make_scenes  # noqa: E402

dev = torch.device("cuda", 0)
b = make_scenes(args.scenes, args.cams, args.dets, seed=0)
plan = ops.PairwisePlan(b.cam_offs, b.n_scenes, b.n_cams, b.pairs, device=dev, row_align="auto")
pts, co, F = (torch.from_numpy(x).to(dev) for x in (b.pts, b.cam_offs, b.F))
am = torch.empty(plan.n_rows, dtype=torch.int32, device=dev)
mv = torch.empty(plan.n_rows, dtype=torch.float32, device=dev)
nbytes = 4.0 * plan.n_dist + 8.0 * plan.n_rows + 16.0 * b.pts.shape[0] + 72.0 * b.F.shape[0]
opts = None
if args.options:
    opts = {k: int(v) for k, v in (kv.split("=") for kv in args.options.split(","))}
bufs = []
for _ in range(args.buffers):
    try:
        bufs.append(torch.empty(plan.dist_size, dtype=torch.float32, device=dev))
    except torch.cuda.OutOfMemoryError:
        break
print(f"{len(bufs)} buffers of {4 * plan.dist_size / 1e9:.1f} GB at "
      + ", ".join(f"0x{x.data_ptr():x}" for x in bufs), flush=True)
ops.pairwise_residual_argmin(pts, co, F, plan, out=(bufs[0], am, mv), options=opts)   # warm-up
torch.cuda.synchronize()
times = defaultdict(list)
reps = defaultdict(lambda: defaultdict(list))   # buffer -> repeat index -> ms
for rnd in range(args.rounds):
    evs = []
    for i, buf in enumerate(bufs):
        for r in range(args.repeat):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            ops.pairwise_residual_argmin(pts, co, F, plan, out=(buf, am, mv), options=opts)
            e1.record()
            evs.append((i, r, e0, e1))
        if args.repeat == 1:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    for i, r, e0, e1 in evs:
        reps[i][r].append(e0.elapsed_time(e1))
        if r == 0:
            times[i].append(e0.elapsed_time(e1))
    print(f"round {rnd}: " + " ".join(f"{times[i][-1]:.3f}" for i in range(len(bufs))), flush=True)
if args.repeat > 1:
    for r in range(args.repeat):
        print(f"repeat {r}: mean {np.mean([np.mean(reps[i][r]) for i in reps]):.4f} ms over the buffers",
              flush=True)
rows = {i: {"ms": float(np.mean(t)), "tb_s": nbytes / (np.mean(t) * 1e-3) / 1e12}
        for i, t in times.items()}
ms = [r["ms"] for r in rows.values()]
print(json.dumps({"per_buffer": rows, "slowest_over_fastest": max(ms) / min(ms)}))
