"""Clock and power under the write probe vs under the residual kernel, on the
same output buffer: each runs back to back for --seconds while bench.py's
ClockSampler reads the card's sclk and this tool reads its hwmon power.  A
store-bound kernel that runs at a lower sclk than the probe (power-capped by
its fp64 arithmetic) would show it here.

python tools/clock_compare.py [--workload c3|c2|cube] [--seconds 3]
"""
import argparse
import glob
import os
import sys
import threading
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from bpc_baseline_amd import ops  # noqa: E402
from bpc_baseline_amd.synth import make_scenes  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--workload", choices=["c3", "c2", "cube"], default="c3")
ap.add_argument("--seconds", type=float, default=3.0)
ap.add_argument("--rounds", type=int, default=2)
args = ap.parse_args()

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
if args.workload == "cube":
    b = make_scenes(250, 3, 256, seed=0)
    plan = ops.TripletPlan(b.cam_offs, b.n_scenes, device=dev)
    n_out = plan.n_cube
else:
    b = (make_scenes(1000, 3, 256, seed=0) if args.workload == "c2"
         else make_scenes(1000, 4, 1024, seed=0))
    plan = ops.PairwisePlan(b.cam_offs, b.n_scenes, b.n_cams, b.pairs, device=dev, row_align="auto")
    n_out = plan.dist_size
pts, co, F = (torch.from_numpy(x).to(dev) for x in (b.pts, b.cam_offs, b.F))
out = torch.empty(n_out, dtype=torch.float32, device=dev)
am = torch.empty(plan.n_rows, dtype=torch.int32, device=dev)
mv = torch.empty(plan.n_rows, dtype=torch.float32, device=dev)


def kernel():
    if args.workload == "cube":
        ops.triplet_cost_argmin(pts, co, F, plan, out=(out, am, mv))
    else:
        ops.pairwise_residual_argmin(pts, co, F, plan, out=(out, am, mv))


def probe():
    ops.hbm_write_probe(out)


dirs, _ = bench.drm_card_dirs(dev)
power_paths = [p for d in dirs for p in glob.glob(f"{d}/hwmon/hwmon*/power1_average")
               + glob.glob(f"{d}/hwmon/hwmon*/power1_input")]


class Power:
    def __init__(self):
        self.samples, self.stop = [], threading.Event()
        self.t = threading.Thread(target=self.run, daemon=True)

    def run(self):
        while not self.stop.is_set():
            for p in power_paths[:1]:
                try:
                    with open(p) as fh:
                        self.samples.append(int(fh.read()) / 1e6)   # microwatts -> W
                except (OSError, ValueError):
                    pass
            time.sleep(0.05)

    def __enter__(self):
        self.t.start()
        return self

    def __exit__(self, *exc):
        self.stop.set()
        self.t.join()


def measure(fn, name):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = 0
    with bench.ClockSampler(dev) as clk, Power() as pw:
        t_end = time.perf_counter() + args.seconds
        e0.record()
        while time.perf_counter() < t_end:
            for _ in range(10):
                fn()
            n += 10
            torch.cuda.synchronize()
        e1.record()
        torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / n
    s = clk.summary("sclk") or {}
    watts = sum(pw.samples) / len(pw.samples) if pw.samples else None
    gbs = 4 * n_out / (ms * 1e-3) / 1e9
    print(f"{name:>7}: {ms:.4f} ms per launch ({gbs:.0f} GB/s of output), sclk mean "
          f"{s.get('mean_mhz', float('nan')):.0f} MHz (min {s.get('min_mhz', float('nan'))}), "
          f"power {watts if watts is None else round(watts)} W ({len(pw.samples)} samples)",
          flush=True)


print(f"{args.workload}: {4 * n_out / 1e9:.2f} GB output per launch; power from "
      f"{power_paths[:1] or 'nothing (no hwmon power file)'}")
for r in range(args.rounds):
    measure(probe, "probe")
    measure(kernel, "kernel")
