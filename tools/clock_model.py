"""C3 launch time against the shader clock: fit
t = a + b / f over every recorded line of the current C3 kernel (five
2,000-scene launches per step, rounds 4-6) and the driver's own records, and
split a launch at a given clock into its clock-independent part (a: the HBM
write path) and its clock-bound part (b / f: the fp64 VALU issue).

    python tools/clock_model.py [--at 1654] [--out profiles/r06/clock_model.json]

Driver records keep no sclk in BENCH_rNN.json's parsed line; their clocks are
the ones the round's VERDICT quotes from the driver's tail (r04 1.755 GHz,
r05 1.654 GHz)."""
import argparse
import glob
import json
import os

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DRIVER = {"BENCH_r04.json": 1755.0, "BENCH_r05.json": 1654.0}


def lines():
    out = []
    # the shipped kernel: round 4's final tree onward (round 4's bench_ab/
    # directories hold A/B builds and intermediate defaults)
    files = (glob.glob(os.path.join(REPO, "profiles", "r04", "final", "**", "*.json"), recursive=True)
             + glob.glob(os.path.join(REPO, "profiles", "r0[5-9]", "**", "*.json"), recursive=True))
    for f in sorted(files):
        try:
            txt = open(f).read()
        except OSError:
            continue
        for l in ([txt] + txt.splitlines()):
            l = l.strip()
            if not l.startswith("{"):
                continue
            try:
                d = json.loads(l)
            except ValueError:
                continue
            cfg = d.get("config") if isinstance(d, dict) else None
            if not isinstance(cfg, dict) or "4-cam x 1024" not in str(cfg.get("workload", "")):
                continue
            if cfg.get("scenes_per_launch") != 2000 or cfg.get("kernel_options") or d.get("n_gpus") != 1:
                continue
            sc, r = d.get("sclk") or {}, d.get("roofline") or {}
            if isinstance(sc, dict) and sc.get("mean_mhz") and r.get("avg_launch_ms"):
                out.append((os.path.relpath(f, REPO), float(sc["mean_mhz"]), float(r["avg_launch_ms"]),
                            r.get("write_probe_gbs")))
            break
    for f, mhz in DRIVER.items():
        p = json.load(open(os.path.join(REPO, f))).get("parsed") or {}
        ms = (p.get("roofline") or {}).get("avg_launch_ms")
        if ms:
            out.append((f + " (driver)", mhz, float(ms), (p.get("roofline") or {}).get("write_probe_gbs")))
    return out


ap = argparse.ArgumentParser()
ap.add_argument("--at", type=float, default=1654.0, help="clock (MHz) to split a launch at")
ap.add_argument("--out", default=None)
args = ap.parse_args()
pts = lines()
# a file and its copy (bench_c3.json / c3_bench_line.json of one run) count once
seen, uniq = set(), []
for p in pts:
    k = (round(p[1], 2), round(p[2], 5))
    if k not in seen:
        seen.add(k)
        uniq.append(p)
f = np.array([p[1] for p in uniq])
t = np.array([p[2] for p in uniq])
A = np.stack([np.ones_like(f), 1.0 / f], axis=1)
(a, b), res, *_ = np.linalg.lstsq(A, t, rcond=None)
pred = A @ np.array([a, b])
rms = float(np.sqrt(np.mean((pred - t) ** 2)))
share = (b / args.at) / (a + b / args.at)
d5 = (a + b / 1654.0) / (a + b / 1755.0) - 1.0
res = {"model": "t_ms = a + b / f_MHz per 2,000-scene C3 launch", "a_ms": a, "b_ms_MHz": b,
       "rms_ms": rms, "points": [{"source": s, "sclk_mhz": m, "ms": x, "write_probe_gbs": w}
                                  for s, m, x, w in uniq],
       "at_mhz": args.at, "valu_share_at": share,
       "predicted_ms_at": a + b / args.at,
       "slowdown_1755_to_1654": d5,
       "rule": "a C3 change is worth an A/B only if this model predicts >= 3% at the driver's clocks"}
for s, m, x, w in uniq:
    print(f"{m:8.1f} MHz {x:7.3f} ms  model {a + b / m:7.3f}  {s}")
print(f"t = {a:.3f} ms + {b:.1f} / f   (rms {rms:.3f} ms over {len(uniq)} lines)")
print(f"at {args.at:.0f} MHz: {a + b / args.at:.3f} ms, of which {share:.1%} scales with the clock; "
      f"1755 -> 1654 MHz costs {d5:.1%}")
if args.out:
    with open(args.out, "w") as fh:
        json.dump(res, fh, indent=1)
