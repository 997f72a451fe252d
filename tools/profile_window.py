"""Reconcile a bench line with the rocprofv3 kernel trace of the SAME process.

    python tools/profile_window.py BENCH_JSON KERNEL_TRACE_CSV [--out OUT.json]

bench.py records, for the dominant kernel, how many of its launches reached
the GPU before the timed region, in it and after it (roofline.dispatch_window).
This script takes the kernel's dispatches from the trace in dispatch order,
splits them into those three windows, and reports:
  * the kernel-trace statistics of the TIMED launches only (what the bench
    line's avg_launch_ms covers), the roofline fraction they give, and its
    ratio to the bench line's own fraction;
  * a per-output-allocation table: every launch of the run writes slot
    (launch index mod slots) -- warm-up launches from slot 0, the graph
    uploads and the timed launches from slot 0 again -- so each slot's first
    touch (its first warm-up launch), its later warm-up/upload launches and
    its timed launches are listed apart.
"""
from __future__ import annotations

import argparse
import csv
import json
import sys

import numpy as np


def load_line(path):
    with open(path) as fh:
        lines = [l for l in fh if l.lstrip().startswith("{")]
    return json.loads(lines[-1])


def kernel_durations(trace, name_part):
    rows = []
    with open(trace) as fh:
        for r in csv.DictReader(fh):
            if name_part in r["Kernel_Name"]:
                rows.append((int(r["Dispatch_Id"]), int(r["Start_Timestamp"]),
                             int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    return ([(e - s) * 1e-6 for _, s, e, _ in rows], sorted({r[3] for r in rows}),
            [(s, e) for _, s, e, _ in rows])


def stats(ms):
    a = np.asarray(ms, dtype=np.float64)
    if a.size == 0:
        return None
    return {"launches": int(a.size), "avg_ms": float(a.mean()), "min_ms": float(a.min()),
            "max_ms": float(a.max()), "median_ms": float(np.median(a)),
            "std_ms": float(a.std())}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("bench_json")
    ap.add_argument("trace_csv")
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    line = load_line(args.bench_json)
    rf = line["roofline"]
    w = rf["dispatch_window"]
    name = w["kernel"] + "<"
    durs, names, spans = kernel_durations(args.trace_csv, name)
    before, timed, after = w["before"], w["timed"], w["after"]
    if len(durs) != before + timed + after:
        sys.exit(f"trace has {len(durs)} {name} dispatches, the bench line expects "
                 f"{before} + {timed} + {after}")
    L, S = w["launches_per_step"], w["slots"]
    warm = line["warmup"] * L                 # eager warm-up launches (slots from 0)
    t_ms = durs[before:before + timed]
    st = stats(t_ms)
    bpl = rf["bytes_per_launch"]
    frac_trace = bpl / (st["avg_ms"] * 1e-3) / 1e9 / rf["peak"]
    # the timed launches' span (first start to last end) per launch: the
    # period the trace shows when launches overlap (--graph steps2: even and
    # odd steps on two streams), where a launch's own duration includes the
    # time it shared the GPU with its neighbour
    ts = spans[before:before + timed]
    span_ms = (max(e for _, e in ts) - min(s for s, _ in ts)) * 1e-6 / timed
    frac_span = bpl / (span_ms * 1e-3) / 1e9 / rf["peak"]
    per_slot = []
    for s in range(S):
        first = [durs[n] for n in range(warm) if n % S == s][:1]
        rest_warm = [durs[n] for n in range(warm) if n % S == s][1:]
        upload = [durs[warm + n] for n in range(before - warm) if n % S == s]
        tim = [t_ms[n] for n in range(timed) if n % S == s]
        per_slot.append({"slot": s, "first_touch_ms": first[0] if first else None,
                         "warmup_retouch_ms": float(np.mean(rest_warm)) if rest_warm else None,
                         "untimed_replay_ms": float(np.mean(upload)) if upload else None,
                         "timed_avg_ms": float(np.mean(tim)) if tim else None,
                         "timed_min_ms": float(np.min(tim)) if tim else None,
                         "timed_max_ms": float(np.max(tim)) if tim else None,
                         "timed_launches": len(tim)})
    out = {
        "kernel": names,
        "bench": {"value": line["value"], "ms_per_step": line["ms_per_step"],
                  "avg_launch_ms": rf["avg_launch_ms"], "frac": rf["frac"],
                  "event_scope": rf["event_scope"], "launch_mode": line["config"].get("launch_mode")},
        "window": w,
        "all_launches": stats(durs),
        "timed": st,
        "timed_frac_of_peak_from_trace": frac_trace,
        "trace_vs_bench_frac": frac_trace / rf["frac"],
        "timed_span_per_launch_ms": span_ms,
        "span_frac_of_peak_from_trace": frac_span,
        "span_vs_bench_frac": frac_span / rf["frac"],
        "timed_sum_per_step_ms": st["avg_ms"] * L,
        "before": stats(durs[:before]),
        "after": stats(durs[before + timed:]),
        "per_slot": per_slot,
    }
    txt = json.dumps(out, indent=1)
    if args.out:
        with open(args.out, "w") as fh:
            fh.write(txt + "\n")
    print(f"timed {st['launches']} launches: avg {st['avg_ms']:.4f} ms (min {st['min_ms']:.4f}, "
          f"max {st['max_ms']:.4f}); frac from trace {frac_trace:.4f} vs bench {rf['frac']:.4f} "
          f"(ratio {frac_trace / rf['frac']:.4f}); {L} x avg = {st['avg_ms'] * L:.3f} ms vs "
          f"ms_per_step {line['ms_per_step']:.3f}; span {span_ms:.4f} ms per launch, frac "
          f"{frac_span:.4f} (ratio {frac_span / rf['frac']:.4f})")
    for p in per_slot:
        print("  slot %2d  first %s  retouch %s  replay %s  timed %s (%s..%s, n=%d)" % (
            p["slot"], *("%.3f" % v if v is not None else "  -  " for v in (
                p["first_touch_ms"], p["warmup_retouch_ms"], p["untimed_replay_ms"],
                p["timed_avg_ms"], p["timed_min_ms"], p["timed_max_ms"])), p["timed_launches"]))


if __name__ == "__main__":
    main()
