"""Per-launch SQ counter summary of one kernel from a rocprofv3 --pmc run
(tools/gpu.sh sq ...): mean over the kernel's launches, plus VALU
lane-instructions per unit of work and wait/active.

python tools/summarise_sq.py COUNTER_CSV KERNEL_PART UNITS_PER_LAUNCH [--what TEXT] [--out OUT.json]
"""
import argparse
import csv
import json
from collections import defaultdict

ap = argparse.ArgumentParser()
ap.add_argument("csv")
ap.add_argument("kernel")
ap.add_argument("units", type=float, help="pairs (or triples) one launch computes")
ap.add_argument("--what", default="")
ap.add_argument("--out", default=None)
args = ap.parse_args()

per = defaultdict(lambda: defaultdict(float))   # dispatch -> counter -> value (summed over dims)
meta = {}
for r in csv.DictReader(open(args.csv)):
    if args.kernel not in r["Kernel_Name"]:
        continue
    d = r["Dispatch_Id"]
    per[d][r["Counter_Name"]] += float(r["Counter_Value"])
    meta = {"kernel": r["Kernel_Name"], "vgpr_count_rocprof": r.get("Arch_VGPR_Count") or r.get("VGPR_Count"), "sgpr": r.get("SGPR_Count"),
            "scratch": r.get("Scratch_Size"), "lds": r.get("LDS_Block_Size"), "grid": r.get("Grid_Size")}
names = sorted({c for d in per.values() for c in d})
mean = {c: sum(d[c] for d in per.values()) / len(per) for c in names}
out = {"what": args.what, **meta, "launches": len(per), "counters": mean}
if "SQ_INSTS_VALU" in mean:
    out["valu_lane_instr_per_unit"] = mean["SQ_INSTS_VALU"] * 64 / args.units
if "SQ_WAVES" in mean and "SQ_INSTS_VALU" in mean:
    out["valu_per_wave"] = mean["SQ_INSTS_VALU"] / mean["SQ_WAVES"]
if "SQ_WAIT_INST_ANY" in mean and "SQ_ACTIVE_INST_ANY" in mean:
    out["wait_over_active"] = mean["SQ_WAIT_INST_ANY"] / mean["SQ_ACTIVE_INST_ANY"]
txt = json.dumps(out, indent=1)
print(txt)
if args.out:
    open(args.out, "w").write(txt + "\n")
