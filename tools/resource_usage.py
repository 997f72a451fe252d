"""Per-kernel register / spill / occupancy table of one HIP source, from the
compiler's kernel-resource-usage remarks (gfx950, the build's flags).

python tools/resource_usage.py bpc_baseline_amd/csrc/mvm_pairwise.hip [--filter pairwise_kernel]
"""
import argparse
import os
import re
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import __graft_entry__ as G  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("src")
ap.add_argument("--filter", default="")
ap.add_argument("--asm", default="", help="also write the device assembly here")
ap.add_argument("-D", dest="defs", action="append", default=[], help="extra -D macro")
args = ap.parse_args()

flags = [f for f in G.HIPCC_FLAGS if f not in ("-shared", "-fPIC")]
cmd = [G._hipcc(), *flags, "-I" + os.path.join(G.PKG, "csrc"), "--cuda-device-only", "-S",
       *("-D" + d for d in args.defs), "-o", args.asm or os.devnull, args.src, "-Rpass-analysis=kernel-resource-usage"]
out = subprocess.run(cmd, capture_output=True, text=True)
if out.returncode:
    sys.exit("\n".join(l for l in out.stderr.splitlines() if "error" in l)[:3000])
rows, cur = [], None
for line in out.stderr.splitlines():
    m = re.search(r"remark: (?:\s*)([^:\[]+?): (\S+) \[", line)
    if not m:
        continue
    key, val = m.group(1).strip(), m.group(2)
    if key == "Function Name":
        dm = subprocess.run(["c++filt", val], capture_output=True,
                            text=True).stdout.strip()
        cur = {"name": dm.replace("(anonymous namespace)::", "")}
        rows.append(cur)
    elif cur is not None:
        cur[key] = val
keys = ["VGPRs", "AGPRs", "TotalSGPRs", "VGPRs Spill", "SGPRs Spill", "ScratchSize [bytes/lane]",
        "Occupancy [waves/SIMD]", "LDS Size [bytes/block]"]
short = ["vgpr", "agpr", "sgpr", "vspill", "sspill", "scratch", "occ", "lds"]
print("  ".join(f"{s:>7}" for s in short), " kernel")
for r in rows:
    if args.filter and args.filter not in r["name"]:
        continue
    print("  ".join(f"{r.get(k, '-'):>7}" for k in keys), "", r["name"][:110])
