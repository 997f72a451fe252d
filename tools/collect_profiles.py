"""Copy the rocprofv3 summaries of a gpu_bench.sh run from gpurun_out/ into
profiles/<round>/ and derive profiles/pmc_traffic.json (HBM bytes per launch
from separate FETCH_SIZE / WRITE_SIZE passes; FETCH_SIZE doubled per the gfx950
correction in MI355X_MICROARCH.md §HBM).  Usage: python tools/collect_profiles.py r01"""
import csv
import json
import os
import shutil
import sys

ROUND = sys.argv[1] if len(sys.argv) > 1 else "r01"
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(REPO, "gpurun_out")
DST = os.path.join(REPO, "profiles", ROUND)
# kernels that together form one bench launch (the op), per workload
OP_KERNELS = {"c3": ["pairwise_kernel<16, true, float, 1"],
              "c2": ["pairwise_kernel<16, true, float, 1"],
              "c2cube": ["triplet_fused_kernel"]}


def per_launch(path, kernels, counter):
    vals = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        for k in kernels:
            if k in r["Kernel_Name"]:
                vals.setdefault(k, []).append(float(r["Counter_Value"]))
    return sum(sum(v) / len(v) for v in vals.values()), {k: len(v) for k, v in vals.items()}


os.makedirs(DST, exist_ok=True)
traffic = {}
tpath = os.path.join(REPO, "profiles", "pmc_traffic.json")
if os.path.exists(tpath):
    traffic = json.load(open(tpath))
for w, kernels in OP_KERNELS.items():
    bench = os.path.join(SRC, f"bench_{w}.json")
    if not os.path.exists(bench):
        continue
    shutil.copy(bench, os.path.join(DST, f"{w}_bench_line.json"))
    shutil.copy(os.path.join(SRC, f"prof_{w}", "run_kernel_stats.csv"),
                os.path.join(DST, f"{w}_kernel_stats.csv"))
    f = os.path.join(SRC, f"pmc_fetch_{w}", "run_counter_collection.csv")
    wr = os.path.join(SRC, f"pmc_write_{w}", "run_counter_collection.csv")
    shutil.copy(f, os.path.join(DST, f"{w}_pmc_fetch_size.csv"))
    shutil.copy(wr, os.path.join(DST, f"{w}_pmc_write_size.csv"))
    fkb, nf = per_launch(f, kernels, "FETCH_SIZE")
    wkb, nw = per_launch(wr, kernels, "WRITE_SIZE")
    line = json.load(open(bench))
    traffic[w] = {
        "bytes_per_launch": fkb * 1024 * 2 + wkb * 1024,
        "fetch_bytes_corrected": fkb * 1024 * 2, "write_bytes": wkb * 1024,
        "fetch_size_kb_raw": fkb, "write_size_kb_raw": wkb, "launches": [nf, nw],
        "algorithmic_bytes_per_launch": line["roofline"]["bytes_per_launch"],
        "scenes_per_launch": line["config"]["scenes_per_launch"],
        "kernels": kernels,
        "source": f"rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes) of bench.py "
                  f"--workload {w}; per-launch sum over {kernels}; FETCH_SIZE x1024 x2 (gfx950), "
                  f"WRITE_SIZE x1024; profiles/{ROUND}/{w}_pmc_*.csv",
    }
    print(w, f"traffic {traffic[w]['bytes_per_launch']/1e9:.3f} GB vs algorithmic "
             f"{traffic[w]['algorithmic_bytes_per_launch']/1e9:.3f} GB per launch")
json.dump(traffic, open(tpath, "w"), indent=1)
