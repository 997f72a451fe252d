"""Copy the summaries of a tools/gpu.sh run (RUN=<name>: gpurun_out/<name>/)
into profiles/<round>/ and derive profiles/pmc_traffic.json: HBM bytes per
launch from the separate FETCH_SIZE / WRITE_SIZE passes, FETCH_SIZE doubled
per the gfx950 correction in MI355X_MICROARCH.md §HBM.

    python tools/collect_profiles.py ROUND RUN_DIR     (e.g. r03 gpurun_out/g6)

Per workload W it takes whatever the run holds: bench_W.json and the
trace_W/ kernel statistics with window_W.json (tools/gpu.sh trace W), and
pmc_{FETCH,WRITE}_SIZE_W/ (tools/gpu.sh pmc W)."""
import csv
import json
import os
import shutil
import sys

ROUND, SRC = sys.argv[1], sys.argv[2]
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DST = os.path.join(REPO, "profiles", ROUND)
# the kernel that is one bench launch, per workload
OP_KERNELS = {"c3": ["pairwise_lazy_kernel<16, 1"],
              "c2": ["pairwise_lazy_kernel<16, 1"],
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


def copy(src, name):
    if os.path.exists(src):
        shutil.copy(src, os.path.join(DST, name))
        return True
    return False


os.makedirs(DST, exist_ok=True)
tpath = os.path.join(REPO, "profiles", "pmc_traffic.json")
traffic = json.load(open(tpath)) if os.path.exists(tpath) else {}
for w, kernels in OP_KERNELS.items():
    bench = os.path.join(SRC, f"bench_{w}.json")
    if not copy(bench, f"{w}_bench_line.json"):
        continue
    copy(os.path.join(SRC, f"trace_{w}", "run_kernel_stats.csv"), f"{w}_kernel_stats.csv")
    copy(os.path.join(SRC, f"window_{w}.json"), f"{w}_window.json")
    f = os.path.join(SRC, f"pmc_FETCH_SIZE_{w}", "run_counter_collection.csv")
    wr = os.path.join(SRC, f"pmc_WRITE_SIZE_{w}", "run_counter_collection.csv")
    if not (os.path.exists(f) and os.path.exists(wr)):
        continue
    shutil.copy(f, os.path.join(DST, f"{w}_pmc_fetch_size.csv"))
    shutil.copy(wr, os.path.join(DST, f"{w}_pmc_write_size.csv"))
    fkb, nf = per_launch(f, kernels, "FETCH_SIZE")
    wkb, nw = per_launch(wr, kernels, "WRITE_SIZE")
    line = json.loads([l for l in open(bench) if l.lstrip().startswith("{")][-1])
    traffic[w] = {
        "bytes_per_launch": fkb * 1024 * 2 + wkb * 1024,
        "fetch_bytes_corrected": fkb * 1024 * 2, "write_bytes": wkb * 1024,
        "fetch_size_kb_raw": fkb, "write_size_kb_raw": wkb, "launches": [nf, nw],
        "algorithmic_bytes_per_launch": line["roofline"]["bytes_per_launch"],
        "scenes_per_launch": line["config"]["scenes_per_launch"],
        "kernels": kernels,
        "source": f"rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes) of bench.py "
                  f"--workload {w}; per-launch mean over {kernels}; FETCH_SIZE x1024 x2 (gfx950), "
                  f"WRITE_SIZE x1024; profiles/{ROUND}/{w}_pmc_*.csv",
    }
    print(w, f"traffic {traffic[w]['bytes_per_launch'] / 1e9:.3f} GB vs algorithmic "
             f"{traffic[w]['algorithmic_bytes_per_launch'] / 1e9:.3f} GB per launch")
json.dump(traffic, open(tpath, "w"), indent=1)
