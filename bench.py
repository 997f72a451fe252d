#!/usr/bin/env python3
"""Benchmark of the MI355X multi-view epipolar matcher (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c3|c2|c2cube|c2match]

A *step* is one pass of the hot path over this rank's whole batch of
synthetic scenes (resident in HBM): pairwise symmetric epipolar residuals for
every (scene, camera pair, detection_i, detection_j), written as float32
matrices, plus the per-row argmin association; for N > 1 the step ends with
the single gather of every rank's association rows to rank 0 (RCCL/xGMI).

Default workload (``c3``, BASELINE.json configs[2], the configuration the
@1/2/4/8-GPU metric is quoted on via configs[3]): 4 cameras x 1024
detections/view x 10,000 scenes, 6 camera pairs -> 6.29e10 detection pairs
per step.  With N GPUs the 10,000 scenes are split over the ranks (strong
scaling, the default), so ``--gpus 8`` is configs[3]: 1,250 scenes per GPU;
``--scaling weak`` gives every rank its own 10,000.  Scenes are processed in
launches of at most ``--chunk`` scenes, at least ``--min-launches`` per rank
(5 with N > 1: the gather piece of launch k overlaps launch k+1, so only the
last piece is exposed, and that last launch is a short one, ~1/4 of the
others); every residual is stored to HBM.  At every N each
launch of each timed step of C3 is a hipGraph captured outside the timed
region and replayed in order, with N > 1 followed by its gather piece, so the
1 -> N curve compares the same launch path (``--graph steps2``, the default
for C2 on one GPU: one graph for all K steps, even and odd steps on two
streams; ``--graph steps``: the same on one stream; ``--graph off``: eager op
calls).

``python bench.py --gpus N`` (N > 1) run without a launcher starts the N
ranks itself: torchrun in a child process, this process making no GPU call;
every rank checks that the process group it joined has N ranks.  After the
timed region every association row of the last step -- all ranks' rows, as
gathered to rank 0 -- is compared with the CPU oracle (``parity_rows``).
By default every launch of the timed steps writes its own output allocation
as far as HBM holds them (C3: five launches of 2,000 scenes into five 50 GB
buffers, 253 GB, one per launch of a step; C2: one per step), taken round
robin, so a step's outputs all stay resident and the measurement covers much
of the HBM rather than wherever one launch-sized buffer happened to land (the
same launch runs up to ~20% apart on different allocations: DESIGN.md §5);
``--output ring`` reuses one buffer.  The first scene of the launch each
allocation last held is compared with the oracle bit for bit (``parity``).

``--workload c2match`` times what ``match_objects`` returns at C2 scale (cube +
scipy-identical assignment + threshold/sort/DLT, units = captures).

Printed by rank 0: ONE JSON line with value = total pairs/s over all ranks,
the dominant kernel's roofline (achieved algorithmic GB/s from HIP events on
the launch stream vs the 8 TB/s HBM peak) and a CPU baseline (the C/OpenMP
restatement in oracle/, timed on a bounded sample on this host).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

from bpc_baseline_amd.distributed import (ChunkedRowGather, gather_rows, init_from_env,  # noqa: E402
                                          max_over_ranks, sum_over_ranks)
from bpc_baseline_amd.synth import make_scenes  # noqa: E402

ops = None   # bpc_baseline_amd.ops, imported by main() once this process is a rank

HBM_PEAK_GBS = 8000.0      # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
METRIC = "detection-pairs matched/sec"

WORKLOADS = {
    # C3 launches of 2,000 scenes (50.6 GB of matrices): 1.66e12 pairs/s on
    # two boxes against 1.57-1.62e12 with 1,000 (fewer launch tails, five
    # output allocations instead of eleven; profiles/r04/bench_ab/chunk/)
    "c3": dict(n_cams=4, n_dets=1024, n_scenes=10000, chunk=2000, mode="pairwise",
               desc="C3: synthetic IPD-like 4-cam x 1024 dets/view x 10000 scenes per GPU, "
                    "pairwise residual matrices + per-row argmin"),
    "c2": dict(n_cams=3, n_dets=256, n_scenes=1000, chunk=1000, mode="pairwise",
               desc="C2: synthetic IPD-like 3-cam x 256 dets/view x 1000 scenes per GPU, "
                    "pairwise residual matrices + per-row argmin"),
    # the cube step as one 16.9 GB launch: 1.76-1.77e12 triples/s against
    # 1.63-1.66e12 as four of 250 scenes (profiles/r04/bench_ab/chunk/)
    "c2cube": dict(n_cams=3, n_dets=256, n_scenes=1000, chunk=1000, mode="cube",
                   desc="C2 cube: 3-cam x 256 dets/view x 1000 scenes per GPU, "
                        "compute_cost_matrix cubes + per-(i,j) argmin (units = triples)"),
    # what match_objects returns at C2 scale: cube + Hungarian + select/DLT
    "c2match": dict(n_cams=3, n_dets=256, n_scenes=1000, chunk=1000, mode="match", threshold=30.0,
                    desc="C2 match: 3-cam x 256 dets/view x 1000 scenes per GPU: "
                         "compute_cost_matrix cubes, scipy-identical linear_sum_assignment of "
                         "every (N*M, P) cube, threshold + cost sort + DLT (units = captures)"),
}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def pairwise_bytes(counts: np.ndarray, pairs: np.ndarray) -> float:
    """Algorithmic HBM bytes of one pairwise launch:
    16 B per centroid read + 72 B per F + per pair matrix 4 B/pair + 8 B/row."""
    na = counts[:, pairs[:, 0]].astype(np.float64)
    nb = counts[:, pairs[:, 1]].astype(np.float64)
    return float(16.0 * counts.sum() + 72.0 * na.size + (4.0 * na * nb + 8.0 * na).sum())


def cube_bytes(counts: np.ndarray) -> float:
    """Cube launch: centroids + 3 F + 4 B/triple + 8 B per (i,j) row."""
    N, M, P = (counts[:, k].astype(np.float64) for k in range(3))
    return float(16.0 * counts.sum() + 3 * 72.0 * len(N) + (4.0 * N * M * P + 8.0 * N * M).sum())


class Chunk:
    def __init__(self, s0, pts, cam_offs, F, plan, row_base, units, size, nbytes):
        self.s0 = s0
        self.pts, self.cam_offs, self.F, self.plan = pts, cam_offs, F, plan
        self.row_base, self.units, self.nbytes = row_base, units, nbytes
        self.size = size          # output floats (>= units when rows are pitched)


def build_chunks(batch, bounds, device, mode):
    C, P = batch.n_cams, batch.n_pairs
    pts_all = torch.from_numpy(batch.pts).to(device)
    F_all = torch.from_numpy(batch.F).to(device)
    counts = batch.counts()
    chunks, row_base = [], 0
    for s0, s1 in bounds:
        co = batch.cam_offs[s0 * C:s1 * C + 1]
        base = int(co[0])
        co_rel = (co - base).astype(np.int64)
        pts = pts_all[base:int(co[-1])]
        F = F_all[s0 * P:s1 * P]
        if mode == "pairwise":
            plan = ops.PairwisePlan(co_rel, s1 - s0, C, batch.pairs, device=device, row_align="auto")
            units, size = int(plan.n_dist), int(plan.dist_size)
            nbytes = pairwise_bytes(counts[s0:s1], batch.pairs)
        else:
            plan = ops.TripletPlan(co_rel, s1 - s0, device=device)
            units = size = int(plan.n_cube)
            nbytes = cube_bytes(counts[s0:s1])
        chunks.append(Chunk(s0, pts, torch.from_numpy(co_rel).to(device), F, plan, row_base, units,
                            size, nbytes))
        chunks[-1].idx = len(chunks) - 1
        row_base += plan.n_rows
    return chunks, row_base


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_threads() -> int:
    """This rank's threads (affinity, capped by OMP_NUM_THREADS): what the
    post-timing oracle runs of every rank use side by side."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit():
        n = min(n, int(omp))
    return max(1, int(n))


def host_cpu_threads() -> tuple:
    """Threads of the CPU baseline, the same at every N: the host cores this
    process may use (affinity, capped by the cgroup's CPU quota) capped by the
    OMP_NUM_THREADS the *host* sets.  A launcher's per-rank value is ignored:
    ``launch_ranks`` hands the host's own value down as MVM_HOST_OMP_THREADS,
    and torchrun's injected OMP_NUM_THREADS=1 at world > 1 is not a host
    setting.  -> (threads, how they were chosen)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    src = [f"affinity {n}"]
    try:
        with open("/sys/fs/cgroup/cpu.max") as fh:
            quota, period = fh.read().split()[:2]
        if quota != "max":
            q = max(1, -(-int(quota) // int(period)))
            n = min(n, q)
            src.append(f"cgroup quota {q}")
    except (OSError, ValueError):
        pass
    omp = os.environ.get("MVM_HOST_OMP_THREADS")
    if omp is None:
        omp = os.environ.get("OMP_NUM_THREADS")
        if omp == "1" and int(os.environ.get("WORLD_SIZE", "1")) > 1:
            omp = None                       # torchrun's per-rank default, not the host's
    if omp and omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
        src.append(f"host OMP_NUM_THREADS {omp}")
    return max(1, int(n)), ", ".join(src)


def cpu_baseline(batch, mode: str, target_s: float):
    """Time the C/OpenMP restatement (oracle/, test infrastructure) on a bounded
    sample of this workload's scenes -> dict for the JSON line."""
    from oracle import oracle as O
    threads, threads_src = host_cpu_threads()
    C = batch.n_cams

    def run(n_sc, nthreads=threads):
        co = batch.cam_offs[:n_sc * C + 1]
        pts = batch.pts[:int(co[-1])]
        t0 = time.perf_counter()
        if mode == "pairwise":
            d, _, _, _, _ = O.pairwise(pts, co, batch.F[:n_sc * batch.n_pairs], batch.pairs, n_sc, C,
                                       nthreads=nthreads)
            units = d.size
        else:
            c, _, _, _, _ = O.cube(pts, co, batch.F[:n_sc * 3], n_sc, nthreads=nthreads)
            units = c.size
        return units, time.perf_counter() - t0

    run(1)                                           # warm (page-in, thread pool)
    u1, t1 = run(min(batch.n_scenes, max(1, threads)))
    per_scene = t1 / min(batch.n_scenes, max(1, threads))
    n_sc = int(min(batch.n_scenes, max(1, round(target_s / max(per_scene, 1e-9)))))
    units, secs = run(n_sc)
    # one core, on a sample ~1/4 as long
    n1 = int(min(batch.n_scenes, max(1, round(target_s / 4 / max(per_scene * threads, 1e-9)))))
    u1, s1 = run(n1, 1)
    unit = "pairs/s" if mode == "pairwise" else "triples/s"
    extra = {}
    if mode == "pairwise":
        # the vectorised NumPy restatement, one process, ~2 s sample
        from oracle import numpy_port as NP
        t0 = time.perf_counter()
        NP.pairwise(batch.pts, batch.cam_offs, batch.F, batch.pairs, 1, C)
        per = time.perf_counter() - t0
        nn = int(min(batch.n_scenes, max(1, round(min(2.0, target_s / 4) / max(per, 1e-9)))))
        t0 = time.perf_counter()
        dn, _ = NP.pairwise(batch.pts, batch.cam_offs, batch.F, batch.pairs, nn, C)
        sn = time.perf_counter() - t0
        extra = {"numpy_value": dn.size / sn,
                 "numpy_sample": f"{nn} scenes in {sn:.1f} s, oracle/numpy_port.py (vectorised NumPy, "
                                 f"one process; no FMA, so a timing baseline)"}
    # the reference's own cost model: one small-array NumPy evaluation per pair
    # in Python loops (oracle/reference_loop.py, bit-exact to the reference)
    from oracle import reference_loop as RL
    co = batch.cam_offs
    if mode == "pairwise":
        a, b = batch.pairs[0]
        n_ref, s_ref = RL.pairs_per_second(batch.pts[co[a]:co[a + 1]], batch.pts[co[b]:co[b + 1]],
                                           batch.F[0], seconds=2.0)
    else:
        views = [batch.pts[co[v]:co[v + 1]][:8] for v in range(3)]
        Fs = [np.asarray(batch.F[q], np.float64).reshape(3, 3) for q in range(3)]
        n_ref, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < 2.0:
            n_ref += RL.cube(*views, *Fs).size
        s_ref = time.perf_counter() - t0
    extra["reference_loop_value"] = n_ref / s_ref if s_ref else None
    extra["reference_loop_sample"] = (f"{n_ref} {unit[:-2]} in {s_ref:.1f} s, oracle/reference_loop.py "
                                      "(the reference's per-pair NumPy calls in Python loops, one core)")
    return {"value": units / secs, "unit": unit, "cores": threads, "cores_at_n1": threads,
            "cores_source": threads_src + " (independent of the rank count)", "kind": "port",
            "one_core_value": u1 / s1, "one_core_sample": f"{n1} scenes in {s1:.1f} s", **extra,
            "sample": f"{n_sc} scenes ({units:.3g} {unit[:-2]}) of this workload in {secs:.1f} s, "
                      f"oracle/mvm_oracle.c fp64 restatement (bit-exact to the reference), "
                      f"OpenMP x{threads} on {cpu_model()}"}


def drm_card_dirs(device: torch.device):
    """The /sys/class/drm/card*/device directory of ``device`` (matched by PCI
    address), and a description of the match.  Falls back to every card when
    the address cannot be matched (then the clocks are max over cards)."""
    import glob
    cards = sorted(glob.glob("/sys/class/drm/card[0-9]*/device"))
    try:
        p = torch.cuda.get_device_properties(device)
        addr = f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}"
    except (AttributeError, RuntimeError, AssertionError):
        addr = None
    if addr:
        mine = [c for c in cards if os.path.basename(os.path.realpath(c)).startswith(addr)]
        if mine:
            return mine, f"card of PCI {addr}"
    return cards, "max over visible cards (PCI address not matched)"


class ClockSampler:
    """Samples the GPU's current clock levels (the starred line of
    /sys/class/drm/cardN/device/pp_dpm_{sclk,mclk,fclk}) of the card under
    test on a host thread while the timed region runs, so run-to-run and
    box-to-box spread can be attributed to clocks or not."""

    KINDS = ("sclk", "mclk", "fclk")

    def __init__(self, device: torch.device, period_s: float = 0.05):
        import glob
        import threading
        dirs, self.card_source = drm_card_dirs(device)
        self.paths = {k: [os.path.join(d, f"pp_dpm_{k}") for d in dirs
                          if os.path.exists(os.path.join(d, f"pp_dpm_{k}"))]
                      for k in self.KINDS}
        self.period = period_s
        self.samples = {k: [] for k in self.KINDS}
        # hwmon temperatures by label (edge / junction / mem), degrees C
        self.temp_paths = {}
        for lab in sorted(l for d in dirs for l in glob.glob(f"{d}/hwmon/hwmon*/temp*_label")):
            try:
                with open(lab) as fh:
                    name = fh.read().strip()
            except OSError:
                continue
            self.temp_paths.setdefault(name, []).append(lab[:-len("label")] + "input")
        self.temps = {k: [] for k in self.temp_paths}
        self.stop_ev = threading.Event()
        self.thread = threading.Thread(target=self._run, daemon=True)

    @staticmethod
    def _read(paths):
        vals = []
        for p in paths:
            try:
                with open(p) as fh:
                    for line in fh:
                        if line.rstrip().endswith("*"):
                            vals.append(int(line.split(":")[1].strip().split("Mhz")[0].split("MHz")[0]))
            except (OSError, ValueError, IndexError):
                pass
        return max(vals) if vals else None

    def _run(self):
        while not self.stop_ev.is_set():
            for k in self.KINDS:
                v = self._read(self.paths[k])
                if v is not None:
                    self.samples[k].append(v)
            for name, paths in self.temp_paths.items():
                vals = []
                for p in paths:
                    try:
                        with open(p) as fh:
                            vals.append(int(fh.read().strip()) / 1000.0)
                    except (OSError, ValueError):
                        pass
                if vals:
                    self.temps[name].append(max(vals))
            self.stop_ev.wait(self.period)

    def __enter__(self):
        if any(self.paths.values()):
            self.thread.start()
        return self

    def __exit__(self, *exc):
        self.stop_ev.set()
        if self.thread.is_alive():
            self.thread.join()

    def temperatures(self):
        """Per hwmon label of the card under test, first and last sample of the
        timed region (degrees C): HBM above ~85 C refreshes twice as often."""
        out = {}
        for name, v in self.temps.items():
            if v:
                out[name] = {"first_c": v[0], "last_c": v[-1], "max_c": max(v)}
        return out or None

    def summary(self, kind: str = "sclk"):
        if not self.samples[kind]:
            return {"source": f"pp_dpm_{kind} unreadable", "samples": 0}
        s = np.asarray(self.samples[kind], dtype=np.float64)
        return {"source": f"pp_dpm_{kind} (starred level, {self.card_source})",
                "samples": int(s.size), "mean_mhz": float(s.mean()), "min_mhz": float(s.min()),
                "max_mhz": float(s.max())}


def output_slots(n_launch: int, slot_bytes: int, free_bytes: int,
                 reserve_bytes: int = 8 << 30) -> int:
    """Output allocations for a step: one per launch when HBM holds them with
    ``reserve_bytes`` to spare, else as many as fit (launches reuse them round
    robin), never fewer than one."""
    fit = (free_bytes - reserve_bytes) // slot_bytes if slot_bytes > 0 else n_launch
    return int(max(1, min(n_launch, fit)))


def load_traffic(workload: str, scenes_per_launch: int):
    """PMC-measured HBM bytes per launch (profiles/pmc_traffic.json), only if it
    was collected on this workload at this launch size."""
    path = os.path.join(REPO, "profiles", "pmc_traffic.json")
    try:
        with open(path) as fh:
            rec = json.load(fh).get(workload)
    except (OSError, ValueError):
        return None
    if not rec or int(rec.get("scenes_per_launch", -1)) != int(scenes_per_launch):
        return None
    return rec


def launch_bounds(n_local: int, chunk: int, min_launches: int, tail_frac: float = 0.0):
    """[(s0, s1)] scene ranges of a rank's launches: as few as keep each at
    most ``chunk`` scenes, but at least ``min_launches`` (never more than one
    per scene), sizes differing by at most one.  With N > 1 the association
    gather of launch k overlaps launch k+1, so only the last launch's piece is
    exposed: more launches per rank make that tail smaller (configs[3]: 1,250
    scenes per rank -> 5 x 250, not 2 x 625).  ``tail_frac`` > 0 adds one
    short last launch of about that fraction of the others (configs[3]:
    5 x 238 + 62), so the exposed piece shrinks with it."""
    from bpc_baseline_amd.distributed import shard_range
    n_launch = max(1, -(-n_local // chunk), min(min_launches, n_local))
    tail = 0
    if tail_frac > 0 and n_local > n_launch:
        tail = max(1, int(round(n_local / n_launch * tail_frac)))
    main = [shard_range(n_local - tail, k, n_launch) for k in range(n_launch)]
    return main + ([(n_local - tail, n_local)] if tail else [])


def compare_rows_streamed(env, ref_am: np.ndarray, ref_mv: np.ndarray, g_am, g_mv):
    """Every rank's oracle rows against rank 0's gathered rows, bit for bit.

    Rank r (> 0) sends its oracle rows to rank 0 over the host (gloo) group,
    one rank at a time, and rank 0 compares them with rank r's slice of what
    the step's gather delivered: rank 0 holds at most one other rank's rows
    at once (not the whole job's).  -> (rows, rows equal, first unequal
    global row or None) on rank 0; (0, 0, None) elsewhere."""
    if not env.initialised:
        total = int(ref_am.size)
        if g_am.size != total:
            return total, 0, 0
        eq = (g_am == ref_am) & (g_mv.view(np.int32) == ref_mv.view(np.int32))
        bad = np.flatnonzero(~eq)
        return total, int(eq.sum()), (int(bad[0]) if bad.size else None)
    import torch.distributed as dist
    grp = env.cpu_group()
    n = torch.tensor([ref_am.size], dtype=torch.int64)
    sizes = [torch.zeros_like(n) for _ in range(env.world)]
    dist.all_gather(sizes, n, group=grp)
    sizes = [int(s.item()) for s in sizes]
    if not env.is_root:
        dist.send(torch.from_numpy(np.ascontiguousarray(ref_am)), dst=0, group=grp)
        dist.send(torch.from_numpy(np.ascontiguousarray(ref_mv)), dst=0, group=grp)
        return 0, 0, None
    total, ok, first_bad, base = sum(sizes), 0, None, 0
    for r, nr in enumerate(sizes):
        if r == 0:
            am, mv = ref_am, ref_mv
        else:
            am_t = torch.empty(nr, dtype=torch.int32)
            mv_t = torch.empty(nr, dtype=torch.float32)
            dist.recv(am_t, src=r, group=grp)
            dist.recv(mv_t, src=r, group=grp)
            am, mv = am_t.numpy(), mv_t.numpy()
        if g_am.size == total:
            ga, gm = g_am[base:base + nr], g_mv[base:base + nr]
            eq = (ga == am) & (gm.view(np.int32) == mv.view(np.int32))
            ok += int(eq.sum())
            bad = np.flatnonzero(~eq)
            if bad.size and first_bad is None:
                first_bad = base + int(bad[0])
        elif first_bad is None:
            first_bad = 0
        base += nr
    return total, ok, first_bad


def launch_ranks(n: int) -> int:
    """``--gpus N`` (N > 1) started without a launcher: run this same command
    as N ranks under torchrun in a CHILD process (this parent has made no GPU
    call and makes none), its output streamed through, and return its exit
    code.  Rendezvous on 127.0.0.1, one rank per GPU (each rank checks that)."""
    import signal
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")     # dmabuf IPC (RCCL)
    # the host's own thread setting, for rank 0's CPU baseline after the timed
    # region (the same at every N); each rank's OpenMP gets a share of the host
    env["MVM_HOST_OMP_THREADS"] = str(host_cpu_threads()[0])
    if "OMP_NUM_THREADS" not in env:                     # torchrun would set 1
        env["OMP_NUM_THREADS"] = str(max(1, min(16, cpu_threads() // n)))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node",
           str(n), "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.abspath(__file__), *sys.argv[1:]]
    log(f"launching {n} ranks: {' '.join(cmd)}")
    proc = subprocess.Popen(cmd, env=env)

    def forward(signum, _frame):
        proc.send_signal(signum)
    for sig in (signal.SIGTERM, signal.SIGINT):
        signal.signal(sig, forward)
    rc = proc.wait()
    if rc != 0:
        log(f"error: the {n}-rank run exited with status {rc}")
    return rc


def match_cpu_chain(batch, proj, s: int, threshold: float, nthreads: int = 1):
    """Scene s through the CPU restatements, as the reference computes it
    (epipolar_matching.py:83-116, process_pose.py:182-187): the oracle cube
    (C), the assignment (scipy, the reference's own call; oracle/lsap.py's
    restatement of it when scipy is absent), threshold, stable sort by cost,
    DLT (numpy SVD).  -> (cube, row_ind, col_ind, matches, X)."""
    from oracle import oracle as O
    from oracle import pipeline as OP
    try:
        from scipy.optimize import linear_sum_assignment as lsa
    except ImportError:                                     # pragma: no cover
        from oracle.lsap import linear_sum_assignment as lsa
    co = batch.cam_offs[3 * s:3 * s + 4]
    pts = batch.pts[int(co[0]):int(co[3])]
    n = np.diff(co)
    cube = O.cube(pts, co - co[0], batch.F[3 * s:3 * s + 3], 1, nthreads=nthreads)[0]
    flat = cube.reshape(n[0] * n[1], n[2])
    r, c = lsa(flat)
    m = [(int(i) // n[1], int(i) % n[1], int(k)) for i, k in zip(r, c) if flat[i, k] < threshold]
    m = sorted(m, key=lambda t: cube.reshape(n)[t])
    rel = co[:3] - co[0]
    X = (OP.triangulate(np.repeat(proj[s][None], len(m), 0),
                        np.stack([pts[rel + np.array(t)] for t in m]))
         if m else np.zeros((0, 3)))
    return cube, np.asarray(r), np.asarray(c), m, X


def run_match(args, env, wl, kernel_options):
    """``--workload c2match``: match_line() printed as the run's JSON line."""
    line, ok = match_line(args, env, wl, kernel_options, steps=args.steps, warmup=args.warmup,
                          cube_mode=args.cube, cpu_seconds=args.cpu_seconds,
                          n_chunks_req=args.match_chunks, lsap_input=args.lsap_input,
                          pipeline=args.match_pipeline == "on")
    if line is None:
        return
    print(json.dumps(line), flush=True)
    if not ok:
        log("error: c2match parity")
        raise SystemExit(3)


FREE_LSAP_INPUT = "blocks"     # the cube-free chain's default block source (--lsap-input auto)


def match_line(args, env, wl, kernel_options, *, steps, warmup, cube_mode="free", cpu_seconds=0.0,
               n_chunks_req=1, lsap_input="auto", pipeline=False):
    """What ``match_objects`` returns, at C2 scale (the ``c2match`` workload).

    A step is every scene of this rank through the device chain of
    ``batch_match.match_captures`` with its plans built once (the counts are
    host knowledge).  ``cube_mode="free"`` (the default, what
    ``match_captures(keep_cube=False)`` runs): the cube's 8-row minima and the
    scenes' fp64 pair residuals (mvm_triplet_minima), the scipy-identical
    assignment of every flattened (N*M, P) cube recomputing the entries it reads
    from them (mvm_lsap_solve_resid), then threshold + stable cost sort + DLT
    (mvm_select_triangulate_resid).  ``"keep"``: the compute_cost_matrix cube
    (mvm_triplet_cost_argmin + its 8-row minima), the assignment reading it
    (mvm_lsap_solve_ex3), select + DLT from it.  epipolar_matching.py:83-116 and
    process_pose.py:182-187.  Units are captures (scenes); HIP events time each
    stage.  After timing, four scenes are checked against the CPU chain: the
    cube (keep) or the 8-row minima and the pair residuals (free) bit for bit,
    the assignment pair for pair, the matches and their order exactly, their
    costs bit for bit and the triangulated points to 1e-10.
    -> (line dict on rank 0 / None elsewhere, parity ok)."""
    from bpc_baseline_amd.distributed import shard_range
    from bpc_baseline_amd.inference.utils.camera_utils import projection_matrices
    dev, world = env.device, env.world
    free = cube_mode == "free"
    if lsap_input == "auto":
        lsap_input = FREE_LSAP_INPUT if free else "bmin8"
    if (free and lsap_input == "cost") or (not free and lsap_input == "blocks"):
        raise SystemExit(f"c2match: --lsap-input {lsap_input} does not apply to --cube {cube_mode}")
    if args.scaling == "weak":
        first, n_local = env.rank * wl["n_scenes"], wl["n_scenes"]
    else:
        a, b = shard_range(wl["n_scenes"], env.rank, world)
        first, n_local = a, b - a
    t0 = time.perf_counter()
    batch = make_scenes(n_local, 3, wl["n_dets"], seed=args.seed, first_scene=first)
    proj = projection_matrices(batch.meta["Ks"], batch.meta["RTs"])
    log(f"[rank {env.rank}] generated {n_local} scenes in {time.perf_counter() - t0:.1f}s")
    threshold = float(wl["threshold"])
    # The step runs in chunks of scenes on two streams: the cubes one after
    # the other on the launch stream, and each chunk's assignment + select on
    # a second stream as soon as its cube is written, so the latency-bound
    # assignment overlaps the HBM-bound cube of the next chunk (the cube of a
    # chunk waits for the previous step's use of its buffers).  --match-chunks 1
    # is the serial chain.
    # pipeline: consecutive steps overlap -- step t's assignment + select on the
    # second stream while step t + 1's minima run on the launch stream -- over
    # two buffer sets (a step waits only for step t - 2's use of its set), as a
    # service matching a stream of capture batches would run them
    n_chunks = max(1, min(n_chunks_req, n_local))
    bounds = np.linspace(0, n_local, n_chunks + 1).astype(np.int64)
    stream = torch.cuda.current_stream(dev)
    side = torch.cuda.Stream(dev) if (n_chunks > 1 or pipeline) else stream

    def make_chunks():
        chunks = []
        for a, b in zip(bounds[:-1], bounds[1:]):
            a, b = int(a), int(b)
            co_h = batch.cam_offs[3 * a:3 * b + 1] - batch.cam_offs[3 * a]
            ch = {"first": a, "n": b - a, "co_h": co_h}
            ch["pts"] = torch.from_numpy(batch.pts[batch.cam_offs[3 * a]:batch.cam_offs[3 * b]]).to(dev)
            ch["cam_offs"] = torch.from_numpy(co_h).to(dev)
            ch["F"] = torch.from_numpy(batch.F[3 * a:3 * b]).to(dev)
            ch["proj"] = torch.from_numpy(np.ascontiguousarray(proj[a:b])).to(dev)
            tp = ops.TripletPlan(co_h, b - a, device=dev)
            c3 = tp.counts
            ch["tplan"] = tp
            if free:
                if not ops.cube_free_scenes(c3).all():
                    raise SystemExit("c2match --cube free: a scene outside the candidate-list class")
                ch["lplan"] = ops.LsapPlan(c3[:, 0] * c3[:, 1], c3[:, 2], device=dev, resid=True)
                ch["cube"] = None
                # --lsap-input blocks: no 8-row minima (the lists gather whole blocks)
                ch["bm8"] = torch.empty(max(tp.n_bmin8, 1) if lsap_input == "bmin8" else 0,
                                        dtype=torch.int16, device=dev)
                ch["bm32"] = torch.empty(max(tp.n_bm32, 8), dtype=torch.int16, device=dev)
            else:
                ch["lplan"] = ops.LsapPlan(c3[:, 0] * c3[:, 1], c3[:, 2], device=dev)
                ch["cube"] = torch.empty(tp.n_cube, dtype=torch.float32, device=dev)
                ch["am"] = torch.empty(tp.n_rows, dtype=torch.int32, device=dev)
                ch["mv"] = torch.empty(tp.n_rows, dtype=torch.float32, device=dev)
                ch["offs"] = tp.cube_offs[:-1].contiguous()
                # the cube kernel also writes its 8-row minima, which the assignment
                # reduces instead of reading the cubes once more (--lsap-input cost: off)
                ch["bm8"] = (torch.empty(max(tp.n_bmin8, 1), dtype=torch.int16, device=dev)
                             if lsap_input == "bmin8" else None)
            ch["used"] = None                   # event: the previous step's reads of the buffers
            chunks.append(ch)
        return chunks

    sets = [make_chunks() for _ in range(2 if pipeline else 1)]

    def step(ev=None, chunks=sets[0]):
        outs = []
        cube_done = []
        for k, ch in enumerate(chunks):
            if ch["used"] is not None:
                stream.wait_event(ch["used"])
            if ev:
                ev[k][0].record(stream)
            if free:
                ops.triplet_minima(ch["pts"], ch["cam_offs"], ch["F"], ch["tplan"], bmin8=ch["bm8"],
                                   bm32=ch["bm32"], options=kernel_options)
            else:
                ops.triplet_cost_argmin(ch["pts"], ch["cam_offs"], ch["F"], ch["tplan"],
                                        out=(ch["cube"], ch["am"], ch["mv"]), options=kernel_options,
                                        bmin8=ch["bm8"])
            e = torch.cuda.Event()
            e.record(stream)
            cube_done.append(e)
            if ev:
                ev[k][1].record(stream)
        for k, ch in enumerate(chunks):
            side.wait_event(cube_done[k])
            with torch.cuda.stream(side):
                if ev:
                    ev[k][2].record(side)
                if free:
                    r, c, st = ops.linear_sum_assignment_resid(ch["lplan"], ch["tplan"],
                                                               (ch["bm8"], ch["bm32"]),
                                                               options=kernel_options)
                else:
                    bm8_args = ((ch["bm8"], ch["tplan"].bmin8_offs, ch["tplan"].segs)
                                if ch["bm8"] is not None else None)
                    r, c, st = ops.linear_sum_assignment_batched(ch["cube"], ch["offs"], ch["lplan"],
                                                                 options=kernel_options, bmin8=bm8_args)
                if ev:
                    ev[k][3].record(side)
                if free:
                    res = ops.select_triangulate_resid(ch["tplan"], ch["cam_offs"], ch["lplan"].out_offs,
                                                       r, c, ch["pts"], ch["proj"], threshold)
                else:
                    res = ops.select_triangulate(ch["cube"], ch["tplan"].cube_offs, ch["cam_offs"],
                                                 ch["lplan"].out_offs, r, c, ch["pts"], ch["proj"],
                                                 threshold)
                if ev:
                    ev[k][4].record(side)
                u = torch.cuda.Event()
                u.record(side)
                ch["used"] = u
            outs.append((r, c, st) + tuple(res))
        if not pipeline:
            stream.wait_stream(side)
        return outs

    for w_ in range(warmup):
        step(chunks=sets[w_ % len(sets)])
    stream.wait_stream(side)
    torch.cuda.synchronize(dev)
    chunks = sets[0]
    evs = [[[torch.cuda.Event(enable_timing=True) for _ in range(5)] for _ in chunks]
           for _ in range(steps)]
    env.barrier()
    torch.cuda.synchronize(dev)
    with ClockSampler(dev) as clocks:
        t_start = time.perf_counter()
        for s_ in range(steps):
            outs = step(evs[s_], chunks=sets[s_ % len(sets)])
        stream.wait_stream(side)
        torch.cuda.synchronize(dev)
        env.barrier()
        elapsed = time.perf_counter() - t_start
    elapsed = max_over_ranks(env, elapsed)
    chunks = sets[(steps - 1) % len(sets)]              # the last step's buffers (parity)
    # kernel time per stage, summed over the chunks (they overlap across stages)
    stage = np.array([[sum(e[k][0].elapsed_time(e[k][1]) for k in range(n_chunks)),
                       sum(e[k][2].elapsed_time(e[k][3]) for k in range(n_chunks)),
                       sum(e[k][3].elapsed_time(e[k][4]) for k in range(n_chunks))]
                      for e in evs])                          # ms per step: cube, lsap, select
    cube_ms, lsap_ms, sel_ms = (float(x) for x in stage.mean(axis=0))
    status = np.concatenate([o[2].cpu().numpy() for o in outs])
    count_h = np.concatenate([o[6].cpu().numpy() for o in outs])
    n_matches = sum_over_ranks(env, int(count_h.sum()))
    n_bmin8 = sum(ch["tplan"].n_bmin8 for ch in chunks)

    # ---- parity (untimed): a few scenes against the CPU chain --------------
    parity_ok, detail = bool((status == 0).all()), []
    if env.is_root:
        from oracle import oracle as O
        picks = sorted({0, n_local // 3, (2 * n_local) // 3, n_local - 1})
        for s in picks:
            k_ch = int(np.searchsorted(bounds, s, side="right")) - 1
            ch, out = chunks[k_ch], outs[k_ch]
            sl = s - ch["first"]
            r, c, st, match, cost, X, count = out
            rc, rr, rcol, rm, rX = match_cpu_chain(batch, proj, s, threshold,
                                                   nthreads=cpu_threads())
            n3 = tuple(int(x) for x in ch["tplan"].counts[sl])
            tp = ch["tplan"]
            if free:
                # the 8-row minima (when written), the block minima and the
                # pair residuals the assignment read
                want8 = O.bmin8_keys(rc.reshape(n3))
                keys_ok = True
                if ch["bm8"].numel():
                    o8 = int(tp.bmin8_offs_host[sl])
                    keys = ch["bm8"][o8:o8 + want8.size].cpu().numpy().view(np.uint16)
                    keys_ok = np.array_equal(keys, want8.reshape(-1))
                want32 = O.bm32_keys(want8, *n3).reshape(-1)
                o32 = int(tp.bm32_offs_host[sl])
                keys_ok &= np.array_equal(ch["bm32"][o32:o32 + want32.size].cpu().numpy().view(np.uint16),
                                          want32)
                co1 = batch.cam_offs[3 * s:3 * s + 4]
                want_r = O.residuals(batch.pts[int(co1[0]):int(co1[3])], co1 - co1[0],
                                     batch.F[3 * s:3 * s + 3], 1, tp.max_n)[0]
                ld = want_r.shape[-1]
                stride = 3 * tp.max_n * ld
                got_r = tp.workspace[:tp.workspace_bytes].view(torch.float64)[sl * stride:(sl + 1) * stride]
                got_r = got_r.cpu().numpy().reshape(3, tp.max_n, ld)
                resid_ok = all(np.array_equal(got_r[m, :a_, :b_].view(np.int64), want_r[m, :a_, :b_].view(np.int64))
                               for m, (a_, b_) in enumerate(((n3[0], n3[1]), (n3[2], n3[0]), (n3[2], n3[1]))))
                cube_ok = keys_ok and resid_ok
            else:
                o = int(tp.cube_offs_host[sl])
                cube_ok = np.array_equal(ch["cube"][o:o + rc.size].cpu().numpy().view(np.int32),
                                         rc.view(np.int32))
            lo = int(ch["lplan"].out_offs_host[sl])
            nn = rr.size
            lsap_ok = (np.array_equal(r[lo:lo + nn].cpu().numpy(), rr)
                       and np.array_equal(c[lo:lo + nn].cpu().numpy(), rcol))
            k = int(count[sl].item())
            m_h = match[lo:lo + k].cpu().numpy()
            got = [tuple(int(v) for v in m_h[w]) for w in range(k)]
            match_ok = got == rm
            cube3 = rc.reshape(n3)
            cost_ok = match_ok and np.array_equal(
                cost[lo:lo + k].cpu().numpy().view(np.int32),
                np.array([cube3[t] for t in rm], np.float32).view(np.int32))
            x_ok = match_ok and (k == 0 or np.allclose(X[lo:lo + k].cpu().numpy(), rX, rtol=1e-10,
                                                       atol=1e-9))
            parity_ok &= bool(cube_ok and lsap_ok and match_ok and cost_ok and x_ok)
            d = {"scene": first + s}
            if free:
                d.update({("bmin8_bm32_bit_exact" if ch["bm8"].numel() else "bm32_bit_exact"): bool(keys_ok),
                          "residuals_bit_exact": bool(resid_ok)})
            else:
                d["cube_bit_exact"] = bool(cube_ok)
            d.update({"assignment_equal": bool(lsap_ok), "matches": k,
                      "matches_equal_in_order": bool(match_ok), "costs_bit_exact": bool(cost_ok),
                      "X_within_1e-10": bool(x_ok)})
            detail.append(d)
    if not env.is_root:
        return None, parity_ok
    total = n_local * world if args.scaling == "weak" else wl["n_scenes"]
    value = total * steps / elapsed
    counts = batch.counts()
    N, M, P = (counts[:, q].astype(np.float64) for q in range(3))
    triples = float((N * M * P).sum())
    cb = cube_bytes(counts)
    cost_bytes = 4.0 * triples
    if free:
        # the minima pass: centroids + F in; 8-row minima, block minima and
        # fp64 residuals out
        n_bm32 = sum(ch["tplan"].n_bm32 for ch in chunks)
        n8w = n_bmin8 if lsap_input == "bmin8" else 0
        first_bytes = (16.0 * counts.sum() + 3 * 72.0 * len(N) + 2.0 * float(n8w)
                       + 2.0 * float(n_bm32) + 8.0 * float((N * M + P * N + P * M).sum()))
        lsap_bytes = 2.0 * float(n_bm32)
        first_kernel = "triplet_minima_kernel"
    else:
        first_bytes = cb
        # the assignment's streamed input: the cube's 8-row minima (default), or
        # every cost entry once (--lsap-input cost)
        lsap_bytes = 2.0 * float(n_bmin8) if lsap_input == "bmin8" else cost_bytes
        first_kernel = "triplet_fused_kernel"
    stages = {"cube": (cube_ms, first_bytes, first_kernel),
              "lsap": (lsap_ms, lsap_bytes, "mvm_lsap_solve kernels"),
              "select": (sel_ms, 0.0, "select_triangulate_kernel")}
    dom = max(stages, key=lambda k: stages[k][0])
    d_ms, d_bytes, d_kernel = stages[dom]
    achieved = d_bytes / (d_ms * 1e-3) / 1e9 if d_ms > 0 else None
    cpu = None
    if cpu_seconds > 0:
        threads, threads_src = host_cpu_threads()
        match_cpu_chain(batch, proj, 0, threshold, nthreads=threads)      # warm
        n_cpu, t0 = 0, time.perf_counter()
        while n_cpu < n_local and time.perf_counter() - t0 < cpu_seconds:
            match_cpu_chain(batch, proj, n_cpu, threshold, nthreads=threads)
            n_cpu += 1
        secs = time.perf_counter() - t0
        cpu = {"value": n_cpu / secs, "unit": "captures/s", "cores": threads,
               "cores_at_n1": threads, "cores_source": threads_src, "kind": "port",
               "sample": (f"{n_cpu} scenes in {secs:.1f} s: oracle/mvm_oracle.c cube (OpenMP "
                          f"x{threads}) + scipy.optimize.linear_sum_assignment (the reference's "
                          "own call, one core) + threshold/sort + numpy SVD per match, on "
                          f"{cpu_model()}")}
    # the minima pass's arithmetic floor: per triple one float32 add (e12 + e23;
    # + e13 and the third run once per 8 triples) and half a v_min3_f32 (two
    # of the group's seven mins), at the VALU's 2-cycle wave64 issue: 78.6e12
    # lane-instructions/s (MI355X_MICROARCH.md); the exact fp64 recheck of
    # the groups near a 16-bit carry is not counted
    valu = None
    if free and cube_ms > 0:
        per_s = 1.5 * triples / (cube_ms * 1e-3)
        valu = {"bound": "f32 valu issue", "kernel": "triplet_minima_kernel",
                "achieved": per_s / 1e12, "peak": 78.6, "unit": "T lane-instr/s",
                "frac": per_s / 1e12 / 78.6, "instr_per_triple": 1.5,
                "note": ("algorithmic VALU lane-instructions (one v_add_f32, half a v_min3_f32 per "
                         "triple) over the stage's HIP-event time, against 256 CUs x 4 SIMDs x 32 "
                         "lanes x 2.4 GHz (MI355X_MICROARCH.md: wave64 issue in 2 cycles)")}
    line = {
        "metric": "captures matched/sec (cost cube + scipy-identical assignment + select/DLT)",
        "value": value, "unit": "captures/s", "n_gpus": world, "steps": steps,
        "warmup": warmup, "ms_per_step": elapsed / steps * 1e3,
        "higher_is_better": True, "scaling": args.scaling, "vs_baseline": None, "dtype": "f64",
        "data": "synthetic (seeded IPD-like rig, SURVEY §8d generator)",
        "config": {"workload": wl["desc"], "n_cams": 3, "n_dets": wl["n_dets"],
                   "n_scenes_per_gpu": n_local, "n_scenes_total": total,
                   "matching_threshold": threshold, "kernel_options": kernel_options,
                   "cube": ("free: 8-row minima + fp64 pair residuals, entries recomputed where read "
                            "(match_captures keep_cube=False)" if free else
                            "keep: the cost cubes written and read (keep_cube=True)"),
                   "lsap_input": lsap_input,
                   "launch": (f"eager op calls, {n_chunks} chunks of scenes: cubes on the launch "
                              "stream, each chunk's assignment + select on a second stream once "
                              "its cube is written" if n_chunks > 1 else "eager op calls, serial"),
                   "match_chunks": n_chunks,
                   "pipeline": (("consecutive steps overlap: step t's assignment + select on a second "
                                 "stream while step t + 1's minima run, two buffer sets")
                                if pipeline else "off: each step's chain completes before the next starts"),
                   "parallelism": f"scene-sharded x{world}" if env.initialised else "single GPU"},
        "stages_ms": {("minima" if free else "cube"): cube_ms, "lsap": lsap_ms, "select_dlt": sel_ms,
                      "note": ("rank 0, HIP events on each stage's stream, summed over the chunks, "
                               "mean over the timed steps; the stages of different chunks overlap")},
        "lsap": {"problems": n_local, "shape": f"{int(counts[0, 0] * counts[0, 1])} x {int(counts[0, 2])}",
                 "ms_per_batch": lsap_ms, "ms_per_problem": lsap_ms / max(1, n_local),
                 "streamed_gb": lsap_bytes / 1e9, "cost_gb": cost_bytes / 1e9,
                 "input": ("the minima pass's block minima + pair residuals (mvm_lsap_solve_resid)" if free
                           else "the cube kernel's 8-row minima (mvm_lsap_solve_ex3)"
                           if lsap_input == "bmin8" else "the cost cubes (mvm_lsap_solve_ex2)")},
        "matches_per_step": n_matches,
        "sclk": clocks.summary("sclk"),
        "roofline": {"bound": "hbm", "stage": dom, "kernel": d_kernel, "achieved": achieved,
                     "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": (achieved / HBM_PEAK_GBS) if achieved else None, "traffic": None,
                     "bytes_per_launch": d_bytes, "avg_launch_ms": d_ms,
                     "note": ("the slowest stage; its algorithmic bytes: the cube's writes (4 B "
                              "per triple + 8 B per row + inputs), or free the minima's and "
                              "residuals' writes, or for the assignment its streamed input "
                              "(lsap.streamed_gb)")},
        "valu_roofline": valu,
        "cpu_baseline": cpu,
        "parity": f"{'equal' if parity_ok else 'MISMATCH'} vs the CPU chain on {len(detail)} scenes",
        "parity_detail": detail,
    }
    return line, parity_ok


def main():
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="c3")
    ap.add_argument("--scenes", type=int, default=None, help="scenes (override; per GPU with "
                    "--scaling weak)")
    ap.add_argument("--chunk", type=int, default=None, help="most scenes per launch (override)")
    ap.add_argument("--min-launches", type=int, default=None,
                    help="fewest launches per rank and step (default: 5 with N > 1, so the "
                         "unoverlapped last gather piece is a small part of a step; 1 on one GPU)")
    ap.add_argument("--scaling", choices=["weak", "strong"], default="strong",
                    help="strong (default): --scenes split over the GPUs, so --gpus 8 measures "
                         "BASELINE configs[3] (C3's 10k scenes, 1,250 per GPU); weak: --scenes "
                         "per GPU")
    ap.add_argument("--dump-association", default=None, metavar="DIR",
                    help="rank 0 saves the gathered association rows (argmin.npy, minval.npy, "
                         "in global scene order) after the timed region")
    ap.add_argument("--cpu-seconds", type=float, default=12.0,
                    help="target length of the CPU-baseline sample (0 disables)")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--output", choices=["resident", "ring"], default="resident",
                    help="resident (default): one output allocation per launch of the timed "
                         "steps as far as HBM holds them (reused round robin); ring: one")
    ap.add_argument("--graph", choices=["auto", "launch", "steps", "steps2", "off"], default="auto",
                    help="auto (default): steps for the c2 workload on one GPU (its 0.14 ms "
                         "launches are shorter than the host's per-replay cost), launch "
                         "otherwise; launch: each launch of each timed step is a hipGraph "
                         "captured outside the timed region and replayed in order, the gather "
                         "piece of launch k issued right after its replay; steps: one hipGraph "
                         "holding all K steps (one GPU only: a step with N > 1 has collectives); "
                         "off: eager op calls")
    ap.add_argument("--parity", choices=["full", "scene"], default="full",
                    help="full (default): after timing, every association row of the last step "
                         "(all ranks' rows, as gathered to rank 0) against the oracle, which each "
                         "rank computes for its own scenes and sends to rank 0 over a gloo group; "
                         "scene: only the last launch's first scene")
    ap.add_argument("--options", default=None, metavar="FIELD=VALUE,...",
                    help="mvm_options fields for the launches (include/mvmatch.h; e.g. "
                         "pairwise_row_groups=2): kernel-path choices that never change results, "
                         "for A/B runs of the line itself; recorded in config.kernel_options")
    ap.add_argument("--match-pipeline", choices=["on", "off"], default="off",
                    help="c2match: overlap consecutive steps (step t's assignment + select on a "
                         "second stream while step t + 1's minima run; two buffer sets)")
    ap.add_argument("--match-chunks", type=int, default=1,
                    help="c2match: scenes per step in this many chunks, the assignment of one "
                         "overlapping the cube of the next on a second stream (1: serial, the "
                         "default: the overlap measured slower, DESIGN §11.9)")
    ap.add_argument("--cube", choices=["free", "keep"], default="free",
                    help="c2match: free (default, match_captures keep_cube=False): the assignment "
                         "and the select/DLT recompute the entries they read from the 8-row minima "
                         "pass's fp64 pair residuals, no cube is written; keep: the cost cubes are "
                         "written and read")
    ap.add_argument("--c2match", choices=["auto", "off"], default="auto",
                    help="auto (default): the c3 workload on one GPU also measures c2match "
                         "(cube-free) after its own line's parity and nests it in the line as "
                         "\"c2match\"; off: not")
    ap.add_argument("--lsap-input", choices=["auto", "bmin8", "blocks", "cost"], default="auto",
                    help="c2match: the assignment's candidate blocks refined by the 8-row minima "
                         "(bmin8), whole 32-column blocks from the block minima alone (blocks: "
                         "--cube free only; no 8-row minima written) or the cost cubes read again "
                         "(cost: --cube keep only); auto: FREE_LSAP_INPUT / bmin8")
    ap.add_argument("--dry-run", action="store_true",
                    help="start the ranks and the process group (gloo, host only) and print the "
                         "world each rank joined; no GPU work (tests the launcher on a CPU host)")
    args = ap.parse_args()
    if args.gpus < 1:
        raise SystemExit(f"error: --gpus {args.gpus}")
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        raise SystemExit(launch_ranks(args.gpus))
    env_world = int(os.environ.get("WORLD_SIZE", "1"))
    if env_world != args.gpus:
        raise SystemExit(f"error: --gpus {args.gpus} but WORLD_SIZE={env_world} (run `python "
                         "bench.py --gpus N` alone, or under torchrun with --nproc-per-node N)")
    if args.dry_run:
        env = init_from_env(backend="gloo", use_gpu=False)
        seen = gather_rows(env, torch.tensor([env.rank], dtype=torch.int64))
        if env.world != args.gpus:
            raise SystemExit(f"error: --gpus {args.gpus} but the process group has {env.world} rank(s)")
        if env.is_root:
            print(json.dumps({"dry_run": True, "n_gpus": env.world,
                              "ranks_seen": [int(x) for x in seen[0]],
                              "process_group": {"world_size": env.world, "backend": env.backend}
                              if env.initialised else None}), flush=True)
        return

    global ops
    from bpc_baseline_amd import ops as _ops
    ops = _ops
    kernel_options = None
    if args.options:
        kernel_options = {}
        for kv in args.options.split(","):
            k, _, v = kv.partition("=")
            kernel_options[k.strip()] = v.strip() if k.strip() in ("pairwise_argmin", "cube_kernel") \
                else int(v)

    wl = dict(WORKLOADS[args.workload])
    if args.scenes:
        wl["n_scenes"] = args.scenes
    if args.chunk:
        wl["chunk"] = args.chunk

    env = init_from_env()
    world = env.world
    if world != args.gpus:
        raise SystemExit(f"error: --gpus {args.gpus} but the process group has {world} rank(s) "
                         "(run `python bench.py --gpus N` alone, or under torchrun with "
                         "--nproc-per-node N)")
    if env.backend == "nccl" and torch.cuda.device_count() < world:
        raise SystemExit(f"error: {world} RCCL ranks but {torch.cuda.device_count()} visible GPU(s)")
    dev = env.device
    if wl["mode"] == "match":
        return run_match(args, env, wl, kernel_options)
    if args.graph == "auto":
        # per-launch replays (and the per-launch HIP events around them) cost the
        # host ~15 us per replay; a 0.14 ms C2 launch cannot hide that, C3's
        # 4 ms launches do.  Events recorded inside a captured graph cannot be
        # timed on ROCm (tools/probes/graph_events.py), so "steps" times the K
        # steps with one event pair.
        # steps so short that a step's tail and the next one's start matter (C2)
        # take two streams ("steps2": +6-8% on the C2 line)
        args.graph = "steps2" if (args.workload == "c2" and not env.initialised) else "launch"
    if args.graph == "steps2" and wl["mode"] != "pairwise":
        # both streams would pass the same plan -- and a workspace-path cube
        # kernel the same plan.workspace -- to concurrent steps
        raise SystemExit("--graph steps2 is for the pairwise workloads (c3, c2): concurrent cube "
                         "steps would share the plan's workspace")
    if args.graph in ("steps", "steps2") and env.initialised:
        raise SystemExit("--graph steps/steps2 need a single GPU without a process group "
                         "(the step's gather is a collective)")
    if args.scaling == "strong" and wl["n_scenes"] < world:
        raise SystemExit(f"--scenes {wl['n_scenes']} < {world} ranks: every rank needs at least "
                         "one scene (strong scaling splits the scenes over the ranks)")
    min_launches = args.min_launches if args.min_launches else (5 if world > 1 else 1)

    # ---- this rank's shard of scenes (global scene ids are seeds) ----------
    if args.scaling == "weak":
        first, n_local = env.rank * wl["n_scenes"], wl["n_scenes"]
    else:
        from bpc_baseline_amd.distributed import shard_range
        a, b = shard_range(wl["n_scenes"], env.rank, world)
        first, n_local = a, b - a
    t0 = time.perf_counter()
    batch = make_scenes(n_local, wl["n_cams"], wl["n_dets"], seed=args.seed, first_scene=first)
    log(f"[rank {env.rank}] generated {n_local} scenes in {time.perf_counter() - t0:.1f}s")
    # with N > 1 a short last launch, so the one gather piece no launch
    # overlaps is small (equal shards: every rank has the same pieces)
    bounds = launch_bounds(n_local, wl["chunk"], min_launches, 0.25 if world > 1 else 0.0)
    chunk = max(s1 - s0 for s0, s1 in bounds)    # scenes per launch (the largest)
    chunks, n_rows = build_chunks(batch, bounds, dev, wl["mode"])
    argmin = torch.empty(n_rows, dtype=torch.int32, device=dev)
    minval = torch.empty(n_rows, dtype=torch.float32, device=dev)
    # "steps2": the odd steps' association rows (they may run beside an even step)
    alt_rows = ((torch.empty_like(argmin), torch.empty_like(minval)) if args.graph == "steps2"
                else None)
    max_units = max(c.size for c in chunks)
    # output slots: one allocation per launch of the timed steps when they fit
    # (a step's residuals all stay resident, and consecutive steps write other
    # allocations, as a service that double-buffers its outputs would),
    # keeping >= 8 GiB of HBM free (RCCL, the gather); launches take the slots round robin
    n_slots = 1
    if args.output == "resident":
        n_slots = output_slots(len(chunks) * max(1, args.steps), 4 * max_units,
                               torch.cuda.mem_get_info(dev)[0])
    out_slots = []
    for _ in range(n_slots):   # fewer if the allocator refuses one (fragmented HBM)
        try:
            out_slots.append(torch.empty(max_units, dtype=torch.float32, device=dev))
        except torch.cuda.OutOfMemoryError:
            if not out_slots:
                raise
            break
    n_slots = len(out_slots)
    if args.graph == "steps2":
        # concurrent (even / odd) steps must not share an allocation: with a
        # multiple of 2 x launches-per-step slots, even steps take one half of
        # the residues and odd steps the other; too few slots: one stream
        L2 = 2 * len(chunks)
        if n_slots >= L2:
            n_slots = n_slots // L2 * L2
            del out_slots[n_slots:]
        else:
            log(f"--graph steps2 needs >= {L2} output allocations ({n_slots}): one stream")
            args.graph, alt_rows = "steps", None
    seq = [0]             # launches issued (or captured) so far: the next slot
    last_slot = {}        # chunk -> the slot its latest launch wrote
    slot_owner = {}       # slot -> index of the chunk whose output it holds
    dispatched = [0]      # kernel launches that reached the GPU (rocprof window, below)
    units_local = sum(c.units for c in chunks)
    stream = torch.cuda.current_stream(dev)

    def launch(c: Chunk, alt: bool = False):
        am_all, mv_all = alt_rows if alt else (argmin, minval)
        am = am_all[c.row_base:c.row_base + c.plan.n_rows]
        mv = mv_all[c.row_base:c.row_base + c.plan.n_rows]
        last_slot[id(c)] = seq[0] % n_slots
        slot_owner[last_slot[id(c)]] = c.idx
        seq[0] += 1
        if not torch.cuda.is_current_stream_capturing():
            dispatched[0] += 1
        out = out_slots[last_slot[id(c)]][:c.size]
        if wl["mode"] == "pairwise":
            ops.pairwise_residual_argmin(c.pts, c.cam_offs, c.F, c.plan, out=(out, am, mv),
                                         options=kernel_options)
        else:
            ops.triplet_cost_argmin(c.pts, c.cam_offs, c.F, c.plan, out=(out, am, mv),
                                    options=kernel_options)

    # the single association gather (N > 1), in per-launch pieces that overlap
    # the next launch's compute; ragged shards fall back to one gather at the end
    overlap = True
    try:
        gatherer = ChunkedRowGather(env, (argmin, minval),
                                    [(c.row_base, c.row_base + c.plan.n_rows) for c in chunks])
    except ValueError:
        gatherer, overlap = None, False

    def eager_step():
        for k, c in enumerate(chunks):
            launch(c)
            if overlap:
                gatherer.issue(k)
        return gatherer.finish() if overlap else gather_rows(env, argmin, minval)

    for _ in range(args.warmup):
        eager_step()
    torch.cuda.synchronize(dev)
    env.barrier()
    seq[0] = 0            # the timed steps start at slot 0

    # ---- hipGraphs, captured outside the timed region.  "launch" (every N):
    # one graph per launch of each timed step, so the gather piece of launch k
    # can be issued right after its replay and N = 1 and N > 1 time the same
    # launch path; "steps" (one GPU): one graph holding all K steps.  Captured
    # thread-locally: the RCCL watchdog thread queries events meanwhile.
    graphs, step_graph = None, None
    graph_slot = {}       # (step, launch) -> the output slot its graph writes
    cap_kw = dict(capture_error_mode="thread_local")
    if args.graph == "launch":
        graphs = []
        for s in range(args.steps):
            row = []
            for k, c in enumerate(chunks):
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, **cap_kw):
                    launch(c)
                graph_slot[(s, k)] = last_slot[id(c)]
                row.append(g)
            graphs.append(row)
        for row in graphs:                      # first replay uploads the graph: untimed
            for g in row:
                g.replay()
                dispatched[0] += 1
    elif args.graph in ("steps", "steps2"):
        # steps2: the K steps captured on two streams, even steps on one and
        # odd steps on the other (each step writes its own output allocation
        # and, for odd steps, its own association rows), so consecutive steps
        # are independent graph branches and one step's tail may overlap the
        # next one's start
        step_graph = torch.cuda.CUDAGraph()
        two = args.graph == "steps2"
        alt_stream = torch.cuda.Stream(dev) if two else None
        with torch.cuda.graph(step_graph, **cap_kw):
            cs = torch.cuda.current_stream(dev)
            if two:
                alt_stream.wait_stream(cs)
            for st in range(args.steps):
                odd = two and st % 2 == 1
                with torch.cuda.stream(alt_stream if odd else cs):
                    for c in chunks:
                        launch(c, alt=odd)
            if two:
                cs.wait_stream(alt_stream)
        step_graph.replay()
        dispatched[0] += args.steps * len(chunks)
    torch.cuda.synchronize(dev)
    seq[0] = 0

    def run_launch(s: int, k: int) -> int:
        """Run launch k of timed step s; returns the output slot it wrote."""
        if graphs is not None:
            graphs[s][k].replay()
            dispatched[0] += 1
            slot_owner[graph_slot[(s, k)]] = k
            return graph_slot[(s, k)]
        launch(chunks[k])
        return last_slot[id(chunks[k])]

    # every event of the timed steps is created up front: creating two per
    # launch inside the loop cost the host ~30 us per C2 step, longer than the
    # GPU took for some launches, so the GPU waited on the host between them
    def new_event():
        return torch.cuda.Event(enable_timing=True)
    step_events = [[(new_event(), new_event()) for _ in chunks] for _ in range(args.steps)]
    tail_events = [(new_event(), new_event()) for _ in range(args.steps)]

    def timed_step(s, events, tails):
        for k, c in enumerate(chunks):
            e0, e1 = step_events[s][k]
            e0.record(stream)
            slot = run_launch(s, k)
            e1.record(stream)
            events.append((e0, e1, c.nbytes, c.units, 1, slot))
            if overlap:
                gatherer.issue(k)
        ec, es = tail_events[s]
        ec.record(stream)     # the step's compute is done here ...
        res = gatherer.finish() if overlap else gather_rows(env, argmin, minval)
        es.record(stream)     # ... and its association is on rank 0 here: the exposed tail
        tails.append((ec, es))
        return res

    events, tails = [], []
    gathered = None
    torch.cuda.synchronize(dev)
    env.barrier()
    window_start = dispatched[0]
    with ClockSampler(dev) as clocks:
        t_start = time.perf_counter()
        if step_graph is not None:   # one event pair over the timed region: no markers between steps
            ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ev0.record(stream)
            step_graph.replay()      # the K steps
            ev1.record(stream)
            dispatched[0] += args.steps * len(chunks)
            events.append((ev0, ev1, sum(c.nbytes for c in chunks) * args.steps,
                           units_local * args.steps, len(chunks) * args.steps, None))
        else:
            for s in range(args.steps):
                gathered = timed_step(s, events, tails)
        torch.cuda.synchronize(dev)
        env.barrier()
        elapsed = time.perf_counter() - t_start
    window_timed = dispatched[0] - window_start
    if alt_rows is not None and (args.steps - 1) % 2 == 1:   # the last step's rows (untimed)
        argmin.copy_(alt_rows[0])
        minval.copy_(alt_rows[1])
        torch.cuda.synchronize(dev)
    elapsed = max_over_ranks(env, elapsed)
    ms_per_step = elapsed / args.steps * 1e3

    # ---- N > 1: the step's two parts timed apart (untimed for `value`) -----
    # compute alone (every launch, no collective) and the association gather
    # alone, each bracketed by barrier + sync and maxed over ranks; and the
    # exposed tail of the timed steps: last launch done -> gather done
    split = None
    if env.initialised:
        reps = max(1, min(args.steps, 5))
        torch.cuda.synchronize(dev)
        env.barrier()
        t0 = time.perf_counter()
        for r in range(reps):
            for k in range(len(chunks)):
                run_launch(r % args.steps, k)
        torch.cuda.synchronize(dev)
        env.barrier()
        t_comp = max_over_ranks(env, time.perf_counter() - t0) / reps
        t0 = time.perf_counter()
        for _ in range(reps):
            if overlap:
                for k in range(len(chunks)):
                    gatherer.issue(k)
                gatherer.finish()
            else:
                gather_rows(env, argmin, minval)
        torch.cuda.synchronize(dev)
        env.barrier()
        t_gath = max_over_ranks(env, time.perf_counter() - t0) / reps
        tail_ms = float(np.mean([a.elapsed_time(b) for a, b in tails])) if tails else 0.0
        tail_ms = max_over_ranks(env, tail_ms)
        split = {"compute_ms": t_comp * 1e3, "gather_ms": t_gath * 1e3,
                 "gather_bytes_per_rank": int(n_rows * 8),
                 "exposed_tail_ms": tail_ms, "exposed_tail_frac": tail_ms / ms_per_step,
                 "note": "compute_ms / gather_ms: each part alone, barrier + sync around, max over "
                         "ranks; exposed_tail_ms: in the timed steps, from the end of a rank's "
                         "last launch to its gather pieces being done (HIP events on the launch "
                         "stream, mean over steps, max over ranks) -- the part of the gather "
                         "that no launch overlaps"}

    # ---- kernel roofline from the events (on the launch stream) ------------
    # (with the "steps" graph, one event pair brackets the K steps' launches)
    durs = np.array([e0.elapsed_time(e1) * 1e-3 for e0, e1, *_ in events])
    byts = np.array([ev[2] for ev in events], dtype=np.float64)
    units_ev = np.array([ev[3] for ev in events], dtype=np.float64)
    n_launch = sum(ev[4] for ev in events)
    # rank 0's launches per output allocation: the same launch runs at
    # different speeds on different HBM allocations
    per_slot = None
    if events and events[0][5] is not None:
        per_slot = []
        for sl in sorted({ev[5] for ev in events}):
            idx = [i for i, ev in enumerate(events) if ev[5] == sl]
            t = float(durs[idx].sum())
            per_slot.append({"slot": sl, "launches": len(idx),
                             "mean_ms": t / len(idx) * 1e3,
                             "achieved_gbs": float(byts[idx].sum()) / t / 1e9})
        rates = [p["achieved_gbs"] for p in per_slot]
        per_slot = {"slots": per_slot, "fastest_over_slowest": max(rates) / min(rates),
                    "note": "rank 0, HIP events per launch grouped by the output allocation "
                            "the launch wrote (achieved = algorithmic bytes / time)"}
    avg_dur = float(durs.sum() / n_launch)
    achieved_gbs = float(byts.sum() / durs.sum() / 1e9)
    # every rank's figure, then the slowest rank's (max launch time, min GB/s)
    avg_dur_max = max_over_ranks(env, avg_dur)
    achieved_min = -max_over_ranks(env, -achieved_gbs)

    # ---- the whole step's association vs the oracle (untimed) --------------
    # Every rank runs the oracle (C/OpenMP, oracle/) over its own scenes and
    # sends the rows to rank 0 over a gloo group (host memory, not the RCCL
    # transport under test); rank 0 compares them with every row it holds
    # after the step's gather: rank 0's own rows and what ranks 1..N-1 sent.
    parity_rows, parity_detail = None, None
    if args.parity == "full":
        from oracle import oracle as O
        t0 = time.perf_counter()
        nth = cpu_threads()
        if wl["mode"] == "pairwise":
            _, ra, rm, _, _ = O.pairwise(batch.pts, batch.cam_offs, batch.F, batch.pairs,
                                         batch.n_scenes, batch.n_cams, want_dist=False, nthreads=nth)
        else:
            _, ra, rm, _, _ = O.cube(batch.pts, batch.cam_offs, batch.F, batch.n_scenes,
                                     want_cube=False, nthreads=nth)
        t_oracle = max_over_ranks(env, time.perf_counter() - t0)
        g_am = g_mv = None
        if env.is_root:
            if env.initialised:
                g_am, g_mv = (g.reshape(-1).cpu().numpy() for g in gathered[:2])
            else:
                g_am, g_mv = argmin.cpu().numpy(), minval.cpu().numpy()
        total, ok_rows, first_bad = compare_rows_streamed(env, ra, rm, g_am, g_mv)
        if env.is_root:
            parity_rows = f"{ok_rows}/{total} bit-exact vs oracle"
            parity_detail = {
                "rows_checked": total, "rows_bit_exact": ok_rows, "gathered_rows": int(g_am.size),
                "transfer": "oracle rows sent to rank 0 one rank at a time (gloo send/recv) and "
                            "compared with that rank's slice of the gathered rows",
                "first_mismatch_row": first_bad, "ranks": world, "oracle_threads_per_rank": nth,
                "oracle_s": t_oracle,
                "what": ("every (argmin, min) row of the last timed step, in global scene order: "
                         + ("rank 0's rows and the rows ranks 1..N-1 sent over the step's gather "
                            f"({env.backend}), against the oracle rows each rank computed for "
                            "its own scenes and sent over a gloo group"
                            if env.initialised else
                            "the GPU's rows against the oracle's for the same scenes")),
                "oracle": "oracle/mvm_oracle.c (the reference's epipolar_error + np.argmin rule)"}
    if args.dump_association and env.is_root:
        os.makedirs(args.dump_association, exist_ok=True)
        if env.initialised:
            g_am, g_mv = (g.reshape(-1).cpu().numpy() for g in gathered[:2])
        else:
            g_am, g_mv = argmin.cpu().numpy(), minval.cpu().numpy()
        np.save(os.path.join(args.dump_association, "argmin.npy"), g_am)
        np.save(os.path.join(args.dump_association, "minval.npy"), g_mv)

    # ---- residual matrices vs the oracle (untimed): the first scene of the
    # launch whose output each allocation still holds, so every allocation the
    # last step wrote is checked (C3: five scenes, five 50 GB allocations) ----
    parity, parity_ok = "skipped", True
    if env.is_root:
        from oracle import oracle as O
        C, P = batch.n_cams, batch.n_pairs
        n_units, checked = 0, []
        # allocations holding the same launch (C2: one launch per step, twenty
        # allocations) are checked on different scenes of it: the m-th of n
        # holders on scene m * scenes / n
        holders = {}
        for sl in sorted(slot_owner):
            holders.setdefault(slot_owner[sl], []).append(sl)
        for sl in sorted(slot_owner):
            c = chunks[slot_owner[sl]]
            hs = holders[slot_owner[sl]]
            s_in = hs.index(sl) * c.plan.n_scenes // len(hs)     # scene within the launch
            s_first = c.s0 + s_in
            co = batch.cam_offs[s_first * C:(s_first + 1) * C + 1]
            pts1 = batch.pts[int(co[0]):int(co[-1])]
            out = out_slots[sl]
            if wl["mode"] == "pairwise":
                rd, ra, _, _, _ = O.pairwise(pts1, co - co[0], batch.F[s_first * P:(s_first + 1) * P],
                                             batch.pairs, 1, C)
                # the scene's matrices, unpitched, read through the plan's offsets
                gd = torch.cat([c.plan.matrix(out, s_in, p).reshape(-1) for p in range(P)]).cpu().numpy()
                r0 = c.row_base + int(c.plan.row_offs_host[s_in * P])
            else:
                rd, ra, _, _, _ = O.cube(pts1, co - co[0], batch.F[s_first * 3:(s_first + 1) * 3], 1)
                o0 = int(c.plan.cube_offs_host[s_in])
                gd = out[o0:o0 + rd.size].cpu().numpy()
                r0 = c.row_base + int(c.plan.row_offs_host[s_in])
            ga = argmin[r0:r0 + ra.size].cpu().numpy()
            ok = np.array_equal(gd.view(np.int32), rd.view(np.int32)) and np.array_equal(ga, ra)
            parity_ok &= ok
            n_units += rd.size
            checked.append(first + s_first)
        what = "pairs" if wl["mode"] == "pairwise" else "triples"
        parity = (f"{'bit-exact' if parity_ok else 'MISMATCH'} vs oracle on {len(checked)} scenes "
                  f"({n_units} {what}, {len(checked)}/{n_slots} allocations; scenes {checked})")

    # ---- PCIe-inclusive rate of one launch (never `value`) ------------------
    # the same launch fed from pinned host buffers: H2D of centroids, offsets
    # and F, the kernel, D2H of the association rows; distances stay in HBM
    pcie = None
    if env.is_root:
        c = chunks[-1]
        srcs = [t.cpu().pin_memory() for t in (c.pts, c.cam_offs, c.F)]
        am = argmin[c.row_base:c.row_base + c.plan.n_rows]
        mv = minval[c.row_base:c.row_base + c.plan.n_rows]
        am_h = torch.empty(am.shape, dtype=am.dtype).pin_memory()
        mv_h = torch.empty(mv.shape, dtype=mv.dtype).pin_memory()
        best = None
        for _ in range(3):
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            for dst, src in zip((c.pts, c.cam_offs, c.F), srcs):
                dst.copy_(src, non_blocking=True)
            launch(c)
            am_h.copy_(am, non_blocking=True)
            mv_h.copy_(mv, non_blocking=True)
            torch.cuda.synchronize(dev)
            dt = time.perf_counter() - t0
            best = dt if best is None else min(best, dt)
        h2d = sum(t.numel() * t.element_size() for t in srcs)
        d2h = am_h.numel() * 4 + mv_h.numel() * 4
        pcie = {"value": c.units / best, "unit": "pairs/s" if wl["mode"] == "pairwise" else "triples/s",
                "ms_per_launch": best * 1e3, "h2d_bytes": h2d, "d2h_bytes": d2h,
                "note": (f"one {c.plan.n_scenes}-scene launch from pinned host buffers: H2D centroids "
                         "+ offsets + F, kernel, D2H argmin/min (best of 3); the distance matrices "
                         "stay in HBM")}

    # ---- the kernel alone: a few launches of the first chunk, one at a time
    # (HIP events around each, the stream drained between them), next to the
    # timed period, which overlaps launch tails (steps / steps2 graphs) ------
    kernel_iso = None
    if env.is_root:
        iso = []
        for _ in range(5):
            i0, i1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize(dev)
            if hasattr(torch.cuda, "_sleep"):
                torch.cuda._sleep(2_000_000)   # the GPU waits ~1 ms: the launch is queued before i0 fires
            i0.record(stream)
            launch(chunks[0])
            i1.record(stream)
            torch.cuda.synchronize(dev)
            iso.append(i0.elapsed_time(i1))
        kernel_iso = {"ms": float(np.median(iso)), "min_ms": float(min(iso)),
                      "launch_scenes": chunks[0].plan.n_scenes,
                      "achieved": chunks[0].nbytes / (float(np.median(iso)) * 1e-3) / 1e9,
                      "note": "median of 5 eager launches of the first launch's scenes, each alone "
                              "on the launch stream between two HIP events (the stream held by a "
                              "~1 ms spin kernel while the host enqueues them)"}

    # ---- achievable HBM write bandwidth on this box (same store form), over
    # the same output allocations the launches wrote ----------------------------
    probe_gbs = probe2_gbs = None
    if env.is_root:
        pe0, pe1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for buf in out_slots:
            ops.hbm_write_probe(buf)
        # per allocation too (an event pair around each probe), so the line
        # shows whether a slow slot is slow for a plain store stream as well
        slot_ev = [[(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                    for _ in out_slots] for _ in range(5)]
        pe0.record(stream)
        for rep in range(5):
            for i, buf in enumerate(out_slots):
                slot_ev[rep][i][0].record(stream)
                ops.hbm_write_probe(buf)
                slot_ev[rep][i][1].record(stream)
        pe1.record(stream)
        torch.cuda.synchronize(dev)
        probe_gbs = 5 * n_slots * max_units * 4 / (pe0.elapsed_time(pe1) * 1e-3) / 1e9
        # steps2 times a two-stream period: the probe in the same shape too
        # (even allocations on the launch stream, odd ones on a second)
        if args.graph == "steps2":
            alt = torch.cuda.Stream(dev)
            q0, q1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            # the stream held by a spin kernel while the host enqueues the
            # probes (eager launches and stream switches would otherwise leave
            # gaps the steps2 graph does not have)
            if hasattr(torch.cuda, "_sleep"):
                torch.cuda._sleep(20_000_000)
            q0.record(stream)
            alt.wait_stream(stream)
            for rep in range(5):
                for i, buf in enumerate(out_slots):
                    with torch.cuda.stream(alt if i % 2 else stream):
                        ops.hbm_write_probe(buf)
            stream.wait_stream(alt)
            q1.record(stream)
            torch.cuda.synchronize(dev)
            probe2_gbs = 5 * n_slots * max_units * 4 / (q0.elapsed_time(q1) * 1e-3) / 1e9
        if per_slot:
            for p in per_slot["slots"]:
                t = float(np.mean([slot_ev[rep][p["slot"]][0].elapsed_time(slot_ev[rep][p["slot"]][1])
                                   for rep in range(5)])) * 1e-3
                p["probe_gbs"] = max_units * 4 / t / 1e9
                p["frac_of_probe"] = p["achieved_gbs"] / p["probe_gbs"]
            pr = [p["probe_gbs"] for p in per_slot["slots"]]
            per_slot["probe_fastest_over_slowest"] = max(pr) / min(pr)

    units_all = sum_over_ranks(env, units_local)   # ragged shards differ by one scene
    if not env.is_root:
        return
    total_units = units_all * args.steps
    value = total_units / elapsed
    unit = "pairs/s" if wl["mode"] == "pairwise" else "triples/s"
    # the CPU baseline runs at every N, on rank 0 after the timed region (the
    # other ranks are done by then), on a sample of rank 0's own scenes
    cpu = None
    if args.cpu_seconds > 0:
        cpu = cpu_baseline(batch, wl["mode"], args.cpu_seconds)
        if world > 1:
            cpu["note"] = (f"rank 0 of {world}, after the timed region, on a sample of its own "
                           "scenes; per host, so compare it with the whole-job value")
    traffic = load_traffic(args.workload, chunk)
    kernel = "pairwise_lazy_kernel" if wl["mode"] == "pairwise" else "triplet_fused_kernel"
    launch_desc = {
        "launch": ("one hipGraph per launch of each timed step (captured once outside the timed "
                   "region), replayed in order; with N > 1 the launch's association gather piece "
                   "is issued right after its replay"),
        "steps": ("one hipGraph holding the K steps' launches, captured once outside the timed "
                  "region, replayed once"),
        "steps2": ("one hipGraph holding the K steps' launches on two streams (even / odd "
                   "steps; each step its own output allocation, odd steps their own "
                   "association rows), captured once outside the timed region, replayed once"),
        "off": "eager op calls",
    }[args.graph]
    out = {
        "metric": METRIC if wl["mode"] == "pairwise" else "cost-cube triples/sec",
        "value": value,
        "unit": unit,
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": args.scaling,
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic (seeded IPD-like rig, SURVEY §8d generator)",
        "config": {
            "workload": wl["desc"],
            "n_cams": wl["n_cams"], "n_dets": wl["n_dets"],
            "n_scenes_per_gpu": n_local,
            "n_scenes_total": n_local * world if args.scaling == "weak" else wl["n_scenes"],
            "scenes_per_launch": chunk, "launches_per_step": len(chunks),
            "output_allocations": n_slots,
            "output_gb": n_slots * max_units * 4 / 1e9,
            "units_per_gpu_step": units_local,
            "launch_mode": args.graph,
            "kernel_options": kernel_options,
            "launch": launch_desc,
            "parallelism": (f"scene-sharded x{world}, association gathered to rank 0 per step "
                            f"({env.backend}{', overlapped per launch' if overlap else ''})")
                           if env.initialised else "single GPU",
            "baseline_config": ("configs[3]: C3 scene-sharded across the GPUs"
                                if args.workload == "c3" and args.scaling == "strong" and world > 1
                                else None),
        },
        "process_group": ({"world_size": world, "backend": env.backend,
                           "source": "torch.distributed.get_world_size()/get_backend() after init"}
                          if env.initialised else None),
        "step_split": split,
        "sclk": clocks.summary("sclk"),
        "mclk": clocks.summary("mclk"),
        "fclk": clocks.summary("fclk"),
        "temperature": clocks.temperatures(),
        "roofline": {
            "bound": "hbm",
            "kernel": kernel,
            "achieved": achieved_min,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": achieved_min / HBM_PEAK_GBS,
            "traffic": (traffic or {}).get("bytes_per_launch"),
            "bytes_per_launch": float(byts.sum() / n_launch),
            "avg_launch_ms": avg_dur_max * 1e3,
            "ranks": ("slowest rank: max over ranks of the mean launch time, min over ranks of "
                      "the achieved GB/s" if world > 1 else "one rank"),
            "rank0": {"avg_launch_ms": avg_dur * 1e3, "achieved": achieved_gbs,
                      "frac": achieved_gbs / HBM_PEAK_GBS},
            "event_scope": ("one event pair over the timed region (one graph replay of the K "
                            "steps): includes the gaps between kernel nodes"
                            if step_graph is not None else "one event pair per launch"),
            "units_per_s_in_kernel": float(units_ev.sum() / durs.sum()),
            "write_probe_gbs": probe_gbs,
            "frac_of_write_probe": ((achieved_gbs / probe2_gbs) if probe2_gbs else
                                    (achieved_gbs / probe_gbs) if probe_gbs else None),
            "write_probe_two_stream_gbs": probe2_gbs,
            "probe_shape": ("two streams (even / odd allocations), as the steps2 graph runs its steps"
                            if probe2_gbs else "one stream"),
            "kernel_isolated": kernel_iso,
            # rank 0's launches of the kernel, in dispatch order: a rocprofv3
            # kernel trace of this command holds `before` launches, then the
            # `timed` ones this line's avg_launch_ms covers, then `after`
            "dispatch_window": {"kernel": kernel, "before": window_start, "timed": window_timed,
                                "after": dispatched[0] - window_start - window_timed,
                                "slots": n_slots, "launches_per_step": len(chunks)},
        },
        "cpu_baseline": cpu,
        "pcie_inclusive": pcie,
        "parity": parity,
        "parity_rows": parity_rows,
        "parity_rows_detail": parity_detail,
    }
    if per_slot:
        out["roofline"]["per_slot"] = per_slot
    if traffic:
        out["roofline"]["traffic_source"] = traffic.get("source")
    # ---- the association the reference returns, under the same clock: the
    # default C3 run on one GPU also times c2match (cube-free, the product path
    # of match_captures) after the C3 line's own parity, with its own parity
    # against the CPU chain, nested in this line ----------
    nested_ok = True
    if args.workload == "c3" and world == 1 and args.c2match == "auto":
        out_slots.clear()                 # C3's 253 GB of output allocations
        chunks.clear()
        graphs = step_graph = gatherer = None
        argmin = minval = alt_rows = None
        torch.cuda.synchronize(dev)
        torch.cuda.empty_cache()
        t0 = time.perf_counter()
        nested, nested_ok = match_line(args, env, dict(WORKLOADS["c2match"]), None, steps=20, warmup=3,
                                       cube_mode="free", cpu_seconds=min(args.cpu_seconds, 5.0),
                                       pipeline=args.match_pipeline == "on")
        nested["wall_s"] = time.perf_counter() - t0
        nested["note"] = ("BASELINE configs[1]'s association (C2: 1,000 captures x 3 x 256, what "
                          "match_objects returns), run after this line's timed region on the same "
                          "GPU; its own steps, clock and parity")
        out["c2match"] = nested
    print(json.dumps(out), flush=True)
    if parity_detail and parity_detail["rows_bit_exact"] != parity_detail["rows_checked"]:
        log(f"error: association parity {parity_rows}")
        raise SystemExit(3)
    if not parity_ok:
        log(f"error: residual parity {parity}")
        raise SystemExit(3)
    if not nested_ok:
        log("error: c2match parity (nested)")
        raise SystemExit(3)


if __name__ == "__main__":
    main()
