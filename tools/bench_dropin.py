"""Latency of the drop-in matching stage at the sizes the Inference Notebook
runs.  The notebook's matcher problems are (4, 4, 4) and
(2, 2, 2) detections per view (Inference Notebook.ipynb JSON lines 69, 180;
call sites /root/reference/bpc/inference/process_pose.py:165,182); 24 and 64
show where the crossover lies.

Per size, one synthetic IPD-like capture (bpc_baseline_amd.synth.make_capture):
  gpu  compute_cost_matrix + match_objects of the drop-in module, called
       exactly as process_pose.py:165,182 calls them (dict detections in,
       NumPy cube / match list out), and the whole _match
       (match_detections, quiet) -- wall clock per call, median;
  cpu  the reference's own cost model: oracle/reference_loop.py's per-pair
       NumPy triple loop (the as-written compute_cost_matrix) + scipy
       linear_sum_assignment + the threshold / decode of match_objects, and
       for _match also the sort and numpy-SVD triangulation -- one core.
The matches of both paths must be equal.  Prints one JSON object.

python tools/bench_dropin.py [--sizes 2,4,24,64] [--seconds 1.0]
"""
import argparse
import json
import os
import platform
import statistics
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scipy.optimize import linear_sum_assignment as scipy_lsa  # noqa: E402

from bpc_baseline_amd.inference import epipolar_matching as em  # noqa: E402
from bpc_baseline_amd.inference.process_pose import match_detections  # noqa: E402
from bpc_baseline_amd.inference.utils.camera_utils import compute_fundamental_matrix  # noqa: E402
from bpc_baseline_amd.synth import make_capture  # noqa: E402
from oracle import reference_loop as RL  # noqa: E402


class Capture:
    def __init__(self, Ks, RTs):
        self.Ks, self.RTs, self.images = list(Ks), list(RTs), [None] * len(Ks)


def timed(fn, seconds, max_reps=10000, warm=3):
    """Median wall time of fn() over ~seconds (`warm` warm-up calls first)."""
    for _ in range(warm):
        out = fn()
    ts = []
    t_end = time.perf_counter() + seconds
    while len(ts) < max_reps and (len(ts) < min(5, max_reps) or time.perf_counter() < t_end):
        t0 = time.perf_counter()
        out = fn()
        ts.append(time.perf_counter() - t0)
    return statistics.median(ts) * 1e3, len(ts), out


def cpu_match_objects(cube, threshold):
    N, M, P = cube.shape
    flat = cube.reshape(N * M, P)
    r, c = scipy_lsa(flat)
    return [(int(a) // M, int(a) % M, int(b)) for a, b in zip(r, c) if flat[a, b] < threshold]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="2,4,24,64")
    ap.add_argument("--seconds", type=float, default=1.0)
    ap.add_argument("--threshold", type=float, default=30.0)
    args = ap.parse_args()
    import torch
    torch.cuda.init()
    rows = []
    for n in (int(x) for x in args.sizes.split(",")):
        rng = np.random.default_rng(100 + n)
        Ks, RTs, dets = make_capture(rng, 3, n)
        d1, d2, d3 = dets[0], dets[1], dets[2]
        R = [rt[:3, :3] for rt in RTs]
        t = [rt[:3, 3] for rt in RTs]
        F12 = compute_fundamental_matrix(Ks[0], R[0], t[0], Ks[1], R[1], t[1])
        F13 = compute_fundamental_matrix(Ks[0], R[0], t[0], Ks[2], R[2], t[2])
        F23 = compute_fundamental_matrix(Ks[1], R[1], t[1], Ks[2], R[2], t[2])
        c1, c2, c3 = ([d["bb_center"] for d in dd] for dd in (d1, d2, d3))

        def gpu_stage():
            cube = em.compute_cost_matrix(d1, d2, d3, F12, F13, F23)
            return cube, em.match_objects(cube, args.threshold)

        def gpu_cube():
            return em.compute_cost_matrix(d1, d2, d3, F12, F13, F23)

        cube0 = gpu_cube()

        def gpu_lsap():
            return em.match_objects(cube0, args.threshold)

        def cpu_stage():
            cube = RL.cube(c1, c2, c3, F12, F13, F23)
            return cube, cpu_match_objects(cube, args.threshold)

        cap = Capture(Ks, RTs)

        def gpu_match():
            np.random.seed(0)
            return match_detections(cap, dets, verbose=False)

        def cpu_match():
            # _match's host steps as the reference runs them (process_pose.py:
            # 157-187): F's, the cube, the stats draws, the assignment, the
            # cost sort and one DLT per match (PosePrediction.triangulate)
            f12 = compute_fundamental_matrix(Ks[0], R[0], t[0], Ks[1], R[1], t[1])
            f13 = compute_fundamental_matrix(Ks[0], R[0], t[0], Ks[2], R[2], t[2])
            f23 = compute_fundamental_matrix(Ks[1], R[1], t[1], Ks[2], R[2], t[2])
            cube = RL.cube(c1, c2, c3, f12, f13, f23)
            np.random.seed(0)
            for _ in range(min(5, cube.size)):   # _match's stats samples (global RNG)
                np.random.randint(0, n), np.random.randint(0, n), np.random.randint(0, n)
            m = cpu_match_objects(cube, args.threshold)
            out = []
            for i, j, k in sorted(m, key=lambda q: cube[q[0], q[1], q[2]]):
                proj = [Ks[c] @ RTs[c][:3] for c in range(3)]
                out.append(em.triangulate_multi_view(proj, np.array([c1[i], c2[j], c3[k]])))
            return out

        t_gpu, k_gpu, (gcube, gm) = timed(gpu_stage, args.seconds)
        t_gcube, _, _ = timed(gpu_cube, args.seconds / 2)
        t_glsap, _, _ = timed(gpu_lsap, args.seconds / 2)
        t_gmatch, _, gpred = timed(gpu_match, args.seconds)
        big = n > 24   # 64^3 = 262k triples at ~80 us each: one timed call, no warm-up
        t_cpu, k_cpu, (ccube, cm) = timed(cpu_stage, args.seconds, max_reps=1 if big else 10000,
                                          warm=0 if big else 3)
        t_cmatch, _, cpred = timed(cpu_match, args.seconds, max_reps=1 if big else 10000,
                                   warm=0 if big else 3)
        assert np.array_equal(gcube.view(np.int32), ccube.view(np.int32)), n
        assert [tuple(int(v) for v in q) for q in gm] == cm, n
        assert len(gpred) == len(cpred)
        for p, x in zip(gpred, cpred):
            np.testing.assert_allclose(p.t, x, rtol=1e-9)
        rows.append({"n": n, "matches": len(cm),
                     "gpu_ms": {"cost_matrix+match_objects": t_gpu, "compute_cost_matrix": t_gcube,
                                "match_objects": t_glsap, "_match": t_gmatch},
                     "cpu_ms": {"cost_matrix+match_objects": t_cpu, "_match": t_cmatch},
                     "speedup_stage": t_cpu / t_gpu, "speedup_match": t_cmatch / t_gmatch,
                     "reps": {"gpu": k_gpu, "cpu": k_cpu}})
        print(f"n={n}: gpu {t_gpu:.3f} ms (cube {t_gcube:.3f}, lsap {t_glsap:.3f}, _match {t_gmatch:.3f}) "
              f"cpu {t_cpu:.3f} ms (_match {t_cmatch:.3f})", file=sys.stderr)
    # mixed shapes: consecutive calls with different detection counts (1..8
    # per view, > 32 distinct shapes, as a real capture stream has): every
    # call a different (N, M, P), so no call repeats the previous one's shape
    rng = np.random.default_rng(7)
    shapes = sorted({tuple(int(x) for x in rng.integers(1, 9, 3)) for _ in range(400)})
    rng.shuffle(shapes)
    calls = []
    for q, counts in enumerate(shapes):
        Ks, RTs, dets = make_capture(np.random.default_rng(5000 + q), 3, max(counts))
        dd = [dets[c][:counts[c]] for c in range(3)]
        R = [rt[:3, :3] for rt in RTs]
        t = [rt[:3, 3] for rt in RTs]
        Fs = (compute_fundamental_matrix(Ks[0], R[0], t[0], Ks[1], R[1], t[1]),
              compute_fundamental_matrix(Ks[0], R[0], t[0], Ks[2], R[2], t[2]),
              compute_fundamental_matrix(Ks[1], R[1], t[1], Ks[2], R[2], t[2]))
        calls.append((dd, Fs))
    from bpc_baseline_amd.inference import capture_session
    capture_session.clear()

    def sweep(gpu):
        ts, res = [], []
        for dd, Fs in calls:
            t0 = time.perf_counter()
            if gpu:
                cube = em.compute_cost_matrix(*dd, *Fs)
                m = [tuple(int(v) for v in q) for q in em.match_objects(cube, args.threshold)]
            else:
                cube = RL.cube(*([d["bb_center"] for d in v] for v in dd), *Fs)
                m = cpu_match_objects(cube, args.threshold)
            ts.append(time.perf_counter() - t0)
            res.append(m)
        return ts, res

    g_cold, g_res = sweep(True)       # first pass: includes every slot build (cold)
    g_warm, _ = sweep(True)
    c_ts, c_res = sweep(False)
    assert g_res == c_res
    mixed = {"distinct_shapes": len(calls), "counts": "1..8 per view, shuffled",
             "gpu_ms_median_first_pass": statistics.median(g_cold) * 1e3,
             "gpu_ms_first_call": g_cold[0] * 1e3,
             "gpu_ms_median_second_pass": statistics.median(g_warm) * 1e3,
             "cpu_ms_median": statistics.median(c_ts) * 1e3,
             "slots_after": capture_session.cache_info(),
             "note": "cost_matrix+match_objects per call; the first pass includes building the "
                     "capacity-class slots (one cube slot and a few assignment slots for all "
                     "shapes), first_call the very first build"}
    print(f"mixed: gpu {mixed['gpu_ms_median_first_pass']:.3f} ms first pass, "
          f"{mixed['gpu_ms_median_second_pass']:.3f} ms second; cpu {mixed['cpu_ms_median']:.3f} ms",
          file=sys.stderr)
    out = {"what": "drop-in matching stage latency per capture (wall clock, median)",
           "mixed_shapes": mixed,
           "cpu": platform.processor() or platform.machine(), "cpu_cores": 1,
           "gpu": torch.cuda.get_device_name(0), "rows": rows}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
