#!/usr/bin/env python3
"""Generate the golden parity fixtures under tests/golden/ by running the
REFERENCE's own hot-path code (bpc/inference) in the build container.

TEST INFRASTRUCTURE ONLY.  The reference exists only in the build container
(/root/reference, read-only); the GPU box never sees it.  Its Python is
imported here with stub modules for the imports the hot path does not use
(cv2 is needed only by the dead visualisation branch of epipolar_error,
epipolar_matching.py:31-69; process_pose additionally imports torchvision,
pyrender and ultralytics for the YOLO / ResNet parts outside the matcher).
Nothing from the reference is copied: only inputs and the reference's outputs
are stored, as arrays.

Fixtures (all .npz, loaded with allow_pickle=False):
  a1_epipolar_error.npz  scalar epipolar_error / epipolar_error_full KATs (fp64 outputs)
  a3_cost_cubes.npz      compute_cost_matrix cubes + match_objects + argmin rows
  a3b_cost_cubes_mid.npz compute_cost_matrix cubes at the fused kernel's lane/tile
                         boundaries (views of 47/48, 97, 150, 250) + argmin rows
  a5_pairwise.npz        4-camera pairwise residual matrices (f32 of epipolar_error)
  a6_fundamental.npz     compute_fundamental_matrix on IPD-like rigs
  a7_match.npz           PoseEstimator._match on synthetic captures (matches, t)
  a8_detect.npz          PoseEstimator._detect box packing, detector replaced by a stub
                         returning synthetic boxes/confidences/classes
  a9_triangulate.npz     triangulate_multi_view on 2/3/4/8-view systems

Run: python oracle/gen_golden.py [--reference /root/reference]
"""
from __future__ import annotations

import argparse
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, REPO)

from bpc_baseline_amd.synth import make_capture  # noqa: E402  (input generator only)

OUT = os.path.join(REPO, "tests", "golden")


def _stub_modules():
    """Empty stand-ins for imports the matcher never executes."""
    def mod(name, **attrs):
        m = types.ModuleType(name)
        m.__dict__.update(attrs)
        sys.modules[name] = m
        return m

    mod("cv2")
    tv = mod("torchvision")
    tv.transforms = mod("torchvision.transforms")
    tv.transforms.functional = mod("torchvision.transforms.functional")
    tv.models = mod("torchvision.models")
    mod("pyrender")
    mod("ultralytics", YOLO=None)


def _import_reference(ref_root: str):
    _stub_modules()
    sys.path.insert(0, ref_root)
    from bpc.inference import epipolar_matching as em
    from bpc.inference.utils import camera_utils as cu
    from bpc.inference import process_pose as pp
    return em, cu, pp


def _dets_array(dets):
    return np.asarray([d["bb_center"] for d in dets], dtype=np.float64).reshape(-1, 2)


def _boxes_array(dets):
    return np.asarray([d["bbox"] for d in dets], dtype=np.int64).reshape(-1, 4)


def gen_a1(em, rng):
    """Scalar KATs for epipolar_error (:5-28) and epipolar_error_full (:73-81)."""
    F, P1, P2, kind = [], [], [], []

    def add(f, p1, p2, k):
        F.append(np.asarray(f, np.float64).reshape(9))
        P1.append(p1)
        P2.append(p2)
        kind.append(k)

    for _ in range(600):                                    # random geometry, real-valued points
        add(rng.normal(size=(3, 3)), rng.normal(size=2) * 1000, rng.normal(size=2) * 1000, 0)
    for _ in range(600):                                    # IPD-like rig, half-integer centroids
        Ks, RTs, dets = make_capture(rng, 2, 1)
        from bpc_baseline_amd.inference.utils.camera_utils import compute_fundamental_matrix
        f = compute_fundamental_matrix(Ks[0], RTs[0][:3, :3], RTs[0][:3, 3],
                                       Ks[1], RTs[1][:3, :3], RTs[1][:3, 3])
        add(f, np.floor(rng.uniform(0, 4800, 2)) / 2, np.floor(rng.uniform(0, 4800, 2)) / 2, 1)
    for _ in range(50):                                     # degenerate l2 (F rows 0,1 = 0) -> 9999
        f = rng.normal(size=(3, 3)); f[0:2, :] = 0
        add(f, rng.normal(size=2) * 100, rng.normal(size=2) * 100, 2)
    for _ in range(50):                                     # degenerate l1 (F cols 0,1 = 0) -> 9999
        f = rng.normal(size=(3, 3)); f[:, 0:2] = 0
        add(f, rng.normal(size=2) * 100, rng.normal(size=2) * 100, 3)
    for _ in range(20):                                     # both degenerate
        add(np.zeros((3, 3)), rng.normal(size=2), rng.normal(size=2), 4)
    for scale in np.geomspace(1e-11, 1e-6, 60):             # norms straddling the 1e-8 threshold
        f = rng.normal(size=(3, 3)) * scale
        add(f, rng.normal(size=2) * 3, rng.normal(size=2) * 3, 5)
    for _ in range(40):                                     # point exactly on the epipolar line (d = 0)
        f = np.zeros((3, 3)); f[2, 2] = 0.0; f[0, 1] = 1.0; f[1, 0] = -1.0
        x = float(rng.integers(0, 100))
        add(f, np.array([x, x]), np.array([2 * x, 2 * x]), 6)
    F, P1, P2, kind = map(np.asarray, (F, P1, P2, kind))
    e = np.array([em.epipolar_error(tuple(p1), tuple(p2), f.reshape(3, 3))
                  for f, p1, p2 in zip(F, P1, P2)], dtype=np.float64)

    # epipolar_error_full on IPD-like triples
    n3 = 300
    F3 = np.empty((n3, 3, 9)); Q = np.empty((n3, 3, 2))
    for t in range(n3):
        Ks, RTs, dets = make_capture(rng, 3, 1)
        from bpc_baseline_amd.inference.utils.camera_utils import fundamental_matrices, camera_pairs
        F3[t] = fundamental_matrices(Ks, RTs, camera_pairs(3))
        Q[t] = np.floor(rng.uniform(0, 4800, (3, 2))) / 2
    efull = np.array([em.epipolar_error_full(tuple(q[0]), tuple(q[1]), tuple(q[2]),
                                             f[0].reshape(3, 3), f[1].reshape(3, 3), f[2].reshape(3, 3))
                      for f, q in zip(F3, Q)], dtype=np.float64)
    np.savez_compressed(os.path.join(OUT, "a1_epipolar_error.npz"), F=F, p1=P1, p2=P2, kind=kind,
                        e=e, full_F=F3, full_pts=Q, full_e=efull)
    print(f"a1: {len(e)} epipolar_error KATs, {n3} epipolar_error_full KATs")


CUBE_CASES = [
    # (name, counts (N, M, P), kind, extra)
    ("c1", (1, 1, 1), "rig", 0),
    ("c2", (2, 2, 2), "rig", 0),
    ("c4", (4, 4, 4), "rig", 0),
    ("c537", (5, 3, 7), "rig", 0),
    ("c16", (16, 16, 16), "rig", 0),
    ("c24", (24, 24, 24), "rig", 0),
    ("c32", (32, 32, 32), "rig", 0),
    ("dup", (6, 6, 6), "rig", 2),          # duplicated detections -> exact ties
    ("pgt", (2, 2, 9), "rig", 0),          # P > N*M (Hungarian leaves columns unassigned)
    ("rndF", (8, 8, 8), "randomF", 0),     # non-rig geometry, wide dynamic range
    ("degen", (5, 4, 6), "degenerate", 0), # F12 with zero rows -> 9999 sentinels
    ("wide", (3, 40, 70), "rig", 0),       # P not a multiple of 4, > 64
]


def gen_a3(em, rng):
    """compute_cost_matrix (:83-98), match_objects (:100-116), per-row argmin."""
    from bpc_baseline_amd.inference.utils.camera_utils import fundamental_matrices, camera_pairs
    arrays = {}
    for name, counts, kind, dup in CUBE_CASES:
        Ks, RTs, dets = make_capture(rng, 3, list(counts), duplicates=dup)
        F = fundamental_matrices(Ks, RTs, camera_pairs(3))
        if kind == "randomF":
            F = rng.normal(size=(3, 9))
        elif kind == "degenerate":
            F[0, 0:6] = 0.0
        F12, F13, F23 = (F[p].reshape(3, 3) for p in range(3))
        cube = em.compute_cost_matrix(dets[0], dets[1], dets[2], F12, F13, F23)
        assert cube.dtype == np.float32
        m30 = em.match_objects(cube, 30)
        minf = em.match_objects(cube, np.inf)
        N, M, P = cube.shape
        flat = cube.reshape(N * M, P)
        arrays[f"{name}_p1"] = _dets_array(dets[0])
        arrays[f"{name}_p2"] = _dets_array(dets[1])
        arrays[f"{name}_p3"] = _dets_array(dets[2])
        arrays[f"{name}_F"] = F
        arrays[f"{name}_cube"] = cube
        arrays[f"{name}_match30"] = np.asarray(m30, dtype=np.int64).reshape(-1, 3)
        arrays[f"{name}_matchinf"] = np.asarray(minf, dtype=np.int64).reshape(-1, 3)
        arrays[f"{name}_argmin"] = np.argmin(flat, axis=1).astype(np.int32)
        print(f"a3: {name} {cube.shape} matches@30={len(m30)}")
    arrays["names"] = np.asarray([c[0] for c in CUBE_CASES])
    np.savez_compressed(os.path.join(OUT, "a3_cost_cubes.npz"), **arrays)


# round 4: views on the fused cube kernel's lane / tile boundaries (3 k per
# lane with a partial last lane and 48-wide j tiles; P not a multiple of 4 at
# two and one rows per instruction), from a stream of their own so that the
# fixtures above regenerate byte-identically
CUBE_CASES_MID = [
    ("m48", (20, 48, 47), "rig", 0),
    ("m97", (10, 30, 97), "rig", 0),
    ("m150", (4, 20, 150), "rig", 0),
    ("m250", (3, 10, 250), "rig", 0),
]


def gen_a3b(em, rng):
    """compute_cost_matrix (:83-98) + the per-row argmin at the boundary sizes above."""
    from bpc_baseline_amd.inference.utils.camera_utils import fundamental_matrices, camera_pairs
    arrays = {}
    for name, counts, _, dup in CUBE_CASES_MID:
        Ks, RTs, dets = make_capture(rng, 3, list(counts), duplicates=dup)
        F = fundamental_matrices(Ks, RTs, camera_pairs(3))
        F12, F13, F23 = (F[p].reshape(3, 3) for p in range(3))
        cube = em.compute_cost_matrix(dets[0], dets[1], dets[2], F12, F13, F23)
        assert cube.dtype == np.float32
        N, M, P = cube.shape
        arrays[f"{name}_p1"] = _dets_array(dets[0])
        arrays[f"{name}_p2"] = _dets_array(dets[1])
        arrays[f"{name}_p3"] = _dets_array(dets[2])
        arrays[f"{name}_F"] = F
        arrays[f"{name}_cube"] = cube
        arrays[f"{name}_argmin"] = np.argmin(cube.reshape(N * M, P), axis=1).astype(np.int32)
        print(f"a3b: {name} {cube.shape}")
    arrays["names"] = np.asarray([c[0] for c in CUBE_CASES_MID])
    np.savez_compressed(os.path.join(OUT, "a3b_cost_cubes_mid.npz"), **arrays)


def gen_a5(em, rng):
    """4-camera pairwise mode: f32(epipolar_error(p_a[i], p_b[j], F_ab)) for every pair."""
    from bpc_baseline_amd.inference.utils.camera_utils import fundamental_matrices, camera_pairs
    counts = [12, 9, 0, 17]                # includes an empty view and non-multiple-of-4 widths
    Ks, RTs, dets = make_capture(rng, 4, counts, duplicates=1)
    pairs = camera_pairs(4)
    F = fundamental_matrices(Ks, RTs, pairs)
    arrays = {"pairs": pairs, "F": F}
    for c in range(4):
        arrays[f"pts{c}"] = _dets_array(dets[c])
    for p, (a, b) in enumerate(pairs):
        e = np.array([[em.epipolar_error(da["bb_center"], db["bb_center"], F[p].reshape(3, 3))
                       for db in dets[b]] for da in dets[a]], dtype=np.float64).reshape(len(dets[a]), len(dets[b]))
        arrays[f"e{a}{b}"] = e.astype(np.float32)
        arrays[f"argmin{a}{b}"] = (np.argmin(e.astype(np.float32), axis=1).astype(np.int32)
                                   if e.shape[1] else np.full(e.shape[0], -1, np.int32))
    np.savez_compressed(os.path.join(OUT, "a5_pairwise.npz"), **arrays)
    print(f"a5: pairwise 4-cam counts={counts}")


def gen_a6(cu, rng):
    """compute_fundamental_matrix (camera_utils.py:23-46) on IPD-like rigs."""
    from bpc_baseline_amd.synth import make_rig
    K, R, t, F = [], [], [], []
    for _ in range(40):
        Ks, RTs = make_rig(rng, 2)
        K.append(np.stack(Ks)); R.append(np.stack([x[:3, :3] for x in RTs]))
        t.append(np.stack([x[:3, 3] for x in RTs]))
        F.append(cu.compute_fundamental_matrix(Ks[0], RTs[0][:3, :3], RTs[0][:3, 3],
                                               Ks[1], RTs[1][:3, :3], RTs[1][:3, 3]))
    np.savez_compressed(os.path.join(OUT, "a6_fundamental.npz"), K=np.stack(K), R=np.stack(R),
                        t=np.stack(t), F=np.stack(F))
    print("a6: 40 fundamental matrices")


def gen_a7(pp, rng):
    """PoseEstimator._match (process_pose.py:144-188) on synthetic captures."""
    class _Capture:
        def __init__(self, Ks, RTs):
            self.Ks, self.RTs, self.images = Ks, RTs, [None] * len(Ks)

    est = pp.PoseEstimator.__new__(pp.PoseEstimator)      # skip YOLO / ResNet loading
    est.params = pp.PoseEstimatorParams()
    arrays = {}
    configs = [(4, 4, 4), (2, 2, 2), (6, 5, 7), (10, 10, 10), (3, 0, 3), (8, 8, 8)]
    state = np.random.get_state()
    for c, counts in enumerate(configs):
        Ks, RTs, dets = make_capture(rng, 3, list(counts), noise_px=0.6)
        np.random.seed(1234 + c)             # _match prints samples drawn from global np.random
        preds = est._match(_Capture(Ks, RTs), dets)
        arrays[f"m{c}_K"] = np.stack(Ks)
        arrays[f"m{c}_RT"] = np.stack(RTs)
        for cam in range(3):
            arrays[f"m{c}_boxes{cam}"] = _boxes_array(dets[cam])
            arrays[f"m{c}_pts{cam}"] = _dets_array(dets[cam])
        arrays[f"m{c}_centroids"] = np.asarray([p.centroids for p in preds], np.float64).reshape(-1, 3, 2)
        arrays[f"m{c}_boxes"] = np.asarray([p.boxes for p in preds], np.int64).reshape(-1, 3, 4)
        arrays[f"m{c}_t"] = np.asarray([p.t for p in preds], np.float64).reshape(-1, 3)
        print(f"a7: capture {counts}: {len(preds)} predictions")
    np.random.set_state(state)
    arrays["n"] = np.asarray(len(configs))
    np.savez_compressed(os.path.join(OUT, "a7_match.npz"), **arrays)


class _StubBoxes:
    """What _detect reads from a YOLO result (process_pose.py:126-129)."""

    def __init__(self, xyxy, conf, cls):
        import torch
        self.xyxy = torch.from_numpy(xyxy)
        self.conf = torch.from_numpy(conf)
        self.cls = torch.from_numpy(cls)

    def __len__(self):
        return int(self.xyxy.shape[0])


class _StubYolo:
    def __init__(self, per_image):
        self.per_image = list(per_image)

    def __call__(self, image, imgsz=None):
        return [types.SimpleNamespace(boxes=_StubBoxes(*self.per_image.pop(0)))]


def _synthetic_yolo_outputs(rng, n_img, thresh):
    """Boxes with fractional, integral, negative and near-integer coordinates;
    confidences straddling the float32 threshold; classes 0/1/2."""
    out = []
    t32 = np.float32(thresh)
    for _ in range(n_img):
        n = int(rng.choice([0, 1, 3, 17, 40, 300]))
        x1 = rng.uniform(-4.0, 1900.0, n)
        y1 = rng.uniform(-4.0, 1100.0, n)
        w = rng.uniform(0.0, 300.0, n)
        h = rng.uniform(0.0, 300.0, n)
        xyxy = np.stack([x1, y1, x1 + w, y1 + h], axis=1).astype(np.float32)
        sel = rng.random(xyxy.shape) < 0.15
        xyxy[sel] = np.round(xyxy[sel])                               # exact integers
        sel = rng.random(xyxy.shape) < 0.1
        xyxy[sel] = np.nextafter(np.round(xyxy[sel]), np.float32(-np.inf))  # 5.9999995 etc.
        sel = rng.random(xyxy.shape) < 0.05
        xyxy[sel] = -rng.uniform(0.0, 0.999, int(sel.sum())).astype(np.float32)  # int() -> 0
        conf = rng.uniform(0.0, 1.0, n).astype(np.float32)
        pick = rng.random(n)
        conf[pick < 0.1] = t32
        conf[(pick >= 0.1) & (pick < 0.2)] = np.nextafter(t32, np.float32(-np.inf))
        cls = rng.choice(np.asarray([0.0, 0.0, 0.0, 1.0, 2.0], np.float32), n)
        out.append((xyxy, conf, cls))
    return out


def gen_a8(pp, rng):
    """PoseEstimator._detect (process_pose.py:116-142) with the detector stubbed."""
    est = pp.PoseEstimator.__new__(pp.PoseEstimator)
    arrays = {}
    sets = [(0.1, 12), (0.25, 9), (0.5, 6)]
    for c, (thresh, n_img) in enumerate(sets):
        est.params = pp.PoseEstimatorParams(yolo_conf_thresh=thresh)
        raw = _synthetic_yolo_outputs(rng, n_img, thresh)
        est.yolo = _StubYolo(raw)
        capture = types.SimpleNamespace(images=[np.zeros((4, 4, 3), np.uint8)] * n_img)
        preds = est._detect(capture)
        in_offs = np.zeros(n_img + 1, np.int64)
        out_offs = np.zeros(n_img + 1, np.int64)
        in_offs[1:] = np.cumsum([r[0].shape[0] for r in raw])
        out_offs[1:] = np.cumsum([len(preds[k]) for k in range(n_img)])
        arrays[f"d{c}_thresh"] = np.asarray(thresh)
        arrays[f"d{c}_in_offs"] = in_offs
        arrays[f"d{c}_boxes"] = np.concatenate([r[0] for r in raw]).reshape(-1, 4)
        arrays[f"d{c}_conf"] = np.concatenate([r[1] for r in raw])
        arrays[f"d{c}_cls"] = np.concatenate([r[2] for r in raw])
        arrays[f"d{c}_out_offs"] = out_offs
        arrays[f"d{c}_bbox"] = np.concatenate(
            [_boxes_array(preds[k]) for k in range(n_img)]).reshape(-1, 4)
        arrays[f"d{c}_center"] = np.concatenate(
            [_dets_array(preds[k]) for k in range(n_img)]).reshape(-1, 2)
        print(f"a8: thresh {thresh}: {n_img} images, {in_offs[-1]} boxes, {out_offs[-1]} kept")
    arrays["n"] = np.asarray(len(sets))
    np.savez_compressed(os.path.join(OUT, "a8_detect.npz"), **arrays)


def gen_a9(em, rng):
    """triangulate_multi_view (epipolar_matching.py:118-127): projections of
    random points through IPD-like rigs, with pixel noise, 2-8 views."""
    from bpc_baseline_amd.synth import make_rig
    arrays = {}
    for V in (2, 3, 4, 8):
        n = 64
        proj = np.empty((n, V, 3, 4))
        pts = np.empty((n, V, 2))
        X = np.empty((n, 3))
        for q in range(n):
            Ks, RTs = make_rig(rng, V)
            P = np.stack([Ks[v] @ RTs[v][:3] for v in range(V)])
            Xw = np.array([*rng.uniform(-250.0, 250.0, 2), rng.uniform(-80.0, 80.0), 1.0])
            uvw = P @ Xw
            uv = uvw[:, :2] / uvw[:, 2:3]
            # centroids are half-integers in the pipeline (0.5 * (x1 + x2))
            uv = np.round(2.0 * (uv + rng.normal(0.0, 2.0, uv.shape))) / 2.0
            proj[q], pts[q] = P, uv
            X[q] = em.triangulate_multi_view(list(P), uv)
        arrays[f"v{V}_proj"], arrays[f"v{V}_pts"], arrays[f"v{V}_X"] = proj, pts, X
        print(f"a9: {n} {V}-view systems")
    np.savez_compressed(os.path.join(OUT, "a9_triangulate.npz"), **arrays)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default="/root/reference")
    ap.add_argument("--only", default="", help="comma list, e.g. a8,a9 (default: all)")
    args = ap.parse_args()
    os.makedirs(OUT, exist_ok=True)
    em, cu, pp = _import_reference(args.reference)
    only = set(filter(None, args.only.split(",")))
    want = (lambda k: not only or k in only)
    rng = np.random.default_rng(20250509)
    if want("a1"):
        gen_a1(em, rng)
    if want("a3"):
        gen_a3(em, rng)
    if want("a5"):
        gen_a5(em, rng)
    if want("a6"):
        gen_a6(cu, rng)
    if want("a7"):
        gen_a7(pp, rng)
    # a8/a9 draw from their own stream so a1-a7 stay reproducible on their own
    rng2 = np.random.default_rng(20250510)
    if want("a8"):
        gen_a8(pp, rng2)
    if want("a9"):
        gen_a9(em, rng2)
    if want("a3b"):
        gen_a3b(em, np.random.default_rng(20250511))


if __name__ == "__main__":
    main()
