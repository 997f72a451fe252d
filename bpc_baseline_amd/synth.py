"""Seeded synthetic IPD-like multi-camera scenes (SURVEY §8d generator).

The IPD dataset and YOLO weights are not available offline, so the benchmark
and the parity tests use synthetic captures shaped like IPD:

* rig: ``n_cams`` cameras with the IPD intrinsics of
  ``blog/documentation.md:71`` (f = 4209.03 px, 2400 x 2400 principal point
  1200), all looking at the world origin from ~1650 mm (the documented
  ``cam_t_w2c`` is (119, 48, 1649)), spread in yaw by 0.35 rad, jittered;
  R and t are float32 (``load_camera_params``) promoted to a float64 [R|t]
  (``calc_pose_matrix``);
* detections: half of each view are projections of shared 3-D object centres
  in [-250,250]^2 x [-80,80] mm plus N(0, 1.5 px) noise, half are clutter
  uniform in the image; each centroid is built the way ``_detect`` does it
  (``process_pose.py:134-136``): integer box corners, centre = 0.5*(x1+x2),
  so every centroid is a half-integer; each view is randomly permuted.

Scene ``s`` draws from ``np.random.default_rng(seed + s)`` so any rank can
build its own shard of scenes without generating the others.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional

import numpy as np

from .inference.utils.camera_utils import (calc_pose_matrix, camera_pairs,
                                           fundamental_matrices_batched)

__all__ = ["IPD_K", "SceneBatch", "make_rig", "make_capture", "make_scenes"]

# blog/documentation.md:71 (scene_camera_cam1.json example)
IPD_K = np.array([[4209.025366776721, 0.0, 1200.0],
                  [0.0, 4209.025366776721, 1200.0],
                  [0.0, 0.0, 1.0]], dtype=np.float32)
IMAGE_SIZE = 2400.0


def _rot_x(a: float) -> np.ndarray:
    c, s = np.cos(a), np.sin(a)
    return np.array([[1, 0, 0], [0, c, -s], [0, s, c]])


def _rot_y(a: float) -> np.ndarray:
    c, s = np.cos(a), np.sin(a)
    return np.array([[c, 0, s], [0, 1, 0], [-s, 0, c]])


def _rot_z(a: float) -> np.ndarray:
    c, s = np.cos(a), np.sin(a)
    return np.array([[c, -s, 0], [s, c, 0], [0, 0, 1]])


def make_rig(rng: np.random.Generator, n_cams: int):
    """IPD-like rig -> (Ks list of f32[3,3], RTs list of f64[4,4])."""
    Ks, RTs = [], []
    for c in range(n_cams):
        yaw = (c - (n_cams - 1) / 2.0) * 0.35 + rng.normal(0.0, 0.01)
        roll = 0.05 * c + rng.normal(0.0, 0.01)
        tilt = np.pi + rng.normal(0.0, 0.01)
        R = (_rot_z(roll) @ _rot_y(yaw) @ _rot_x(tilt)).astype(np.float32)
        t = (np.array([0.0, 10.0 * c, 1650.0]) + rng.normal(0.0, 5.0, size=3)).astype(np.float32)
        Ks.append(IPD_K.copy())
        RTs.append(calc_pose_matrix(R, t))
    return Ks, RTs


def _project(K: np.ndarray, RT: np.ndarray, X: np.ndarray) -> np.ndarray:
    cam = X @ RT[:3, :3].T + RT[:3, 3]
    uv = cam @ K.astype(np.float64).T
    return uv[:, :2] / uv[:, 2:3]


def _views(rng: np.random.Generator, Ks, RTs, counts, *, box_px: float, noise_px: float):
    """Per-camera integer boxes and half-integer centres (arrays)."""
    n_obj = max(counts) // 2 if counts else 0
    X = np.stack([rng.uniform(-250, 250, n_obj), rng.uniform(-250, 250, n_obj),
                  rng.uniform(-80, 80, n_obj)], axis=1)
    views = []
    for c, n in enumerate(counts):
        k = min(n // 2, n_obj)
        true_uv = _project(Ks[c], RTs[c], X[:k]) + rng.normal(0.0, noise_px, size=(k, 2))
        clutter = rng.uniform(0.0, IMAGE_SIZE, size=(n - k, 2))
        centres = np.concatenate([true_uv, clutter], axis=0)[rng.permutation(n)]
        half = np.abs(rng.normal(box_px / 2, box_px / 8, size=(n, 2))) + 1.0
        # int(box) truncates toward zero (process_pose.py:134)
        boxes = np.trunc(np.concatenate([centres - half, centres + half], axis=1)).astype(np.int64)
        cxy = 0.5 * (boxes[:, 0:2] + boxes[:, 2:4])          # process_pose.py:135-136
        views.append((boxes, cxy.astype(np.float64)))
    return views


def make_capture(rng: np.random.Generator, n_cams: int, n_dets, *, box_px: float = 80.0,
                 noise_px: float = 1.5, duplicates: int = 0):
    """One capture: rig + per-camera detections in the reference's dict format.

    ``n_dets`` is an int or a per-camera list.  Returns
    ``(Ks, RTs, detections)`` with ``detections = {cam: [{'bbox': (x1,y1,x2,y2),
    'bb_center': (cx, cy)}, ...]}`` exactly as ``PoseEstimator._detect`` builds
    it (process_pose.py:133-140: Python ints and floats).  ``duplicates``
    repeats the first few detections of every view (exact ties for the argmin
    and Hungarian tests).
    """
    counts = [int(n_dets)] * n_cams if np.isscalar(n_dets) else [int(n) for n in n_dets]
    Ks, RTs = make_rig(rng, n_cams)
    detections: Dict[int, List[dict]] = {}
    for c, (boxes, cxy) in enumerate(_views(rng, Ks, RTs, counts, box_px=box_px, noise_px=noise_px)):
        dets = [{"bbox": tuple(int(v) for v in b), "bb_center": (float(x), float(y))}
                for b, (x, y) in zip(boxes, cxy)]
        dets.extend(dict(d) for d in dets[:duplicates])
        detections[c] = dets
    return Ks, RTs, detections


@dataclass
class SceneBatch:
    """A batch of scenes in the matcher's device layout (host numpy copy).

    pts       f64 [sum n, 2]  centroids, scene-major then camera-minor
    cam_offs  i64 [S*C + 1]   CSR offsets of (scene, camera) into ``pts``
    F         f64 [S*P, 9]    fundamental matrix of (scene, pair), row-major
    pairs     i32 [P, 2]      camera pair (a, b) of each pair slot
    """
    pts: np.ndarray
    cam_offs: np.ndarray
    F: np.ndarray
    pairs: np.ndarray
    n_scenes: int
    n_cams: int
    seed: int = 0
    meta: dict = field(default_factory=dict)   # also the rig: Ks f32 [S,C,3,3], RTs f64 [S,C,4,4]

    @property
    def n_pairs(self) -> int:
        return int(self.pairs.shape[0])

    def counts(self) -> np.ndarray:
        return np.diff(self.cam_offs).reshape(self.n_scenes, self.n_cams)

    def n_residual_pairs(self) -> int:
        c = self.counts()
        return int(sum((c[:, a] * c[:, b]).sum() for a, b in self.pairs))


def make_scenes(n_scenes: int, n_cams: int, n_dets, *, seed: int = 0, first_scene: int = 0,
                ragged: bool = False, pairs: Optional[np.ndarray] = None) -> SceneBatch:
    """Scenes ``first_scene .. first_scene + n_scenes - 1`` of the seeded family.

    ``n_dets`` is one count for every view or a per-camera list;
    ``ragged=True`` draws each view's count uniformly from [0, n_dets] (empty
    views included) instead.
    """
    if pairs is None:
        pairs = camera_pairs(n_cams)
    pts_parts: List[np.ndarray] = []
    counts = np.zeros((n_scenes, n_cams), dtype=np.int64)
    K_all = np.empty((n_scenes, n_cams, 3, 3), dtype=np.float32)
    RT_all = np.empty((n_scenes, n_cams, 4, 4), dtype=np.float64)
    for s in range(n_scenes):
        rng = np.random.default_rng(seed + first_scene + s)
        if ragged:
            per_view = rng.integers(0, int(n_dets) + 1, size=n_cams)
        else:
            per_view = [int(n_dets)] * n_cams if np.isscalar(n_dets) else [int(x) for x in n_dets]
        Ks, RTs = make_rig(rng, n_cams)
        K_all[s], RT_all[s] = np.stack(Ks), np.stack(RTs)
        for c, (_, cxy) in enumerate(_views(rng, Ks, RTs, list(per_view), box_px=80.0, noise_px=1.5)):
            counts[s, c] = len(cxy)
            pts_parts.append(cxy)
    F = fundamental_matrices_batched(K_all, RT_all, pairs) if n_scenes else np.zeros((0, 9))
    cam_offs = np.zeros(n_scenes * n_cams + 1, dtype=np.int64)
    np.cumsum(counts.reshape(-1), out=cam_offs[1:])
    pts = np.concatenate(pts_parts, axis=0) if pts_parts else np.zeros((0, 2))
    return SceneBatch(pts=np.ascontiguousarray(pts), cam_offs=cam_offs,
                      F=np.ascontiguousarray(F), pairs=np.asarray(pairs, np.int32),
                      n_scenes=n_scenes, n_cams=n_cams, seed=seed,
                      meta={"first_scene": first_scene, "n_dets": n_dets, "ragged": ragged,
                            "Ks": K_all, "RTs": RT_all})


@dataclass
class DetectorBatch:
    """Synthetic detector outputs of S 3-camera captures (what YOLO's
    ``results.boxes`` would hold), image 3s + c = capture s, camera c.

    boxes  f32 [n, 4] xyxy with fractional parts (int() truncates them)
    conf   f32 [n]    true detections >= 0.2; clutter partly below threshold
    cls    f32 [n]    0 for the object, 1 for some clutter
    img_offs i64 [3S + 1]
    Ks f32 [S, 3, 3, 3], RTs f64 [S, 3, 4, 4]
    """
    boxes: np.ndarray
    conf: np.ndarray
    cls: np.ndarray
    img_offs: np.ndarray
    Ks: np.ndarray
    RTs: np.ndarray

    @property
    def n_captures(self) -> int:
        return int(self.Ks.shape[0])


def make_detector_batch(n_captures: int, n_dets: int, *, seed: int = 0, clutter: int = 4,
                        first_capture: int = 0) -> DetectorBatch:
    """Per capture ``rng = default_rng(seed + first_capture + s)``: an IPD-like
    rig, ``n_dets`` boxes per view from ``_views`` (half true objects, half
    clutter) with sub-pixel offsets, plus up to ``clutter`` detector boxes per
    view that the conf/class filter of _detect (process_pose.py:130) drops."""
    boxes, conf, cls, counts = [], [], [], []
    Ks_all = np.empty((n_captures, 3, 3, 3), np.float32)
    RTs_all = np.empty((n_captures, 3, 4, 4), np.float64)
    for s in range(n_captures):
        rng = np.random.default_rng(seed + first_capture + s)
        Ks, RTs = make_rig(rng, 3)
        Ks_all[s], RTs_all[s] = np.stack(Ks), np.stack(RTs)
        for b, _ in _views(rng, Ks, RTs, [n_dets] * 3, box_px=80.0, noise_px=1.5):
            b = np.asarray(b, np.float64).reshape(-1, 4)
            b = b + np.where(b >= 0, 1.0, -1.0) * rng.uniform(0.0, 0.999, b.shape)
            nj = int(rng.integers(0, clutter + 1))
            jb = rng.uniform(0.0, IMAGE_SIZE, (nj, 4))
            jc = np.where(rng.random(nj) < 0.5, rng.uniform(0.0, 0.09, nj), 0.9)
            jk = np.where(jc > 0.5, 1.0, 0.0)
            per = rng.permutation(len(b) + nj)
            boxes.append(np.concatenate([b, jb])[per])
            conf.append(np.concatenate([rng.uniform(0.2, 1.0, len(b)), jc])[per])
            cls.append(np.concatenate([np.zeros(len(b)), jk])[per])
            counts.append(len(b) + nj)
    img_offs = np.zeros(3 * n_captures + 1, np.int64)
    np.cumsum(counts, out=img_offs[1:])
    cat = lambda xs, w: (np.concatenate(xs) if xs else np.zeros((0,) + w))
    return DetectorBatch(boxes=np.ascontiguousarray(cat(boxes, (4,)), np.float32).reshape(-1, 4),
                         conf=np.ascontiguousarray(cat(conf, ()), np.float32),
                         cls=np.ascontiguousarray(cat(cls, ()), np.float32),
                         img_offs=img_offs, Ks=Ks_all, RTs=RTs_all)
