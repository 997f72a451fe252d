"""CPU restatement of the steps either side of the matcher.

TEST INFRASTRUCTURE ONLY: the checker for mvm_pack_detections and
mvm_triangulate_dlt (bpc_baseline_amd/csrc/mvm_pipeline.hip).  Pinned against
tests/golden/a8_detect.npz and a9_triangulate.npz, which hold the reference's
own outputs (oracle/gen_golden.py).
"""
from __future__ import annotations

import numpy as np


def detect_pack(boxes: np.ndarray, conf: np.ndarray, cls: np.ndarray, in_offs: np.ndarray,
                thresh: float, class_id: float = 0.0):
    """PoseEstimator._detect's packing (bpc/inference/process_pose.py:122-140),
    over a CSR batch of images.

    Per image: ``valid = (cls == 0) & (conf >= thresh)`` in float32 (:130; a
    Python float against a float32 array compares in float32), boxes kept in
    order, ``int()`` of each float32 coordinate (:134, toward zero), centre
    ``0.5 * (x1 + x2)`` as float64 (:135-136).
    -> (bbox int64 [k, 4], center f64 [k, 2], out_offs int64 [n_img + 1]).
    """
    boxes = np.asarray(boxes, np.float32).reshape(-1, 4)
    conf = np.asarray(conf, np.float32)
    cls = np.asarray(cls, np.float32)
    in_offs = np.asarray(in_offs, np.int64)
    t32 = np.float32(thresh)
    bbox, center, counts = [], [], []
    for k in range(in_offs.size - 1):
        b, e = int(in_offs[k]), int(in_offs[k + 1])
        valid = (cls[b:e] == np.float32(class_id)) & (conf[b:e] >= t32)
        kept = boxes[b:e][valid]
        q = np.trunc(kept.astype(np.float64)).astype(np.int64)
        bbox.append(q)
        center.append(np.stack([0.5 * (q[:, 0] + q[:, 2]), 0.5 * (q[:, 1] + q[:, 3])], axis=1)
                      .astype(np.float64))
        counts.append(q.shape[0])
    out_offs = np.zeros(len(counts) + 1, np.int64)
    out_offs[1:] = np.cumsum(counts)
    return (np.concatenate(bbox).reshape(-1, 4) if bbox else np.zeros((0, 4), np.int64),
            np.concatenate(center).reshape(-1, 2) if center else np.zeros((0, 2)),
            out_offs)


def triangulate(proj: np.ndarray, pts: np.ndarray) -> np.ndarray:
    """triangulate_multi_view (bpc/inference/epipolar_matching.py:118-127) for
    a stack of systems: proj [n, V, 3, 4], pts [n, V, 2] -> X [n, 3].

    A row pair per view ``x * P[2] - P[0]``, ``y * P[2] - P[1]``; X is the last
    row of Vt from numpy's SVD, returned as X[:3] / X[3].
    """
    proj = np.asarray(proj, np.float64)
    pts = np.asarray(pts, np.float64)
    n, V = proj.shape[:2]
    A = np.empty((n, 2 * V, 4))
    A[:, 0::2] = pts[:, :, 0:1] * proj[:, :, 2] - proj[:, :, 0]
    A[:, 1::2] = pts[:, :, 1:2] * proj[:, :, 2] - proj[:, :, 1]
    X = np.empty((n, 3))
    for q in range(n):
        _, _, Vt = np.linalg.svd(A[q])
        X[q] = Vt[-1][:3] / Vt[-1][3]
    return X
