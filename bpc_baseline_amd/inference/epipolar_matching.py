"""Drop-in replacement for ``bpc/inference/epipolar_matching.py`` (MI355X).

Same names, signatures, return types and edge-case behaviour as the
reference module; the residual and cube arithmetic runs in the HIP kernels
of ``libmvmatch.so`` (via ``torch.ops.mvmatch``), bit-identical to the
reference's numpy evaluation:

  epipolar_error        (epipolar_matching.py:5-71)   -> np.float64
  epipolar_error_full   (epipolar_matching.py:73-81)  -> np.float64
  compute_cost_matrix   (epipolar_matching.py:83-98)  -> np.ndarray float32 (N, M, P)
  match_objects         (epipolar_matching.py:100-116)-> list[(i, j, k)]
  triangulate_multi_view(epipolar_matching.py:118-127)-> np.ndarray (3,)

``match_objects`` runs the assignment on the GPU (``mvm_lsap_solve``): the
same shortest-augmenting-path algorithm as scipy's ``linear_sum_assignment``,
with the same tie-breaking and output order.
``triangulate_multi_view`` keeps the reference's 6x4 SVD on the host.  The ``img*`` arguments only drove the
reference's matplotlib visualisation (:31-69, unreachable from
compute_cost_matrix); they are accepted and ignored.

There is no CPU fallback: without a GPU or without the built library every
residual entry point raises.
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

import numpy as np
import torch
from .. import ops
from .capture_session import cube_slot, lsap_slot

__all__ = [
    "epipolar_error", "epipolar_error_full", "compute_cost_matrix", "match_objects",
    "triangulate_multi_view", "compute_cost_matrices",
]


def _device() -> torch.device:
    if not torch.cuda.is_available():
        raise RuntimeError("bpc_baseline_amd matcher needs a ROCm GPU (no CPU path)")
    return torch.device("cuda", torch.cuda.current_device())


def _centroids(dets) -> np.ndarray:
    """Pack ``dets[*]['bb_center']`` (process_pose.py:135-140) as float64 [n, 2]."""
    return np.asarray([d["bb_center"] for d in dets], dtype=np.float64).reshape(-1, 2)


def _F(F) -> np.ndarray:
    # the reference multiplies the given F with float64 points; float32 F is
    # promoted, so float64 here is exact
    return np.ascontiguousarray(np.asarray(F, dtype=np.float64).reshape(9))


def _pairs_f64(views: Sequence[np.ndarray], Fs: Sequence, pairs: Sequence[Tuple[int, int]]):
    """fp64 residual matrices of several camera pairs of one capture (one launch)."""
    dev = _device()
    counts = [len(v) for v in views]
    cam_offs_h = np.zeros(len(views) + 1, dtype=np.int64)
    np.cumsum(counts, out=cam_offs_h[1:])
    pts = torch.from_numpy(np.ascontiguousarray(np.concatenate(views, axis=0))).to(dev)
    cam_offs = torch.from_numpy(cam_offs_h).to(dev)
    Fd = torch.from_numpy(np.ascontiguousarray(np.stack([_F(f) for f in Fs]))).to(dev)
    plan = ops.PairwisePlan(cam_offs_h, 1, len(views), pairs, device=dev)
    e = ops.pairwise_residual_f64(pts, cam_offs, Fd, plan).cpu().numpy()
    return [e[p, :counts[a], :counts[b]] for p, (a, b) in enumerate(pairs)]


def epipolar_error(pt1, pt2, F, img1=None, img2=None):
    """Symmetric point-to-epipolar-line distance (epipolar_matching.py:5-28).

    ``0.5 * (|l1 . p1| + |l2 . p2|)`` with ``l2 = F p1``, ``l1 = F^T p2``
    normalised by the norm of their first two components, or the 9999
    sentinel for a line whose norm is not > 1e-8.  Returns ``np.float64``.
    """
    p1 = np.asarray([[pt1[0], pt1[1]]], dtype=np.float64)
    p2 = np.asarray([[pt2[0], pt2[1]]], dtype=np.float64)
    return np.float64(_pairs_f64([p1, p2], [F], [(0, 1)])[0][0, 0])


def epipolar_error_full(pt1, pt2, pt3, F12, F13, F23):
    """Three-camera error ``(e12 + e13 + e23) / 3`` (epipolar_matching.py:73-81).

    The three fp64 residuals come from one GPU launch; like the reference the
    result is the float64 value (the float32 cast happens only in the cube).
    """
    pts = [np.asarray([[p[0], p[1]]], dtype=np.float64) for p in (pt1, pt2, pt3)]
    e12, e13, e23 = (m[0, 0] for m in _pairs_f64(pts, (F12, F13, F23), [(0, 1), (0, 2), (1, 2)]))
    return (np.float64(e12) + np.float64(e13) + np.float64(e23)) / 3


def compute_cost_matrices(views: Sequence[Tuple[np.ndarray, np.ndarray, np.ndarray]],
                          Fs: Sequence[Tuple[np.ndarray, np.ndarray, np.ndarray]]):
    """Batched compute_cost_matrix over several captures in ONE launch pair.

    ``views[s] = (p1, p2, p3)`` float64 centroid arrays, ``Fs[s] = (F12, F13,
    F23)``.  Returns (list of float32 cubes, list of per-(i,j) argmin arrays).
    """
    dev = _device()
    S = len(views)
    counts = np.array([[len(v) for v in vs] for vs in views], dtype=np.int64).reshape(S, 3)
    cam_offs_h = np.zeros(S * 3 + 1, np.int64)
    np.cumsum(counts.reshape(-1), out=cam_offs_h[1:])
    pts_h = np.concatenate([np.asarray(v, np.float64).reshape(-1, 2) for vs in views for v in vs]
                           + [np.zeros((0, 2))], axis=0)
    F_h = np.stack([_F(f) for fs in Fs for f in fs]) if S else np.zeros((0, 9))
    plan = ops.TripletPlan(cam_offs_h, S, device=dev)
    pts = torch.from_numpy(np.ascontiguousarray(pts_h)).to(dev)
    cam_offs = torch.from_numpy(cam_offs_h).to(dev)
    F = torch.from_numpy(np.ascontiguousarray(F_h)).to(dev)
    cube, argmin, _ = ops.triplet_cost_argmin(pts, cam_offs, F, plan)
    cube_h = cube.cpu().numpy()
    argmin_h = argmin.cpu().numpy()
    cubes, argmins = [], []
    for s in range(S):
        N, M, P = (int(c) for c in counts[s])
        cubes.append(cube_h[plan.cube_offs_host[s]:plan.cube_offs_host[s + 1]].reshape(N, M, P).copy())
        argmins.append(argmin_h[plan.row_offs_host[s]:plan.row_offs_host[s + 1]].copy())
    return cubes, argmins


def compute_cost_matrix(dets1, dets2, dets3, F12, F13, F23, img1=None, img2=None, img3=None):
    """N x M x P float32 cost cube from bounding-box centres (epipolar_matching.py:83-98).

    ``cost[i, j, k] = float32(epipolar_error_full(c1[i], c2[j], c3[k], F12, F13, F23))``
    computed in one GPU launch pair (fp64 pair matrices, then the cube).
    Returns a freshly allocated C-order ``np.ndarray`` owned by the caller.
    """
    views = (_centroids(dets1), _centroids(dets2), _centroids(dets3))
    N, M, P = (len(v) for v in views)
    if N == 0 or M == 0 or P == 0:
        return np.zeros((N, M, P), dtype=np.float32)     # the reference loop never runs
    # one staged copy in, one launch, one copy out (capture_session)
    return cube_slot(N, M, P, _device()).run(views, (F12, F13, F23))


_LSAP_ERRORS = {1: "matrix contains invalid numeric entries", 2: "cost matrix is infeasible",
                3: "assignment workgroups failed to synchronise (internal error)"}


def linear_sum_assignment(cost_matrix):
    """GPU ``scipy.optimize.linear_sum_assignment`` for one matrix -> (row_ind, col_ind).

    scipy converts any input to float64 before assigning; a float32 matrix
    converts exactly, so it is assigned in its own type (half the bytes),
    every other dtype is converted to float64 as scipy does and assigned in
    float64 (``mvm_lsap_solve_ex`` with MVM_F64)."""
    dev = _device()
    arr = np.asarray(cost_matrix)
    dt = np.float32 if arr.dtype == np.float32 else np.float64
    cost = np.ascontiguousarray(arr, dtype=dt)
    if cost.ndim != 2:
        raise ValueError("expected a matrix")
    tdt = torch.float32 if dt == np.float32 else torch.float64
    if cost.size == 0:                  # scipy: empty assignment
        return np.zeros(0, np.int64), np.zeros(0, np.int64)
    # one staged copy in, one launch, one copy out (capture_session)
    r, c, status = lsap_slot(cost.shape[0], cost.shape[1], tdt, dev).run(cost)
    if status:
        raise ValueError(_LSAP_ERRORS.get(status, f"assignment failed ({status})"))
    return r, c


def match_objects(cost_matrix, threshold) -> List[Tuple[int, int, int]]:
    """Flatten -> Hungarian -> keep matches < threshold (epipolar_matching.py:100-116).

    The assignment runs on the GPU and equals scipy ``linear_sum_assignment``
    on the ``(N*M, P)`` flattening, in the precision scipy uses for the
    cube's dtype; strict ``<`` threshold on the cube's own values;
    ``i = r // M``, ``j = r % M``.
    """
    N, M, P = cost_matrix.shape
    flat = cost_matrix.reshape(N * M, P)
    rows, cols = linear_sum_assignment(flat)
    out = []
    for r, c in zip(rows, cols):
        if flat[r, c] < threshold:
            out.append((np.int64(r) // M, np.int64(r) % M, np.int64(c)))
    return out


def triangulate_multi_view(proj_mats, points_2D) -> np.ndarray:
    """Direct Linear Transform triangulation (epipolar_matching.py:118-127)."""
    rows = []
    for P, (x, y) in zip(proj_mats, points_2D):
        rows.append(x * P[2] - P[0])
        rows.append(y * P[2] - P[1])
    _, _, Vt = np.linalg.svd(np.array(rows))
    X = Vt[-1]
    return X[:3] / X[3]
