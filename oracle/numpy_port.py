"""Vectorised NumPy restatement of the pairwise residuals (SURVEY §8d's
"vectorised NumPy restatement" CPU baseline).

TEST / BENCH INFRASTRUCTURE ONLY: bench.py times it on a small sample beside
the C/OpenMP oracle.  It follows epipolar_error (bpc/inference/
epipolar_matching.py:5-28) with whole-view arrays instead of per-pair calls.
NumPy has no fused multiply-add, so its fp64 residuals can differ from the
reference's OpenBLAS evaluation in the last bit (34% of fp64
values, 0 of 20,000 float32 casts).  It is therefore a timing baseline; parity
is the C oracle's job (tests/test_oracle_golden.py), and
tests/test_host_logic.py checks that its float32 output agrees.
"""
from __future__ import annotations

import numpy as np


def _lines(F: np.ndarray, x: np.ndarray, y: np.ndarray, transpose: bool):
    """l = F @ (x, y, 1) (or F.T @ ...) normalised by its first two components
    (:13-23) -> (l0, l1, l2, degenerate mask)."""
    M = F.T if transpose else F
    l0 = M[0, 0] * x + M[0, 1] * y + M[0, 2]
    l1 = M[1, 0] * x + M[1, 1] * y + M[1, 2]
    l2 = M[2, 0] * x + M[2, 1] * y + M[2, 2]
    n = np.sqrt(l0 * l0 + l1 * l1)
    deg = ~(n > 1e-8)
    safe = np.where(deg, 1.0, n)
    return l0 / safe, l1 / safe, l2 / safe, deg


def pair_matrix(pa: np.ndarray, pb: np.ndarray, F: np.ndarray) -> np.ndarray:
    """float32 [na, nb] of 0.5 * (|l1 . p1| + |l2 . p2|) for every (i, j)."""
    xa, ya = pa[:, 0], pa[:, 1]
    xb, yb = pb[:, 0], pb[:, 1]
    r0, r1, r2, rdeg = _lines(F, xa, ya, transpose=False)    # l2 = F p1, rows
    c0, c1, c2, cdeg = _lines(F, xb, yb, transpose=True)     # l1 = F^T p2, columns
    d1 = np.abs(c0[None, :] * xa[:, None] + c1[None, :] * ya[:, None] + c2[None, :])
    d2 = np.abs(r0[:, None] * xb[None, :] + r1[:, None] * yb[None, :] + r2[:, None])
    d1 = np.where(cdeg[None, :], 9999.0, d1)
    d2 = np.where(rdeg[:, None], 9999.0, d2)
    return (0.5 * (d1 + d2)).astype(np.float32)


def pairwise(pts, cam_offs, F, pairs, n_scenes: int, n_cams: int):
    """Every (scene, pair) matrix, flattened as the GPU op lays them out, plus
    the per-row argmin (np.argmin: first minimum)."""
    out, arg = [], []
    P = len(pairs)
    for s in range(n_scenes):
        for p, (a, b) in enumerate(pairs):
            oa, ea = cam_offs[s * n_cams + a], cam_offs[s * n_cams + a + 1]
            ob, eb = cam_offs[s * n_cams + b], cam_offs[s * n_cams + b + 1]
            m = pair_matrix(pts[oa:ea], pts[ob:eb], np.asarray(F[s * P + p]).reshape(3, 3))
            out.append(m.reshape(-1))
            if m.shape[1]:
                arg.append(np.argmin(m, axis=1).astype(np.int32))
            else:
                arg.append(np.full(m.shape[0], -1, np.int32))
    return (np.concatenate(out) if out else np.zeros(0, np.float32),
            np.concatenate(arg) if arg else np.zeros(0, np.int32))
