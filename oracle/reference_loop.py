"""The reference's own CPU cost model, restated: one small-array NumPy
evaluation per detection pair / triple, in Python loops.

TEST / BENCH INFRASTRUCTURE ONLY.  The reference's Python cannot travel to the
GPU box, so bench.py times this restatement there as the "reference loop" CPU
figure beside the GPU number.  It performs the same NumPy calls per pair as
epipolar_error (bpc/inference/epipolar_matching.py:10-28: two homogeneous
3-vectors, F @ p and F.T @ p, the norm of each line's first two components,
the 1e-8 test, two dot products, the 9999 sentinel) and the same triple loop
as compute_cost_matrix (:83-98), so its speed is the reference's; being the
same NumPy arithmetic it is also bit-identical to the golden vectors
(tests/test_host_logic.py).
"""
from __future__ import annotations

import numpy as np


def residual(p1, p2, F) -> float:
    """Symmetric point-to-epipolar-line distance of one pair (the a1 formula)."""
    h1 = np.array([p1[0], p1[1], 1.0])
    h2 = np.array([p2[0], p2[1], 1.0])
    line_in_2 = F @ h1
    line_in_1 = F.T @ h2
    n1 = np.linalg.norm(line_in_1[:2])
    n2 = np.linalg.norm(line_in_2[:2])
    ok1, ok2 = n1 > 1e-8, n2 > 1e-8
    if ok1:
        line_in_1 /= n1
    if ok2:
        line_in_2 /= n2
    a = abs(np.dot(line_in_1, h1)) if ok1 else 9999
    b = abs(np.dot(line_in_2, h2)) if ok2 else 9999
    return 0.5 * (a + b)


def cube(c1, c2, c3, F12, F13, F23) -> np.ndarray:
    """compute_cost_matrix's triple loop over centroid lists -> float32 (N, M, P)."""
    out = np.zeros((len(c1), len(c2), len(c3)), dtype=np.float32)
    for i, p in enumerate(c1):
        for j, q in enumerate(c2):
            for k, r in enumerate(c3):
                out[i, j, k] = (residual(p, q, F12) + residual(p, r, F13) + residual(q, r, F23)) / 3
    return out


def pairs_per_second(pts_a, pts_b, F, seconds: float = 2.0) -> tuple:
    """Evaluate residual() over (i, j) pairs of two views for ~`seconds`
    -> (pairs evaluated, elapsed seconds)."""
    import time
    if len(pts_a) == 0 or len(pts_b) == 0:
        return 0, 0.0
    n = 0
    t0 = time.perf_counter()
    F = np.asarray(F, dtype=np.float64).reshape(3, 3)
    while True:
        for i in range(len(pts_a)):
            for j in range(len(pts_b)):
                residual(pts_a[i], pts_b[j], F)
            n += len(pts_b)
            if time.perf_counter() - t0 >= seconds:
                return n, time.perf_counter() - t0
