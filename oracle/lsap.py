"""Restatement of scipy's rectangular linear-sum-assignment solver.

TEST INFRASTRUCTURE ONLY (checker for the GPU LSAP kernel).

The reference's association step is ``scipy.optimize.linear_sum_assignment``
(bpc/inference/epipolar_matching.py:107; scipy pinned to 1.14.0 in
docker/requirements.txt:3, a third-party dependency absent from
/root/reference).  scipy implements the shortest-augmenting-path algorithm of
D.F. Crouse, "On implementing 2D rectangular assignment algorithms", IEEE TAES
52(4), 2016: a tall matrix is transposed; one augmenting path per (short-side)
row, each found by a Dijkstra-like scan over the remaining columns kept in an
array initialised in REVERSE column order and shrunk by swap-with-last
removal; among equal shortest-path costs the scan keeps the first minimum
unless a later equal column is unassigned (then the last such one); dual
variables u, v are updated after each path; for a transposed problem the
assignment is returned sorted by original row.

This restatement reproduces those choices (including the tie rule that
matters for duplicated detections) and is pinned against scipy itself and
against the reference's golden match lists in tests/test_lsap.py.
"""
from __future__ import annotations

import numpy as np


class LsapError(ValueError):
    pass


def linear_sum_assignment(cost: np.ndarray):
    """-> (row_ind int64, col_ind int64) exactly as scipy.optimize.linear_sum_assignment."""
    cost = np.asarray(cost)
    if cost.ndim != 2:
        raise LsapError("expected a matrix")
    nr, nc = cost.shape
    if nr == 0 or nc == 0:
        return np.zeros(0, np.int64), np.zeros(0, np.int64)
    transpose = nc < nr
    C = (cost.T if transpose else cost).astype(np.float64)
    if transpose:
        nr, nc = nc, nr
    if np.any(np.isnan(C)) or np.any(C == -np.inf):
        raise LsapError("matrix contains invalid numeric entries")
    u = np.zeros(nr)
    v = np.zeros(nc)
    path = np.full(nc, -1, np.int64)
    col4row = np.full(nr, -1, np.int64)
    row4col = np.full(nc, -1, np.int64)
    for cur in range(nr):
        min_val = 0.0
        remaining = np.arange(nc - 1, -1, -1)
        nrem = nc
        SR = np.zeros(nr, bool)
        SC = np.zeros(nc, bool)
        spc = np.full(nc, np.inf)
        i, sink = cur, -1
        while sink == -1:
            SR[i] = True
            js = remaining[:nrem]
            r = ((min_val + C[i, js]) - u[i]) - v[js]
            upd = r < spc[js]
            path[js[upd]] = i
            spc[js[upd]] = r[upd]
            vals = spc[js]
            lowest = vals.min()
            if lowest == np.inf:
                raise LsapError("cost matrix is infeasible")
            eq = np.nonzero(vals == lowest)[0]
            free = eq[row4col[js[eq]] == -1]
            index = free[-1] if free.size else eq[0]
            min_val = lowest
            j = remaining[index]
            if row4col[j] == -1:
                sink = j
            else:
                i = row4col[j]
            SC[j] = True
            nrem -= 1
            remaining[index] = remaining[nrem]
        u[cur] += min_val
        rows = np.nonzero(SR)[0]
        rows = rows[rows != cur]
        u[rows] += min_val - spc[col4row[rows]]
        cols = np.nonzero(SC)[0]
        v[cols] -= min_val - spc[cols]
        j = sink
        while True:
            i = path[j]
            row4col[j] = i
            col4row[i], j = j, col4row[i]
            if i == cur:
                break
    if transpose:
        order = np.argsort(col4row, kind="stable")
        return col4row[order].astype(np.int64), order.astype(np.int64)
    return np.arange(nr, dtype=np.int64), col4row.astype(np.int64)


def match_objects(cost_matrix: np.ndarray, threshold):
    """epipolar_matching.py:100-116 on top of the restated solver."""
    N, M, P = cost_matrix.shape
    flat = cost_matrix.reshape(N * M, P)
    rows, cols = linear_sum_assignment(flat)
    return [(int(r) // M, int(r) % M, int(c)) for r, c in zip(rows, cols) if flat[r, c] < threshold]
