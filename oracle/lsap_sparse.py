"""Model of the GPU's candidate-list assignment solver (``lsap_sparse_kernel``).

TEST INFRASTRUCTURE ONLY: a plain-Python statement of the decomposition the
HIP kernels in ``bpc_baseline_amd/csrc/mvm_lsap_sparse.hip`` implement, run
against ``oracle/lsap.py`` (scipy's solver restated, pinned to scipy) on
random, tie-heavy and cube-shaped problems by ``tests/test_lsap_sparse_model.py``.
Nothing in the product path imports it.

Why it is exact.  scipy's solver (Crouse's shortest augmenting path,
``oracle/lsap.py``) on a wide problem (S short-side rows, L >> S columns)
scans every remaining column at every Dijkstra step.  But a column that no
search has assigned yet ("free") has ``v[j] == 0`` (duals change only for the
columns a search visits, and every visited column is assigned or becomes the
sink), it is never removed from the scan before the search ends, and its
``r = ((minVal + C[i,j]) - u[i]) - 0`` is a monotone (non-strict) function of
``C[i,j]`` alone.  So within a search:

* the free columns' smallest shortest-path cost is ``F = min_s f_s`` over the
  rows visited so far, ``f_s`` = r of row s's smallest free entry;
* the free columns that reach a value ``lowest`` are, per visited row s with
  ``f_s == lowest``, the free entries of row s whose r equals it;
* the at most S assigned columns are scanned explicitly ("slots").

Each row keeps a candidate list: every column with ``C <= theta_s``, where
``theta_s`` is the TB-th smallest of the minima of 64 groups of the row's
block minima (blocks of B columns, group l = blocks l, l+64, ...: one wave
lane each), so the list holds at least TB entries and every column outside it
has ``C >= beta_s = nextafter(theta_s, inf)``.  Its smallest free entry is the
row's free minimum whenever the list holds a free entry; the list holds every
free tie at ``lowest`` whenever ``r(beta_s) > lowest``.  Otherwise (or when
the list would exceed LCAP entries) the row is scanned densely -- the
fallback keeps the result exact for any input, ties and duplicates included.

The decision rule is scipy's: among the columns whose shortest-path cost is
the step's minimum, the free one latest in scan order if any is free, else
the first in scan order.  Scan order is the reversed column order shrunk by
swap-with-last removals; only the removed (assigned) columns and the columns
moved into their places leave their default position ``L-1-j``.
"""
from __future__ import annotations

import math

import numpy as np

from .lsap import LsapError

__all__ = ["linear_sum_assignment", "candidate_lists", "DEFAULTS"]

DEFAULTS = dict(B=32, TB=16, LCAP=128)


def _key16_upper(x: np.ndarray) -> np.ndarray:
    """The largest float32 >= 0 whose key shares the upper 16 bits with x's
    (x >= +0 or +inf): what the kernel takes for a block minimum it knows from
    the cube's 16-bit keys (sp_b8_upper, capped at +inf)."""
    k = (x.astype(np.float32).view(np.uint32) | np.uint32(0x80000000)) >> np.uint32(16)
    up = np.minimum((k << np.uint32(16)) | np.uint32(0xFFFF), np.uint32(0xFF800000))
    return (up & np.uint32(0x7FFFFFFF)).view(np.float32)


def candidate_lists(W: np.ndarray, B: int, TB: int, LCAP: int, key16: bool = False):
    """Per wide row s: (cols int64 | None, beta float64 | None).

    cols = every column with W[s, j] <= theta_s (None: more than LCAP of
    them, the row is scanned densely); beta = the smallest value an unlisted
    column can hold (None: no column is unlisted).  key16: theta from the
    block minima's 16-bit key upper bounds (the kernel's input from the
    cube's 8-row minima; float32 costs >= 0): a theta some TB blocks still
    reach, a little above the exact rule's."""
    S, L = W.shape
    nb = -(-L // B)
    pad = np.full((S, nb * B), np.inf, W.dtype)
    pad[:, :L] = W
    bm = pad.reshape(S, nb, B).min(axis=2)
    if key16:
        bm = _key16_upper(bm)
    out = []
    for s in range(S):
        # the kernel's rule: lane l of a wave holds blocks l, l + 64, ...;
        # theta is the TB-th smallest of the 64 lanes' minima
        lanes = np.full(64, np.inf, W.dtype)
        for l in range(min(64, nb)):
            lanes[l] = bm[s, l::64].min()
        theta = np.sort(lanes)[TB - 1] if nb > TB else W.dtype.type(np.inf)
        cols = np.nonzero(W[s] <= theta)[0]      # the candidate blocks' columns <= theta
        beta = None
        if not np.isinf(theta):
            beta = float(np.nextafter(W.dtype.type(theta), W.dtype.type(np.inf)))
        out.append((None if cols.size > LCAP else cols, beta))
    return out


def linear_sum_assignment(cost: np.ndarray, B: int = 32, TB: int = 16, LCAP: int = 128,
                          stats: dict | None = None, key16: bool = False):
    """-> (row_ind, col_ind) exactly as scipy.optimize.linear_sum_assignment."""
    cost = np.asarray(cost)
    if cost.ndim != 2:
        raise LsapError("expected a matrix")
    nr, nc = cost.shape
    if nr == 0 or nc == 0:
        return np.zeros(0, np.int64), np.zeros(0, np.int64)
    transpose = nc < nr
    W = cost.T if transpose else cost
    S, L = W.shape
    if np.any(np.isnan(W)) or np.any(W == -np.inf):
        raise LsapError("matrix contains invalid numeric entries")
    lists = candidate_lists(W, B, TB, LCAP, key16)
    st = stats if stats is not None else {}
    for key in ("steps", "dense_min", "dense_ties", "dense_rows", "searches"):
        st.setdefault(key, 0)
    st["dense_rows"] += sum(1 for c, _ in lists if c is None)

    u = np.zeros(S)
    c4r = np.full(S, -1, np.int64)          # row -> slot
    slot_col, slot_v, slot_r4c = [], [], []  # slot = assigned column, in assignment order
    assigned = np.zeros(L, bool)

    def rfree(m, c, ui):
        return ((m + float(c)) - ui) - 0.0

    def free_min(i, m, ui):
        """(f, rb): smallest r over row i's free columns, and r at beta."""
        cols, beta = lists[i]
        if cols is not None:
            fc = cols[~assigned[cols]]
            if fc.size:
                f = min(rfree(m, W[i, j], ui) for j in fc)
                rb = rfree(m, beta, ui) if beta is not None else math.inf
                return f, rb
        st["dense_min"] += 1
        fc = np.nonzero(~assigned)[0]
        f = min((rfree(m, W[i, j], ui) for j in fc), default=math.inf)
        return f, None                       # None: ties need the dense scan too

    for cur in range(S):
        st["searches"] += 1
        na = len(slot_col)
        spc = [math.inf] * na
        sps = [-1] * na                      # path step of each slot
        spos = [L - 1 - slot_col[q] for q in range(na)]
        removed = [False] * na
        moved = {}                           # free column -> position
        n_rem = L
        rows, mins, fs, rbs, ms_prev = [], [], [], [], []
        chosen_slot, chosen_ps = [], []
        i, m_prev, F = cur, 0.0, math.inf
        while True:
            st["steps"] += 1
            k = len(rows)
            ui = u[i]
            rows.append(i)
            ms_prev.append(m_prev)
            for q in range(na):
                if removed[q]:
                    continue
                r = ((m_prev + float(W[i, slot_col[q]])) - ui) - slot_v[q]
                if r < spc[q]:
                    spc[q] = r
                    sps[q] = k
            a_min, a_pos, a_q = math.inf, None, None
            for q in range(na):
                if removed[q]:
                    continue
                if spc[q] < a_min or (spc[q] == a_min and a_pos is not None and spos[q] < a_pos):
                    a_min, a_pos, a_q = spc[q], spos[q], q
            f, rb = free_min(i, m_prev, ui)
            fs.append(f)
            rbs.append(rb)
            F = min(F, f)
            lowest = min(a_min, F)
            if lowest == math.inf:
                raise LsapError("cost matrix is infeasible")
            if F == lowest:                  # a free column reaches the minimum: the sink
                best_pos, best_j, best_s = -1, -1, -1
                for s in range(k + 1):
                    if fs[s] != lowest:
                        continue
                    cols, _ = lists[rows[s]]
                    if cols is None or rbs[s] is None or rbs[s] == lowest:
                        st["dense_ties"] += 1
                        cols = np.nonzero(~assigned)[0]
                    for j in cols:
                        if assigned[j] or rfree(ms_prev[s], W[rows[s], j], u[rows[s]]) != lowest:
                            continue
                        p = moved.get(int(j), L - 1 - int(j))
                        if p > best_pos:             # first row reaching it = its path
                            best_pos, best_j, best_s = p, int(j), s
                mins.append(lowest)
                chosen_slot.append(-1)
                chosen_ps.append(best_s)
                sink = best_j
                break
            q = a_q
            mins.append(lowest)
            chosen_slot.append(q)
            chosen_ps.append(sps[q])
            x, last = a_pos, n_rem - 1
            if x != last:                    # swap-with-last: the column at `last` moves to x
                hit = [p for p in range(na) if not removed[p] and spos[p] == last]
                if hit:
                    spos[hit[0]] = x
                else:
                    fm = [c for c, p in moved.items() if p == last]
                    moved[fm[0] if fm else L - 1 - last] = x
            removed[q] = True
            n_rem -= 1
            i, m_prev = slot_r4c[q], lowest
        # duals: u[cur] += minVal; u[i_t] += minVal - m_(t-1); v[q] -= minVal - spc[q]
        k = len(rows) - 1
        u[cur] += lowest
        for t in range(1, k + 1):
            u[rows[t]] += lowest - mins[t - 1]
        for q in range(na):
            if removed[q]:
                slot_v[q] -= lowest - spc[q]
        ns = len(slot_col)
        slot_col.append(sink)
        slot_v.append(0.0)
        slot_r4c.append(-1)
        assigned[sink] = True
        chosen_slot[k] = ns
        kk = k                               # augment along the path steps
        while True:
            s = chosen_ps[kk]
            i2, qq = rows[s], chosen_slot[kk]
            c4r[i2] = qq
            slot_r4c[qq] = i2
            if s == 0:
                break
            kk = s - 1
    col4row = np.array([slot_col[q] for q in c4r], np.int64)
    if transpose:
        order = np.argsort(col4row, kind="stable")
        return col4row[order].astype(np.int64), order.astype(np.int64)
    return np.arange(S, dtype=np.int64), col4row
