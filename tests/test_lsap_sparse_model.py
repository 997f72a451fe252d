"""The candidate-list decomposition of the assignment (oracle/lsap_sparse.py,
the model the HIP kernels of mvm_lsap_sparse.hip implement) gives scipy's
answer: against the scipy restatement (oracle/lsap.py, itself pinned to scipy)
on random, tie-heavy, infeasible and invalid problems with list parameters
small enough that every fallback (dense rows, exhausted lists, ties at the
list bound, columns moved by swap-with-last) runs, and against scipy on real
flattened cubes with the kernels' own parameters (no dense row there)."""
import numpy as np
import pytest

from oracle import lsap as L
from oracle import lsap_sparse as SP


def _solve(fn, C, **kw):
    try:
        return fn(C, **kw)
    except L.LsapError as e:
        return str(e)


def _same(a, b):
    if isinstance(a, str) or isinstance(b, str):
        return a == b
    return np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])


def test_model_equals_restatement_random():
    rng = np.random.default_rng(0)
    stats = {}
    for it in range(1200):
        kind = it % 6
        nr, nc = int(rng.integers(1, 12)), int(rng.integers(1, 120))
        if rng.random() < 0.5:
            nr, nc = nc, nr
        if kind == 0:
            C = rng.random((nr, nc)).astype(np.float32)
        elif kind == 1:
            C = rng.integers(0, 3, (nr, nc)).astype(np.float32)      # heavy ties
        elif kind == 2:
            C = np.zeros((nr, nc), np.float32)
        elif kind == 3:
            C = rng.integers(0, 5, (nr, nc)).astype(np.float32)
            C[rng.random((nr, nc)) < 0.3] = np.inf                  # forbidden / infeasible
        elif kind == 4:
            C = (rng.random((nr, nc)) * 4).astype(np.float32)
            C[:, ::3] = C[:, :1]                                    # duplicated columns
        else:
            C = rng.normal(size=(nr, nc))                            # float64
        if it % 97 == 5:
            C = C.astype(np.float64)
            C[0, 0] = np.nan if it % 2 else -np.inf                 # invalid entries
        kw = dict(B=int(rng.choice([1, 2, 4, 32])), TB=int(rng.choice([1, 2, 3, 16])),
                  LCAP=int(rng.choice([1, 4, 8, 128])), stats=stats)
        assert _same(_solve(SP.linear_sum_assignment, C, **kw), _solve(L.linear_sum_assignment, C)), \
            (it, C.shape, kw)
    # every fallback of the model ran
    assert stats["dense_min"] > 0 and stats["dense_ties"] > 0 and stats["dense_rows"] > 0


@pytest.mark.parametrize("key16", [False, True])
@pytest.mark.parametrize("n", [48, 64, 100])
def test_model_on_cubes_equals_scipy(n, key16):
    scipy = pytest.importorskip("scipy.optimize")
    from bpc_baseline_amd.synth import make_scenes
    from oracle import oracle as O
    b = make_scenes(2, 3, n, seed=9)
    cube = O.cube(b.pts, b.cam_offs, b.F, 2)[0]
    for s in range(2):
        flat = cube[s * n ** 3:(s + 1) * n ** 3].reshape(n * n, n)
        stats = {}
        got = SP.linear_sum_assignment(flat, **SP.DEFAULTS, stats=stats, key16=key16)
        ref = scipy.linear_sum_assignment(flat)
        assert _same(got, ref)
        if n >= 64:     # the lists carry the whole search: no row scanned densely
            assert stats["dense_min"] == 0 and stats["dense_ties"] == 0, stats


def test_key16_upper_bounds():
    """theta from 16-bit keys: an upper bound of each value within 1/128, +inf kept"""
    x = np.array([0.0, 1e-30, 0.37, 1.0, 5e3, 3.4e38, np.inf], np.float32)
    up = SP._key16_upper(x)
    assert (up >= x).all() and np.isinf(up[-1])
    assert (up[1:-1] <= x[1:-1] * (1 + 2.0 ** -7)).all()
