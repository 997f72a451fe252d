"""Assignment (match_objects, epipolar_matching.py:100-116): the restated scipy
LSAP solver (oracle/lsap.py) vs scipy itself and vs the reference's golden
match lists; CPU."""
import numpy as np
import pytest
from scipy.optimize import linear_sum_assignment as scipy_lsa

from oracle import lsap


@pytest.mark.parametrize("shape", [(1, 1), (3, 5), (5, 3), (7, 7), (40, 9), (9, 40), (64, 16)])
def test_restated_lsap_equals_scipy_random(shape):
    rng = np.random.default_rng(sum(shape))
    for trial in range(20):
        c = rng.normal(size=shape).astype(np.float32)
        if trial % 4 == 1:
            c = np.round(c * 2) / 2           # many exact ties
        if trial % 4 == 2:
            c[:, : shape[1] // 2] = c[:, :1]  # duplicated columns
        if trial % 4 == 3:
            c = np.zeros(shape, np.float32)   # all ties
        r0, c0 = scipy_lsa(c)
        r1, c1 = lsap.linear_sum_assignment(c)
        assert np.array_equal(r0, r1) and np.array_equal(c0, c1), trial


def test_restated_lsap_on_golden_cubes(golden):
    g = golden("a3_cost_cubes.npz")
    for n in g["names"]:
        cube = g[f"{n}_cube"]
        assert np.array_equal(np.asarray(lsap.match_objects(cube, 30)).reshape(-1, 3),
                              g[f"{n}_match30"]), n
        assert np.array_equal(np.asarray(lsap.match_objects(cube, np.inf)).reshape(-1, 3),
                              g[f"{n}_matchinf"]), n


def test_restated_lsap_errors():
    with pytest.raises(lsap.LsapError):
        lsap.linear_sum_assignment(np.array([[np.nan, 1.0]]))
    with pytest.raises(lsap.LsapError):
        lsap.linear_sum_assignment(np.array([[np.inf, np.inf], [1.0, 2.0]]))
    r, c = lsap.linear_sum_assignment(np.zeros((0, 3)))
    assert r.size == 0 and c.size == 0
