"""GPU assignment (mvm_lsap_solve) == scipy.optimize.linear_sum_assignment:
random shapes with heavy ties, the reference's golden match lists, ragged
batches in one launch, error statuses, and a full 256^3 cube."""
import numpy as np
import pytest
import torch
from scipy.optimize import linear_sum_assignment as scipy_lsa

pytestmark = pytest.mark.gpu


def _batched(cuda, mats):
    from bpc_baseline_amd import ops
    plan = ops.LsapPlan([m.shape[0] for m in mats], [m.shape[1] for m in mats], device=cuda)
    flat = np.concatenate([m.astype(np.float32).reshape(-1) for m in mats] + [np.zeros(1, np.float32)])
    offs = np.zeros(len(mats), np.int64)
    np.cumsum([m.size for m in mats[:-1]], out=offs[1:]) if len(mats) > 1 else None
    r, c, st = ops.linear_sum_assignment_batched(torch.from_numpy(flat).to(cuda),
                                                 torch.from_numpy(offs).to(cuda), plan)
    r, c, st = r.cpu().numpy(), c.cpu().numpy(), st.cpu().numpy()
    o = plan.out_offs_host
    return [(r[o[k]:o[k + 1]], c[o[k]:o[k + 1]], int(st[k])) for k in range(len(mats))]


@pytest.fixture(params=["default", "lds", "workgroup", "workgroup256", "multi"])
def lsap_path(request, monkeypatch):
    """default: long sides <= 1024 one problem per wave, up to 4096 one
    workgroup with the column state in LDS, larger ones split over co-resident
    workgroups when the batch leaves room; lds: every problem of <= 4096 in
    the LDS-state workgroup; workgroup: one 1024-thread workgroup per problem
    with the state in the workspace; multi: every problem split over 4
    workgroups."""
    if request.param == "lds":
        monkeypatch.setenv("MVM_LSAP_WAVE_MAX_COLS", "0")
        monkeypatch.setenv("MVM_LSAP_MULTI_G", "0")
    elif request.param == "workgroup":
        monkeypatch.setenv("MVM_LSAP_WAVE_MAX_COLS", "0")
        monkeypatch.setenv("MVM_LSAP_MULTI_G", "0")
        monkeypatch.setenv("MVM_LSAP_LDS_MAX_COLS", "0")
    elif request.param == "workgroup256":
        monkeypatch.setenv("MVM_LSAP_WAVE_MAX_COLS", "0")
        monkeypatch.setenv("MVM_LSAP_MULTI_G", "0")
        monkeypatch.setenv("MVM_LSAP_LDS_MAX_COLS", "0")
        monkeypatch.setenv("MVM_LSAP_MID_MAX_COLS", "1000000")
    elif request.param == "multi":
        monkeypatch.setenv("MVM_LSAP_WAVE_MAX_COLS", "0")
        monkeypatch.setenv("MVM_LSAP_MULTI_G", "4")
    return request.param


def test_random_shapes_and_ties_batched(cuda, lsap_path):
    rng = np.random.default_rng(0)
    mats = []
    for shape in [(1, 1), (3, 5), (5, 3), (7, 7), (40, 9), (9, 40), (64, 16), (300, 20), (0, 4), (4, 0),
                  (65, 2), (129, 7), (257, 30), (600, 24), (24, 600), (1024, 3), (1100, 5), (70, 70),
                  (4096, 6), (6, 4096), (2500, 11), (4097, 3)]:
        for trial in range(4):
            c = rng.normal(size=shape).astype(np.float32)
            if trial == 1:
                c = np.round(c * 2) / 2
            if trial == 2 and shape[1] > 1:
                c[:, : shape[1] // 2] = c[:, :1]
            if trial == 3:
                c = np.zeros(shape, np.float32)
            mats.append(c)
    for m, (r, c, st) in zip(mats, _batched(cuda, mats)):
        r0, c0 = scipy_lsa(m)
        assert st == 0
        assert np.array_equal(r, r0) and np.array_equal(c, c0), m.shape


def test_golden_match_lists(cuda, golden, lsap_path):
    from bpc_baseline_amd.inference.epipolar_matching import match_objects
    g = golden("a3_cost_cubes.npz")
    for n in g["names"]:
        cube = g[f"{n}_cube"]
        for thr, key in ((30, "match30"), (np.inf, "matchinf")):
            got = np.asarray(match_objects(cube, thr), np.int64).reshape(-1, 3)
            assert np.array_equal(got, g[f"{n}_{key}"]), (n, thr)


def test_error_statuses(cuda, lsap_path):
    from bpc_baseline_amd.inference.epipolar_matching import linear_sum_assignment
    with pytest.raises(ValueError, match="invalid numeric"):
        linear_sum_assignment(np.array([[np.nan, 1.0], [0.0, 2.0]]))
    with pytest.raises(ValueError, match="invalid numeric"):
        linear_sum_assignment(np.array([[-np.inf, 1.0]]))
    with pytest.raises(ValueError, match="infeasible"):
        linear_sum_assignment(np.array([[np.inf, np.inf], [1.0, 2.0]]))
    r, c = linear_sum_assignment(np.array([[np.inf, 1.0], [1.0, np.inf]]))
    assert list(c) == [1, 0]


@pytest.mark.parametrize("multi_g", ["-1", "0", "16"])
def test_full_256_cube_equals_scipy(cuda, monkeypatch, multi_g):
    """Config-2 scale: the (65536 x 256) flattened 256^3 cube of one scene."""
    from bpc_baseline_amd.synth import make_scenes
    from bpc_baseline_amd.inference.epipolar_matching import linear_sum_assignment
    from oracle import oracle as O
    monkeypatch.setenv("MVM_LSAP_MULTI_G", multi_g)
    b = make_scenes(1, 3, 256, seed=42)
    cube, _, _, _, _ = O.cube(b.pts, b.cam_offs, b.F, 1)
    flat = cube.reshape(256 * 256, 256)
    r0, c0 = scipy_lsa(flat)
    r1, c1 = linear_sum_assignment(flat)
    assert np.array_equal(r0, r1) and np.array_equal(c0, c1)


@pytest.mark.parametrize("shapes", [
    [(0, 4), (3, 0), (100, 3), (3, 100)],        # no problem in the first wave class, empties
    [(0, 0), (4, 0)],                             # all empty
    [(5, 7), (0, 2), (64, 2)],                    # small only
    [(0, 3), (2000, 5), (1100, 40)],              # workgroup classes + empties
])
def test_bounded_launch_sets_every_status(cuda, shapes, lsap_path):
    """The plan's long-side bounds skip kernel classes without work; every
    problem (empty ones included) still gets its status and assignment."""
    rng = np.random.default_rng(3)
    mats = [rng.normal(size=s).astype(np.float32) for s in shapes]
    for m, (r, c, st) in zip(mats, _batched(cuda, mats)):
        assert st == 0
        if m.size:
            r0, c0 = scipy_lsa(m)
            assert np.array_equal(r, r0) and np.array_equal(c, c0)
        else:
            assert r.size == 0 and c.size == 0
