"""GPU assignment (mvm_lsap_solve) == scipy.optimize.linear_sum_assignment:
random shapes with heavy ties, the reference's golden match lists, ragged
batches in one launch, error statuses, and a full 256^3 cube."""
import numpy as np
import pytest
import torch
from scipy.optimize import linear_sum_assignment as scipy_lsa

pytestmark = pytest.mark.gpu


def _batched(cuda, mats, options=None, dtype=np.float32):
    from bpc_baseline_amd import ops
    tdt = torch.float32 if dtype == np.float32 else torch.float64
    plan = ops.LsapPlan([m.shape[0] for m in mats], [m.shape[1] for m in mats], device=cuda, dtype=tdt)
    flat = np.concatenate([m.astype(dtype).reshape(-1) for m in mats] + [np.zeros(1, dtype)])
    offs = np.zeros(len(mats), np.int64)
    np.cumsum([m.size for m in mats[:-1]], out=offs[1:]) if len(mats) > 1 else None
    r, c, st = ops.linear_sum_assignment_batched(torch.from_numpy(flat).to(cuda),
                                                 torch.from_numpy(offs).to(cuda), plan,
                                                 options=options)
    r, c, st = r.cpu().numpy(), c.cpu().numpy(), st.cpu().numpy()
    o = plan.out_offs_host
    return [(r[o[k]:o[k + 1]], c[o[k]:o[k + 1]], int(st[k])) for k in range(len(mats))]


@pytest.fixture(params=["default", "reg", "reg1024", "mreg", "lds", "workgroup", "workgroup256", "multi",
                        "nomreg", "sparse", "sparse_lo", "sparse_tb1", "sparse_tb64"])
def lsap_path(request):
    """mvm_options of each assignment kernel class.  default: long sides <=
    1024 one problem per wave, up to 4096 (short sides <= 1024) one workgroup
    with the column state in registers, larger ones split over co-resident
    workgroups when the batch leaves room, else one workgroup with the state
    in LDS or the workspace; reg / reg1024: every problem of <= 4096 in the
    register-state workgroup (512 / 1024 threads); lds: every problem of <=
    4096 in the LDS-state workgroup; workgroup: one 1024-thread workgroup per
    problem with the state in the workspace; workgroup256: the same with 256
    threads; multi: every problem split over 4 workgroups; mreg: every problem
    with a short side <= 1024 in the register-state kernel spread over
    ceil(long / 4096) workgroups (the default above 4096 columns), small
    ones included; nomreg: the default without it (long sides above 4096 in
    the split / LDS / workspace kernels); sparse: every problem with a short
    side <= 1024 and a long side <= 65536 through the candidate-list kernels
    (the default above 4096 columns: mvm_lsap_sparse.hip), small ones (whose
    rows are all scanned densely) included; sparse_lo: the same from long
    sides of 1025 on (lists and dense rows side by side); sparse_tb1 /
    sparse_tb64: one / 64 candidate blocks per row (short lists that run out,
    so rows fall back to dense scans, and long ones).  Every other path
    turns the candidate-list class off."""
    off = {"lsap_wave_max_cols": -1, "lsap_multi_g": -1, "lsap_mreg_max_cols": -1,
           "lsap_sparse_min_cols": -1}
    noreg = dict(off, lsap_reg_max_cols=-1)
    return {"default": None, "reg": off, "reg1024": dict(off, lsap_reg_threads=1024),
            "mreg": {"lsap_wave_max_cols": -1, "lsap_reg_max_cols": -1, "lsap_multi_g": -1,
                     "lsap_sparse_min_cols": -1},
            "lds": noreg,
            "workgroup": dict(noreg, lsap_lds_max_cols=-1),
            "workgroup256": dict(noreg, lsap_lds_max_cols=-1, lsap_mid_max_cols=1000000),
            "multi": {"lsap_wave_max_cols": -1, "lsap_multi_g": 4, "lsap_mreg_max_cols": -1,
                      "lsap_sparse_min_cols": -1},
            "nomreg": {"lsap_mreg_max_cols": -1, "lsap_sparse_min_cols": -1},
            "sparse": {"lsap_wave_max_cols": -1, "lsap_sparse_min_cols": 1},
            "sparse_lo": {"lsap_sparse_min_cols": 1025},
            "sparse_tb1": {"lsap_wave_max_cols": -1, "lsap_sparse_min_cols": 1, "lsap_sparse_blocks": 1},
            "sparse_tb64": {"lsap_sparse_min_cols": 1025, "lsap_sparse_blocks": 64}}[request.param]


def test_random_shapes_and_ties_batched(cuda, lsap_path):
    rng = np.random.default_rng(0)
    mats = []
    for shape in [(1, 1), (3, 5), (5, 3), (7, 7), (40, 9), (9, 40), (64, 16), (300, 20), (0, 4), (4, 0),
                  (65, 2), (129, 7), (257, 30), (600, 24), (24, 600), (1024, 3), (1100, 5), (70, 70),
                  (4096, 6), (6, 4096), (2500, 11), (4097, 3), (513, 7), (768, 5), (5, 768), (769, 4),
                  (1025, 2), (4096, 64), (1100, 1100), (1030, 1025), (5000, 20), (20, 5000),
                  (8193, 8), (12000, 30)]:
        for trial in range(4):
            c = rng.normal(size=shape).astype(np.float32)
            if trial == 1:
                c = np.round(c * 2) / 2
            if trial == 2 and shape[1] > 1:
                c[:, : shape[1] // 2] = c[:, :1]
            if trial == 3:
                c = np.zeros(shape, np.float32)
            mats.append(c)
    for m, (r, c, st) in zip(mats, _batched(cuda, mats, lsap_path)):
        r0, c0 = scipy_lsa(m)
        assert st == 0
        assert np.array_equal(r, r0) and np.array_equal(c, c0), m.shape


def test_float64_costs_equal_scipy(cuda, lsap_path):
    """float64 matrices are assigned in float64 (scipy's own precision):
    values that collapse when narrowed to float32 -- differences below the
    float32 ulp, ties only in float32 -- must still give scipy's answer."""
    rng = np.random.default_rng(7)
    mats = []
    for shape in [(5, 5), (40, 9), (9, 40), (300, 20), (1100, 5), (2500, 11), (70, 70), (4097, 3)]:
        mats.append(10.0 + rng.integers(0, 50, size=shape) * 1e-9)   # all equal in float32
        mats.append(rng.normal(size=shape) * 1e3)
    got = _batched(cuda, mats, lsap_path, dtype=np.float64)
    n_diff32 = 0
    for m, (r, c, st) in zip(mats, got):
        r0, c0 = scipy_lsa(m)
        assert st == 0
        assert np.array_equal(r, r0) and np.array_equal(c, c0), m.shape
        r32, c32 = scipy_lsa(m.astype(np.float32))
        n_diff32 += not (np.array_equal(r32, r0) and np.array_equal(c32, c0))
    assert n_diff32 > 0   # the float32 narrowing really changes some assignments


def test_golden_match_lists(cuda, golden, lsap_path):
    """The reference's match_objects lists from the flattened golden cubes."""
    from bpc_baseline_amd.inference.epipolar_matching import match_objects
    g = golden("a3_cost_cubes.npz")
    cubes = [g[f"{n}_cube"] for n in g["names"]]
    flats = [c.reshape(c.shape[0] * c.shape[1], c.shape[2]) for c in cubes]
    for n, cube, flat, (r, c, st) in zip(g["names"], cubes, flats, _batched(cuda, flats, lsap_path)):
        assert st == 0
        M = cube.shape[1]
        for thr, key in ((30, "match30"), (np.inf, "matchinf")):
            got = np.asarray([(ri // M, ri % M, ci) for ri, ci in zip(r, c) if flat[ri, ci] < thr],
                             np.int64).reshape(-1, 3)
            assert np.array_equal(got, g[f"{n}_{key}"]), (n, thr)
            if lsap_path is None:   # the drop-in itself
                ours = np.asarray(match_objects(cube, thr), np.int64).reshape(-1, 3)
                assert np.array_equal(ours, g[f"{n}_{key}"]), (n, thr)


def test_match_objects_float64_cube(cuda):
    """match_objects on a float64 cube assigns in float64 like the reference's
    scipy call (epipolar_matching.py:106-107), not on a float32 copy."""
    from bpc_baseline_amd.inference.epipolar_matching import match_objects
    rng = np.random.default_rng(3)
    found = 0
    for trial in range(10):
        cube = 5.0 + rng.integers(0, 9, (4, 4, 5)) * 1e-10         # all equal in float32
        flat = cube.reshape(16, 5)
        r0, c0 = scipy_lsa(flat)
        ref = [(r // 4, r % 4, c) for r, c in zip(r0, c0) if flat[r, c] < 30]
        got = match_objects(cube, 30)
        assert [tuple(int(x) for x in m) for m in got] == [tuple(int(x) for x in m) for m in ref]
        r32, _ = scipy_lsa(flat.astype(np.float32))
        found += not np.array_equal(r32, r0)
    assert found > 0


def test_error_statuses(cuda, lsap_path):
    for mats, want in (([np.array([[np.nan, 1.0], [0.0, 2.0]])], 1), ([np.array([[-np.inf, 1.0]])], 1),
                       ([np.array([[np.inf, np.inf], [1.0, 2.0]])], 2)):
        for dtype in (np.float32, np.float64):
            assert _batched(cuda, mats, lsap_path, dtype=dtype)[0][2] == want
    r, c, st = _batched(cuda, [np.array([[np.inf, 1.0], [1.0, np.inf]])], lsap_path)[0]
    assert st == 0 and list(c) == [1, 0]


def test_drop_in_error_messages(cuda):
    from bpc_baseline_amd.inference.epipolar_matching import linear_sum_assignment
    with pytest.raises(ValueError, match="invalid numeric"):
        linear_sum_assignment(np.array([[np.nan, 1.0], [0.0, 2.0]]))
    with pytest.raises(ValueError, match="invalid numeric"):
        linear_sum_assignment(np.array([[-np.inf, 1.0]]))
    with pytest.raises(ValueError, match="infeasible"):
        linear_sum_assignment(np.array([[np.inf, np.inf], [1.0, 2.0]]))
    r, c = linear_sum_assignment(np.array([[np.inf, 1.0], [1.0, np.inf]]))
    assert list(c) == [1, 0]


def test_register_split_class_edges(cuda, lsap_path):
    """Around the split register-state class: long sides 4,097 and 65,536
    (16 workgroups) and 65,537 (beyond: another kernel), the 1,024 short side
    at its LDS capacity, and error problems between valid ones of one slot."""
    rng = np.random.default_rng(11)
    mats = [rng.normal(size=(65536, 5)).astype(np.float32),
            rng.normal(size=(3, 65537)).astype(np.float32),
            rng.normal(size=(4500, 1024)).astype(np.float32),
            np.round(rng.normal(size=(4097, 64)) * 2).astype(np.float32)]
    for m, (r, c, st) in zip(mats, _batched(cuda, mats, lsap_path)):
        r0, c0 = scipy_lsa(m)
        assert st == 0 and np.array_equal(r, r0) and np.array_equal(c, c0), m.shape
    nan = rng.normal(size=(5000, 4)).astype(np.float32)
    nan[4321, 2] = np.nan
    inf = rng.normal(size=(5000, 3)).astype(np.float32)
    inf[:, 1] = np.inf
    ok = rng.normal(size=(6000, 7)).astype(np.float32)
    got = _batched(cuda, [nan, inf, ok, nan, ok], lsap_path)
    assert [g[2] for g in got] == [1, 2, 0, 1, 0]
    r0, c0 = scipy_lsa(ok)
    for r, c, _ in (got[2], got[4]):
        assert np.array_equal(r, r0) and np.array_equal(c, c0)


@pytest.mark.parametrize("path", ["default", "mreg", "one_workgroup", "multi16"])
def test_full_256_cube_equals_scipy(cuda, path):
    """Config-2 scale: the (65536 x 256) flattened 256^3 cube of one scene
    (default: the candidate-list kernels; the split register-state kernel;
    one workgroup; sixteen workgroups of the split workspace-state kernel)."""
    from bpc_baseline_amd.synth import make_scenes
    from oracle import oracle as O
    b = make_scenes(1, 3, 256, seed=42)
    cube, _, _, _, _ = O.cube(b.pts, b.cam_offs, b.F, 1)
    flat = cube.reshape(256 * 256, 256)
    r0, c0 = scipy_lsa(flat)
    opts = {"default": None, "mreg": {"lsap_sparse_min_cols": -1},
            "one_workgroup": {"lsap_multi_g": -1, "lsap_mreg_max_cols": -1, "lsap_sparse_min_cols": -1},
            "multi16": {"lsap_multi_g": 16, "lsap_mreg_max_cols": -1, "lsap_sparse_min_cols": -1}}[path]
    r1, c1, st = _batched(cuda, [flat], opts)[0]
    assert st == 0 and np.array_equal(r0, r1) and np.array_equal(c0, c1)


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_sparse_cubes_batched_equal_scipy(cuda, dtype):
    """The candidate-list kernels on real flattened cubes of 40-130
    detections per view (ragged, several per launch), with duplicated
    detections (exact ties across columns) in some, against scipy."""
    from bpc_baseline_amd.synth import make_capture
    from oracle import oracle as O
    rng = np.random.default_rng(5)
    flats = []
    for k in range(10):
        n = [int(x) for x in rng.integers(40, 131, 3)]
        Ks, RTs, dets = make_capture(np.random.default_rng(100 + k), 3, n, duplicates=3 * (k % 3))
        from bpc_baseline_amd.inference.utils.camera_utils import camera_pairs, fundamental_matrices
        F = fundamental_matrices(Ks, RTs, camera_pairs(3))
        pts = np.concatenate([np.array([d["bb_center"] for d in dets[c]]) for c in range(3)])
        cnt = [len(dets[c]) for c in range(3)]
        co = np.concatenate([[0], np.cumsum(cnt)]).astype(np.int64)
        cube = O.cube(pts, co, np.asarray(F).reshape(3, 9), 1)[0]
        flats.append(cube.reshape(cnt[0] * cnt[1], cnt[2]).astype(dtype))
    for f, (r, c, st) in zip(flats, _batched(cuda, flats, {"lsap_sparse_min_cols": 1025}, dtype=dtype)):
        r0, c0 = scipy_lsa(f)
        assert st == 0 and np.array_equal(r, r0) and np.array_equal(c, c0), f.shape


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
    for m, (r, c, st) in zip(mats, _batched(cuda, mats, lsap_path)):
        assert st == 0
        if m.size:
            r0, c0 = scipy_lsa(m)
            assert np.array_equal(r, r0) and np.array_equal(c, c0)
        else:
            assert r.size == 0 and c.size == 0
