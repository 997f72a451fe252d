"""The cube-free association (ABI 7): mvm_triplet_minima -> mvm_lsap_solve_resid
-> mvm_select_triangulate_resid, what match_captures(keep_cube=False) runs for
the scenes of the candidate-list class.

* the 8-row minima equal, bit for bit, the ones the cube kernel writes next to
  the cube and the ones numpy takes over the oracle cube; the pair residuals
  equal the oracle's (oracle/mvm_oracle.c, epipolar_matching.py:5-28);
* the assignment recomputed from them equals the one reading the cube, and
  scipy's on the oracle cube (epipolar_matching.py:100-116);
* the select/DLT tail equals the cube form: costs, matches, order and X;
* match_captures gives identical matches, costs and X with and without the
  cube on C2-sized, ragged and mixed batches (process_pose.py:165-187);
* invalid inputs: NaN centroids give scipy's invalid-entries status for their
  scene only, problems outside the class status 4, host bounds outside it an
  error, and a short_max below a problem's short side status 4."""
import numpy as np
import pytest
import torch
from scipy.optimize import linear_sum_assignment as scipy_lsa

pytestmark = pytest.mark.gpu


def _scenes(counts, seed, nan_scene=None, nan_view=2, degenerate_scene=None):
    from bpc_baseline_amd.synth import make_scenes
    scenes = [make_scenes(1, 3, list(c), seed=seed + 17 * s) for s, c in enumerate(counts)]
    pts = np.concatenate([x.pts for x in scenes])
    F = np.concatenate([x.F for x in scenes])
    co = np.zeros(3 * len(counts) + 1, np.int64)
    np.cumsum(np.array(counts).reshape(-1), out=co[1:])
    if nan_scene is not None:
        pts = pts.copy()
        pts[co[3 * nan_scene + nan_view] + 5] = np.nan
    if degenerate_scene is not None:
        F = F.copy()
        F[3 * degenerate_scene + 1] = 0.0          # F13 = 0: every e13 is the 9999 sentinel
    return pts, F, co


def _minima(cuda, counts, seed, options=None, **kw):
    from bpc_baseline_amd import ops
    pts, F, co = _scenes(counts, seed, **kw)
    plan = ops.TripletPlan(co, len(counts), device=cuda)
    t = lambda a: torch.from_numpy(a).to(cuda)
    P, C, FF = t(pts), t(co), t(F)
    bm8 = torch.full((max(plan.n_bmin8, 1),), -1, dtype=torch.int16, device=cuda)
    bm32 = torch.full((max(plan.n_bm32, 8),), 0x5A5A, dtype=torch.int16, device=cuda)
    plan.workspace.fill_(0xFF)                       # NaN everywhere the kernel does not write
    minima = ops.triplet_minima(P, C, FF, plan, bmin8=bm8, bm32=bm32, options=options)
    return plan, minima, (pts, F, co), (P, C, FF)


def _want_bm32(keys: np.ndarray, N: int, M: int, P: int) -> np.ndarray:
    from oracle import oracle as O
    return O.bm32_keys(keys, N, M, P)


MINIMA_BATCHES = {
    "c2": [(256, 256, 256), (256, 256, 256)],
    "ragged": [(100, 100, 100), (130, 67, 99), (64, 64, 64), (250, 193, 7), (9, 131, 200)],
    "tails": [(17, 9, 3), (1, 1, 1), (33, 250, 255), (5, 8, 4), (200, 31, 130)],
    "empty": [(0, 10, 10), (10, 0, 10), (10, 10, 0), (40, 70, 50)],
}


@pytest.mark.parametrize("batch", sorted(MINIMA_BATCHES))
def test_minima_equal_cube_kernel_and_oracle(cuda, batch):
    """The 8-row minima (vs the cube kernel's and the oracle cube's), the
    32-column block minima (vs their definition over the oracle's 8-row
    minima, padding rows included) and the fp64 residuals (vs the oracle's)."""
    from bpc_baseline_amd import ops
    from oracle import oracle as O
    counts = MINIMA_BATCHES[batch]
    plan, (bm8, bm32), (pts, F, co), (P, C, FF) = _minima(cuda, counts, 5)
    got = bm8.cpu().numpy().view(np.uint16)
    got32 = bm32.cpu().numpy().view(np.uint16)
    # the cube kernel's own minima on the same batch
    ref8 = torch.full_like(bm8, -1)
    cube, _, _ = ops.triplet_cost_argmin(P, C, FF, plan, bmin8=ref8)
    want_dev = ref8.cpu().numpy().view(np.uint16)
    oc = O.cube(pts, co, F, len(counts))[0]
    max_n = plan.max_n
    ld = (max_n + 3) // 4 * 4
    resid = plan.workspace[:plan.workspace_bytes].view(torch.float64).cpu().numpy()
    resid = resid.reshape(len(counts), 3, max_n, ld)
    want_r = O.residuals(pts, co, F, len(counts), max_n)
    for s, (N, M, Pn) in enumerate(counts):
        if N * M * Pn == 0:
            continue
        o, n8 = plan.bmin8_offs_host[s], N * ((M + 7) // 8) * Pn
        assert np.array_equal(got[o:o + n8], want_dev[o:o + n8]), (batch, s, "vs cube kernel")
        cs = oc[plan.cube_offs_host[s]:plan.cube_offs_host[s + 1]].reshape(N, M, Pn)
        assert np.array_equal(got[o:o + n8], O.bmin8_keys(cs).reshape(-1)), (batch, s, "vs oracle")
        o32 = plan.bm32_offs_host[s]
        want32 = _want_bm32(O.bmin8_keys(cs), N, M, Pn).reshape(-1)
        assert np.array_equal(got32[o32:o32 + want32.size], want32), (batch, s, "block minima")
        for m, (a, b) in enumerate(((N, M), (Pn, N), (Pn, M))):
            g, w = resid[s, m, :a, :b], want_r[s, m, :a, :b]
            assert np.array_equal(g.view(np.int64), w.view(np.int64)), (batch, s, m)


def test_minima_nonfinite_chunks(cuda):
    """NaN centroids and a degenerate F: the rows with non-finite or huge
    residuals take the exact per-entry path (keys equal the oracle's)."""
    from oracle import oracle as O
    counts = [(40, 70, 50), (64, 64, 64), (30, 100, 17)]
    for kw in ({"nan_scene": 1, "nan_view": 0}, {"nan_scene": 0, "nan_view": 1},
               {"nan_scene": 2, "nan_view": 2}, {"degenerate_scene": 1}):
        plan, (bm8, bm32), (pts, F, co), _ = _minima(cuda, counts, 9, **kw)
        got = bm8.cpu().numpy().view(np.uint16)
        got32 = bm32.cpu().numpy().view(np.uint16)
        oc = O.cube(pts, co, F, len(counts))[0]
        for s, (N, M, Pn) in enumerate(counts):
            o, n8 = plan.bmin8_offs_host[s], N * ((M + 7) // 8) * Pn
            cs = oc[plan.cube_offs_host[s]:plan.cube_offs_host[s + 1]].reshape(N, M, Pn)
            assert np.array_equal(got[o:o + n8], O.bmin8_keys(cs).reshape(-1)), (kw, s)
            o32 = plan.bm32_offs_host[s]
            want32 = _want_bm32(O.bmin8_keys(cs), N, M, Pn).reshape(-1)
            assert np.array_equal(got32[o32:o32 + want32.size], want32), (kw, s, "block minima")
        # the block minima alone (no 8-row minima): the same bits
        from bpc_baseline_amd import ops
        t = lambda a: torch.from_numpy(a).to(cuda)
        _, bm32_only = ops.triplet_minima(t(pts), t(co), t(F), plan, with_bmin8=False)
        assert torch.equal(bm32_only[:plan.n_bm32], bm32[:plan.n_bm32]), kw


def _assign_both(cuda, counts, seed, options=None, **kw):
    from bpc_baseline_amd import ops
    plan, minima, host, (P, C, FF) = _minima(cuda, counts, seed, **kw)
    c3 = plan.counts
    lres = ops.LsapPlan(c3[:, 0] * c3[:, 1], c3[:, 2], device=cuda, resid=True)
    r1, c1, s1 = ops.linear_sum_assignment_resid(lres, plan, minima, options=options)
    # the cube form on the same batch
    ref8 = torch.empty_like(minima[0])
    cube, _, _ = ops.triplet_cost_argmin(P, C, FF, plan, bmin8=ref8)
    lplan = ops.LsapPlan(c3[:, 0] * c3[:, 1], c3[:, 2], device=cuda)
    r0, c0, s0 = ops.linear_sum_assignment_batched(cube, plan.cube_offs[:-1].contiguous(), lplan,
                                                   options=options,
                                                   bmin8=(ref8, plan.bmin8_offs, plan.segs))
    return plan, lres, lplan, cube, (r1, c1, s1), (r0, c0, s0), host, (P, C, FF)


ASSIGN_BATCHES = [
    [(256, 256, 256), (256, 256, 256), (256, 256, 256)],
    [(64, 64, 64), (100, 100, 100), (130, 67, 99), (200, 31, 130), (64, 100, 1), (0, 80, 80)],
    [(128, 128, 128), (90, 110, 100), (250, 193, 7)],
]


@pytest.mark.parametrize("counts", ASSIGN_BATCHES)
@pytest.mark.parametrize("blocks", [0, 1, 64])
def test_resid_assignment_equals_cube_and_scipy(cuda, counts, blocks):
    """lsap_sparse_blocks 1: lists run out of free entries and rows fall back to
    the dense scan (recomputed entries everywhere); 64: long lists."""
    opts = {"lsap_sparse_blocks": blocks} if blocks else None
    plan, lres, lplan, cube, (r1, c1, s1), (r0, c0, s0), _, _ = _assign_both(cuda, counts, 11, opts)
    assert (s1.cpu().numpy() == 0).all() and (s0.cpu().numpy() == 0).all()
    r1, c1, r0, c0 = (x.cpu().numpy() for x in (r1, c1, r0, c0))
    assert np.array_equal(r1, r0) and np.array_equal(c1, c0)
    c = cube.cpu().numpy()
    o = lres.out_offs_host
    for s, (N, M, P) in enumerate(counts):
        if N * M * P == 0:
            continue
        rr, cc = scipy_lsa(c[plan.cube_offs_host[s]:plan.cube_offs_host[s + 1]].reshape(N * M, P))
        assert np.array_equal(r1[o[s]:o[s + 1]], rr) and np.array_equal(c1[o[s]:o[s + 1]], cc), (N, M, P)


@pytest.mark.parametrize("counts", ASSIGN_BATCHES)
@pytest.mark.parametrize("blocks", [0, 1])
def test_resid_assignment_without_bmin8(cuda, counts, blocks):
    """No 8-row minima (with_bmin8=False): the block minima and residuals are
    the same bits, and the lists, gathering whole 32-column blocks, give the
    same assignment as the cube form."""
    from bpc_baseline_amd import ops
    opts = {"lsap_sparse_blocks": blocks} if blocks else None
    plan, lres, lplan, cube, _, (r0, c0, s0), _, (P, C, FF) = _assign_both(cuda, counts, 11, opts)
    bm32_with = ops.triplet_minima(P, C, FF, plan)[1].clone()
    ws_with = plan.workspace.clone()
    plan.workspace.fill_(0xFF)
    bm8, bm32 = ops.triplet_minima(P, C, FF, plan, with_bmin8=False)
    assert bm8.numel() == 0
    assert torch.equal(bm32[:plan.n_bm32], bm32_with[:plan.n_bm32])
    for s, (N, M, Pn) in enumerate(counts):      # the residuals the kernel writes, bit for bit
        stride = 3 * plan.max_n * ((plan.max_n + 3) // 4 * 4) * 8
        a = ws_with[s * stride:(s + 1) * stride].view(torch.float64).view(3, plan.max_n, -1)
        b = plan.workspace[s * stride:(s + 1) * stride].view(torch.float64).view(3, plan.max_n, -1)
        for m, (x, y) in enumerate(((N, M), (Pn, N), (Pn, M))):
            assert torch.equal(a[m, :x, :y].view(torch.int64), b[m, :x, :y].view(torch.int64)), (s, m)
    r1, c1, s1 = ops.linear_sum_assignment_resid(lres, plan, (bm8, bm32), options=opts)
    assert (s1.cpu().numpy() == 0).all() and (s0.cpu().numpy() == 0).all()
    assert torch.equal(r1, r0) and torch.equal(c1, c0)


@pytest.mark.parametrize("threshold", [30.0, 200.0, float("inf")])
def test_resid_select_equals_cube_select(cuda, threshold):
    from bpc_baseline_amd import ops
    from bpc_baseline_amd.inference.utils.camera_utils import projection_matrices
    from bpc_baseline_amd.synth import make_scenes
    counts = ASSIGN_BATCHES[1]
    plan, lres, lplan, cube, (r1, c1, _), (r0, c0, _), host, (P, C, FF) = _assign_both(cuda, counts, 13)
    rig = make_scenes(len(counts), 3, 8, seed=3)     # any projection matrices
    proj = torch.from_numpy(np.ascontiguousarray(
        projection_matrices(rig.meta["Ks"], rig.meta["RTs"]))).to(cuda)
    a = ops.select_triangulate_resid(plan, C, lres.out_offs, r1, c1, P, proj, threshold)
    b = ops.select_triangulate(cube, plan.cube_offs, C, lplan.out_offs, r0, c0, P, proj, threshold)
    ca, cb = a[3].cpu().numpy(), b[3].cpu().numpy()
    assert np.array_equal(ca, cb) and ca.sum() > 0
    o = lres.out_offs_host
    for s in range(len(counts)):
        k = slice(o[s], o[s] + ca[s])
        assert np.array_equal(a[0][k].cpu().numpy(), b[0][k].cpu().numpy())
        assert np.array_equal(a[1][k].cpu().numpy().view(np.int32), b[1][k].cpu().numpy().view(np.int32))
        assert np.array_equal(a[2][k].cpu().numpy().view(np.int64), b[2][k].cpu().numpy().view(np.int64))


@pytest.mark.parametrize("nan_view", [0, 1, 2])
def test_resid_nan_status(cuda, nan_view):
    from bpc_baseline_amd import ops
    counts = [(40, 160, 64)] * 3
    plan, minima, _, _ = _minima(cuda, counts, 4, nan_scene=1, nan_view=nan_view)
    c3 = plan.counts
    lres = ops.LsapPlan(c3[:, 0] * c3[:, 1], c3[:, 2], device=cuda, resid=True)
    _, _, st = ops.linear_sum_assignment_resid(lres, plan, minima)
    assert list(st.cpu().numpy()) == [0, 1, 0]


def test_resid_bounds(cuda):
    """Problems outside the candidate-list class cannot be solved without a
    cube: host bounds outside it are an error; on the device (bounds that lie)
    such a problem gets status 4, the others are solved."""
    from bpc_baseline_amd import _native, ops
    counts = [(64, 64, 64), (20, 30, 40), (70, 70, 70)]      # scene 1: a 600 x 40 problem
    plan, minima, _, _ = _minima(cuda, counts, 6)
    c3 = plan.counts
    lres = ops.LsapPlan(c3[:, 0] * c3[:, 1], c3[:, 2], device=cuda, resid=True)
    with pytest.raises(_native.MvmError, match="candidate-list class"):
        ops.linear_sum_assignment_resid(lres, plan, minima)
    lres.long_min = 4096                                      # a caller whose bounds are wrong
    _, _, st = ops.linear_sum_assignment_resid(lres, plan, minima)
    assert list(st.cpu().numpy()) == [0, 4, 0]


def test_short_max_below_a_problem_is_refused(cuda):
    """mvm_lsap_solve_ex3 with a short_max below a problem's short
    side (the LDS and the slots per thread are sized from it) returns status 4
    for that problem instead of writing past its LDS or dropping slots."""
    from bpc_baseline_amd import ops
    counts = [(64, 64, 64), (100, 100, 200), (70, 70, 70)]
    pts, F, co = _scenes(counts, 2)
    plan = ops.TripletPlan(co, 3, device=cuda)
    t = lambda a: torch.from_numpy(a).to(cuda)
    bm8 = torch.empty(plan.n_bmin8, dtype=torch.int16, device=cuda)
    cube, _, _ = ops.triplet_cost_argmin(t(pts), t(co), t(F), plan, bmin8=bm8)
    c3 = plan.counts
    lplan = ops.LsapPlan(c3[:, 0] * c3[:, 1], c3[:, 2], device=cuda)
    lplan.short_max = 100                                     # scene 1 has 200
    _, _, st = ops.linear_sum_assignment_batched(cube, plan.cube_offs[:-1].contiguous(), lplan,
                                                 bmin8=(bm8, plan.bmin8_offs, plan.segs))
    assert list(st.cpu().numpy()) == [0, 4, 0]


def _detector_batch(parts, seed):
    """Concatenated make_detector_batch captures of the given n_dets."""
    from bpc_baseline_amd.synth import make_detector_batch
    bs = [make_detector_batch(n, d, seed=seed + 101 * q) for q, (n, d) in enumerate(parts)]
    img = [np.array([0], np.int64)]
    base = 0
    for b in bs:
        img.append(b.img_offs[1:] + base)
        base += int(b.img_offs[-1])
    cat = lambda k: np.concatenate([getattr(b, k) for b in bs])
    return cat("boxes"), cat("conf"), cat("cls"), np.concatenate(img), cat("Ks"), cat("RTs")


@pytest.mark.parametrize("parts", [
    [(40, 256)],                      # C2-sized captures: every scene cube-free
    [(30, 80), (20, 130)],            # ragged views, all of the class
    [(12, 24), (10, 100), (8, 40)],   # mixed: small scenes keep the cube (split batch)
    [(6, 20)],                        # none of the class: the cube path
])
def test_match_captures_cube_free_equals_keep_cube(cuda, parts):
    from bpc_baseline_amd import ops
    from bpc_baseline_amd.inference.batch_match import match_captures
    boxes, conf, cls, img_offs, Ks, RTs = _detector_batch(parts, 21)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(cuda)
    args = (t(boxes), t(conf), t(cls), t(img_offs), Ks, RTs)
    a = match_captures(*args, keep_cube=False)
    b = match_captures(*args, keep_cube=True)
    assert a.cube is None and b.cube is not None
    assert np.array_equal(a.count, b.count) and np.array_equal(a.offs, b.offs) and a.count.sum() > 0
    for s in range(len(a.count)):
        k = slice(int(a.offs[s]), int(a.offs[s]) + int(a.count[s]))
        assert np.array_equal(a.match[k].cpu().numpy(), b.match[k].cpu().numpy()), s
        assert np.array_equal(a.cost[k].cpu().numpy().view(np.int32), b.cost[k].cpu().numpy().view(np.int32))
        assert np.array_equal(a.X[k].cpu().numpy().view(np.int64), b.X[k].cpu().numpy().view(np.int64))
    counts = np.diff(a.cam_offs).reshape(-1, 3)
    free = ops.cube_free_scenes(counts)
    if len(parts) == 3:
        assert free.any() and not free.all()


@pytest.mark.parametrize("n", [64, 100, 256])
def test_resid_lists_hold_on_small_rows(cuda, n):
    """Every lane of the list kernel holds block keys whatever a row's key
    count (64^3 problems have 128 per row, 256^3 2,048), so theta stays the
    16th-smallest of 64 lane minima and the lists do not overflow wholesale
    (a 64^3 batch once overflowed every list and fell back to dense scans)."""
    from bpc_baseline_amd import ops
    counts = [(n, n, n)] * 8
    plan, lres, _, _, (r1, c1, s1), (r0, c0, s0), _, _ = _assign_both(cuda, counts, 21)
    assert (s1.cpu().numpy() == 0).all()
    assert torch.equal(r1, r0) and torch.equal(c1, c0)
    stats = ops.lsap_sparse_stats(lres)
    rows = sum(c[2] for c in counts)
    assert stats[:, 2].sum() <= 0.02 * rows, stats[:, 2]          # overflowed lists
    assert stats[:, 0].sum() <= 0.05 * rows, stats[:, 0]          # dense free-minimum scans
