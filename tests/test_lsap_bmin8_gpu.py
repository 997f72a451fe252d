"""The cube's 8-row minima (mvm_triplet_cost_argmin_bmin8) and the assignment
that reduces them instead of re-reading the cube (mvm_lsap_solve_ex3):

* the minima equal numpy's over the cube the same launch wrote, on every cube
  kernel path (the fused kernel writes them itself at views of 129-256, the
  others read them back from the cube), ragged views and empty views included;
* the assignment taking them equals the one reading the cost, and scipy's."""
import numpy as np
import pytest
import torch
from scipy.optimize import linear_sum_assignment as scipy_lsa

pytestmark = pytest.mark.gpu


def _keys(cube_flat: np.ndarray) -> np.ndarray:
    """upper 16 bits of the order-preserving key of each cube value (>= +0 or
    +inf; NaN -> 0)"""
    b = (cube_flat.view(np.uint32) | np.uint32(0x80000000)) >> np.uint32(16)
    return np.where(np.isnan(cube_flat), np.uint32(0), b).astype(np.uint16)


def _run(cuda, counts, seed, options=None, nan_scene=None, nan_view=2):
    from bpc_baseline_amd import ops
    from bpc_baseline_amd.synth import make_scenes
    scenes = [make_scenes(1, 3, list(c), seed=seed + 17 * s) for s, c in enumerate(counts)]
    pts = np.concatenate([x.pts for x in scenes])
    F = np.concatenate([x.F for x in scenes])
    co = np.zeros(3 * len(counts) + 1, np.int64)
    np.cumsum(np.array(counts).reshape(-1), out=co[1:])
    if nan_scene is not None:
        pts = pts.copy()
        pts[co[3 * nan_scene + nan_view] + 5] = np.nan       # one point of that scene's view
    dev = cuda
    plan = ops.TripletPlan(co, len(counts), device=dev)
    bm8 = torch.full((max(plan.n_bmin8, 1),), -1, dtype=torch.int16, device=dev)
    cube, _, _ = ops.triplet_cost_argmin(torch.from_numpy(pts).to(dev), torch.from_numpy(co).to(dev),
                                         torch.from_numpy(F).to(dev), plan, options=options, bmin8=bm8)
    return plan, cube, bm8


# batches by largest view (it picks the cube kernel): the fused kernel writes
# the minima itself at one, two, four and eight rows per instruction (3 or 4 k
# per lane, or 5-8 in two panels); the 48-j tiles (views of 33-48), forced
# 32-row tiles at two or four rows per instruction, the small kernel (<= 16),
# the k-chunked kernel (> 256) and the workspace / generic paths read them back
# from the cube
BATCHES = {
    "fused": [(20, 256, 256), (7, 250, 193), (9, 131, 200), (5, 130, 64), (3, 45, 40), (4, 0, 9),
              (6, 33, 0), (11, 8, 1)],
    "fused_kpl3": [(9, 150, 190), (4, 177, 131), (6, 131, 1)],
    "small_views": [(12, 100, 128), (5, 64, 70), (3, 45, 40), (2, 0, 5)],
    "chunked": [(2, 300, 20), (3, 260, 257), (2, 50, 300)],
    "rows2_panels": [(6, 100, 150), (4, 130, 129), (3, 9, 140), (2, 1, 1)],
    "rows4": [(9, 64, 60), (5, 33, 17), (3, 40, 64), (4, 7, 3)],
    "rows4_panels": [(6, 100, 100), (4, 90, 110), (2, 3, 97)],
    "rows8": [(7, 32, 30), (4, 17, 25), (3, 9, 5), (2, 31, 1)],
    "j48": [(5, 48, 40), (3, 40, 33)],
    "tiny": [(3, 16, 16), (4, 5, 12)],
}


@pytest.mark.parametrize("batch", sorted(BATCHES))
@pytest.mark.parametrize("path", ["default", "workspace", "generic", "kpl4", "rows4", "tile32"])
def test_bmin8_equals_numpy(cuda, path, batch):
    opts = {"default": None, "workspace": {"cube_kernel": "workspace"},
            "generic": {"cube_kernel": "generic"}, "kpl4": {"cube_cols_per_lane": 4},
            "rows4": {"cube_rows_per_instr": 4}, "tile32": {"cube_tile_rows": 32}}[path]
    counts = BATCHES[batch]
    plan, cube, bm8 = _run(cuda, counts, 3, opts)
    c = cube.cpu().numpy()
    got = bm8.cpu().numpy().view(np.uint16)
    for s, (N, M, P) in enumerate(counts):
        if N * M * P == 0:
            continue
        cs = c[plan.cube_offs_host[s]:plan.cube_offs_host[s + 1]].reshape(N, M, P)
        g8 = (M + 7) // 8
        pad = np.full((N, g8 * 8, P), np.inf, np.float32)
        pad[:, :M] = cs
        want = _keys(pad.reshape(N, g8, 8, P).min(axis=2).reshape(-1))
        o = plan.bmin8_offs_host[s]
        assert np.array_equal(got[o:o + N * g8 * P], want), (path, s, (N, M, P))


@pytest.mark.parametrize("counts", [
    [(64, 64, 64), (40, 250, 130), (30, 200, 256), (20, 256, 256), (9, 131, 200), (17, 99, 70),
     (3, 2, 5), (5, 0, 3)],
    [(16, 300, 40), (40, 120, 64), (2, 1000, 7)],
    [(64, 64, 64), (80, 100, 100), (60, 90, 64)],
    [(128, 32, 30), (200, 30, 32), (7, 3, 2)],
])
@pytest.mark.parametrize("sparse_from", [0, 1025])
def test_assignment_from_bmin8_equals_scipy(cuda, sparse_from, counts):
    from bpc_baseline_amd import ops
    plan, cube, bm8 = _run(cuda, counts, 8)
    opts = {"lsap_sparse_min_cols": sparse_from} if sparse_from else None
    c3 = plan.counts
    lplan = ops.LsapPlan(c3[:, 0] * c3[:, 1], c3[:, 2], device=cuda)
    offs = plan.cube_offs[:-1].contiguous()
    r1, c1, s1 = ops.linear_sum_assignment_batched(cube, offs, lplan, options=opts,
                                                    bmin8=(bm8, plan.bmin8_offs, plan.segs))
    r0, c0, s0 = ops.linear_sum_assignment_batched(cube, offs, lplan, options=opts)
    r1, c1, r0, c0 = (x.cpu().numpy() for x in (r1, c1, r0, c0))
    assert np.array_equal(s1.cpu().numpy(), s0.cpu().numpy()) and (s0.cpu().numpy() == 0).all()
    assert np.array_equal(r1, r0) and np.array_equal(c1, c0)
    c = cube.cpu().numpy()
    o = lplan.out_offs_host
    for s, (N, M, P) in enumerate(counts):
        if N * M * P == 0:
            continue
        flat = c[plan.cube_offs_host[s]:plan.cube_offs_host[s + 1]].reshape(N * M, P)
        rr, cc = scipy_lsa(flat)
        assert np.array_equal(r1[o[s]:o[s + 1]], rr) and np.array_equal(c1[o[s]:o[s + 1]], cc), (N, M, P)


@pytest.mark.parametrize("nan_view", [0, 1, 2])
@pytest.mark.parametrize("counts", [[(40, 160, 64)] * 3, [(20, 256, 256)] * 3])
def test_assignment_from_bmin8_nan_status(cuda, counts, nan_view):
    """A NaN centroid makes NaN cube entries: the 8-row minima carry them
    (a NaN j point is one NaN row of its eight: the NaN key is the smallest)
    and the assignment reports scipy's invalid-entries status for that scene
    only."""
    from bpc_baseline_amd import ops
    plan, cube, bm8 = _run(cuda, counts, 4, nan_scene=1, nan_view=nan_view)
    c3 = plan.counts
    lplan = ops.LsapPlan(c3[:, 0] * c3[:, 1], c3[:, 2], device=cuda)
    _, _, st = ops.linear_sum_assignment_batched(cube, plan.cube_offs[:-1].contiguous(), lplan,
                                                 bmin8=(bm8, plan.bmin8_offs, plan.segs))
    assert list(st.cpu().numpy()) == [0, 1, 0]
