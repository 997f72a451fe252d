"""GPU parity: HIP kernels (through the C ABI / torch ops) vs the pinned oracle
and the reference's golden vectors.  Bit-exact is the bar: float32 outputs are
compared as bit patterns, argmin indices exactly."""
import numpy as np
import pytest
import torch

from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _bits(a):
    return np.asarray(a, dtype=np.float32).view(np.int32)


def run_pairwise(dev, pts, cam_offs, F, pairs, S, C, want_dist=True, options=None):
    """-> (residuals in the unpitched flat layout, argmin, minval).  ``options``
    may carry "_row_align" (the plan's row pitch; default "auto")."""
    from bpc_baseline_amd import ops
    options = dict(options or {})
    row_align = options.pop("_row_align", "auto")
    plan = ops.PairwisePlan(cam_offs, S, C, pairs, device=dev, row_align=row_align)
    d, a, m = ops.pairwise_residual_argmin(
        torch.from_numpy(np.ascontiguousarray(pts, np.float64)).to(dev),
        torch.from_numpy(np.ascontiguousarray(cam_offs, np.int64)).to(dev),
        torch.from_numpy(np.ascontiguousarray(F, np.float64)).to(dev), plan, want_dist=want_dist,
        options=options or None)
    torch.cuda.synchronize()
    if want_dist:
        if plan.dist_size != plan.n_dist:
            assert_padding_inf(plan, d.cpu().numpy())
        d = plan.compact(d)
    return d.cpu().numpy(), a.cpu().numpy(), m.cpu().numpy()


def assert_padding_inf(plan, h):
    """include/mvmatch.h: every kernel path writes +inf into a pitched row's
    padding columns (degenerate and non-finite rows, the generic and strided
    paths, multi-tile views included)."""
    for sp in range(plan.na.size):
        o, na, nb, ld = (int(x) for x in (plan.dist_offs_host[sp], plan.na[sp], plan.nb[sp],
                                           plan.ld[sp]))
        pad = h[o:o + na * ld].reshape(na, ld)[:, nb:]
        assert np.all(np.isposinf(pad)), \
            f"matrix {sp} ({na}x{nb}, ld {ld}): padding not +inf at {np.argwhere(~np.isposinf(pad))[:4]}"


def run_cube(dev, pts, cam_offs, F, S, options=None):
    from bpc_baseline_amd import ops
    plan = ops.TripletPlan(cam_offs, S, device=dev)
    c, a, m = ops.triplet_cost_argmin(
        torch.from_numpy(np.ascontiguousarray(pts, np.float64)).to(dev),
        torch.from_numpy(np.ascontiguousarray(cam_offs, np.int64)).to(dev),
        torch.from_numpy(np.ascontiguousarray(F, np.float64)).to(dev), plan, options=options)
    torch.cuda.synchronize()
    return c.cpu().numpy(), a.cpu().numpy(), m.cpu().numpy()


def assert_pairwise_equal(dev, pts, cam_offs, F, pairs, S, C, options=None):
    d, a, m = run_pairwise(dev, pts, cam_offs, F, pairs, S, C, options=options)
    rd, ra, rm, _, _ = O.pairwise(pts, cam_offs, F, pairs, S, C)
    assert d.shape == rd.shape
    bad = np.nonzero(_bits(d) != _bits(rd))[0]
    assert bad.size == 0, f"{bad.size} dist mismatches, first at {bad[:5]}: {d[bad[:5]]} vs {rd[bad[:5]]}"
    assert np.array_equal(a, ra), f"argmin mismatches at {np.nonzero(a != ra)[0][:10]}"
    assert np.array_equal(_bits(m), _bits(rm))


# ----------------------------------------------------------- pairwise ----
@pytest.fixture(params=["default", "unpitched", "eager", "eager_unpitched", "rpw8_rg2", "rpw4",
                        "interleaved", "contiguous", "interleaved_unpitched_rpw8", "fronts3",
                        "fronts16_unpitched"])
def argmin_path(request):
    """mvm_options of a pairwise kernel path: the lazy argmin (clean row
    groups: per-chunk minimum bits, column recovered per group through one
    LDS transpose; the default), the eager argmin, other row-group shapes (8
    rows per wave x 2 groups, 4 rows per wave), a row group's rows interleaved
    over the waves or contiguous per wave (forced either way; the default
    picks by view size) -- each with the plan's default row pitch (128-byte
    lines for ragged views) and some also unpitched (rows of n_b, the
    unaligned-row paths), and the XCD write-front counts forced (3, 16: ranges
    of unequal length per XCD)."""
    return {"default": {}, "unpitched": {"_row_align": 1},
            "interleaved": {"pairwise_row_interleave": 1},
            "contiguous": {"pairwise_row_interleave": -1},
            "interleaved_unpitched_rpw8": {"pairwise_row_interleave": 1, "_row_align": 1,
                                           "pairwise_rows_per_wave": 8},
            "eager": {"pairwise_argmin": "eager"},
            "eager_unpitched": {"pairwise_argmin": "eager", "_row_align": 1},
            "rpw8_rg2": {"pairwise_rows_per_wave": 8, "pairwise_row_groups": 2},
            "rpw4": {"pairwise_rows_per_wave": 4},
            "fronts3": {"pairwise_xcd_fronts": 3},
            "fronts16_unpitched": {"pairwise_xcd_fronts": 16, "_row_align": 1}}[request.param]


@pytest.mark.parametrize("S,C,n,ragged", [(3, 4, 256, False), (5, 4, 300, True), (2, 4, 1024, False),
                                          (4, 3, 37, True), (2, 2, 1, False), (3, 6, 130, True),
                                          (1, 3, 2500, False), (3, 2, 1500, True), (1, 8, 300, True),
                                          (3, 4, 1000, True), (2, 3, 800, False), (2, 2, 1021, False),
                                          (2, 3, 1024, True), (1, 2, 1000, False)])
def test_pairwise_synthetic_vs_oracle(cuda, S, C, n, ragged, argmin_path):
    from bpc_baseline_amd.synth import make_scenes
    b = make_scenes(S, C, n, seed=100 + S * n, ragged=ragged)
    assert_pairwise_equal(cuda, b.pts, b.cam_offs, b.F, b.pairs, S, C, options=argmin_path)


def test_pairwise_golden_4cam(cuda, golden):
    """Reference epipolar_error over every pair of a 4-camera capture (empty view, duplicates)."""
    g = golden("a5_pairwise.npz")
    pairs = g["pairs"]
    views = [g[f"pts{c}"] for c in range(4)]
    cam_offs = np.zeros(5, np.int64)
    np.cumsum([len(v) for v in views], out=cam_offs[1:])
    pts = np.concatenate(views)
    d, a, _ = run_pairwise(cuda, pts, cam_offs, g["F"], pairs, 1, 4)
    from bpc_baseline_amd.ops import PairwisePlan
    plan = PairwisePlan(cam_offs, 1, 4, pairs, device="cpu", row_align=1)
    for p, (ca, cb) in enumerate(pairs):
        ref = g[f"e{ca}{cb}"]
        got = plan.matrix(torch.from_numpy(d), 0, p).numpy()
        assert got.shape == ref.shape
        assert np.array_equal(_bits(got), _bits(ref)), f"pair {ca}{cb}"
        ro = plan.row_offs_host
        assert np.array_equal(a[ro[p]:ro[p + 1]], g[f"argmin{ca}{cb}"])


def test_pairwise_f64_kats(cuda, golden):
    """Every scalar epipolar_error KAT as its own scene: fp64 bits must match the reference."""
    from bpc_baseline_amd import ops
    g = golden("a1_epipolar_error.npz")
    n = len(g["e"])
    pts = np.stack([g["p1"], g["p2"]], axis=1).reshape(-1, 2)
    cam_offs = np.arange(2 * n + 1, dtype=np.int64)
    plan = ops.PairwisePlan(cam_offs, n, 2, [[0, 1]], device=cuda)
    e = ops.pairwise_residual_f64(torch.from_numpy(pts).to(cuda), torch.from_numpy(cam_offs).to(cuda),
                                  torch.from_numpy(g["F"].copy()).to(cuda), plan)
    got = e[:, 0, 0].cpu().numpy()
    bad = np.nonzero(got.view(np.int64) != g["e"].view(np.int64))[0]
    assert bad.size == 0, f"{bad.size} fp64 mismatches (kinds {np.unique(g['kind'][bad])}): " \
                          f"{got[bad[:3]]} vs {g['e'][bad[:3]]}"


def test_pairwise_edge_cases(cuda, argmin_path):
    """Degenerate lines (9999 sentinel), NaN / inf / huge centroids, tails, misalignment."""
    rng = np.random.default_rng(5)
    C, S = 3, 6
    counts = np.array([[5, 7, 3], [1, 1, 1], [9, 0, 4], [3, 6, 5], [2, 3, 2], [6, 5, 7]])
    cam_offs = np.zeros(S * C + 1, np.int64)
    np.cumsum(counts.reshape(-1), out=cam_offs[1:])
    pts = np.floor(rng.uniform(0, 4800, size=(cam_offs[-1], 2))) / 2
    pts[3] = [np.nan, 4.0]
    pts[9] = [np.inf, 1.0]
    pts[20] = [1e300, -1e300]
    pts[21] = [2.0 ** 41, 7.0]
    pairs = np.array([[0, 1], [0, 2], [1, 2]], np.int32)
    F = rng.normal(size=(S * 3, 9))
    F[0, 0:6] = 0.0             # degenerate row lines (F rows 0,1 = 0)
    F[1, [0, 1, 3, 4, 6, 7]] = 0.0   # degenerate column lines (F cols 0,1 = 0)
    F[2] = 0.0                  # both
    F[5] *= 1e-9                # norms near the 1e-8 threshold
    F[7, 2] = 1e70              # huge l2
    assert_pairwise_equal(cuda, pts, cam_offs, F, pairs, S, C, options=argmin_path)


@pytest.mark.parametrize("counts", [(1000, 996, 1016, 1012), (72, 100, 132, 1020), (260, 4, 1000, 36)])
def test_pairwise_rows_off_line_boundaries(cuda, counts, argmin_path):
    """Views whose counts are not multiples of 32 (n_b % 4 == 0): unpitched,
    rows start mid-line and the lazy path masks the lanes past n_b in the
    last chunk; pitched (the default), rows start on lines and the padding is
    written.  Views of different sizes in one scene (misaligned matrix
    offsets when unpitched), a degenerate pair and a NaN centroid."""
    rng = np.random.default_rng(sum(counts))
    S, C = 2, len(counts)
    cnt = np.array([counts, counts[::-1]], np.int64)
    cam_offs = np.zeros(S * C + 1, np.int64)
    np.cumsum(cnt.reshape(-1), out=cam_offs[1:])
    pts = np.floor(rng.uniform(0, 4800, size=(cam_offs[-1], 2))) / 2
    pairs = np.array([[a, b] for a in range(C) for b in range(C) if a != b], np.int32)
    F = rng.normal(size=(S * len(pairs), 9))
    F[1, [0, 1, 3, 4, 6, 7]] = 0.0      # degenerate column lines: the generic path, shifted
    pts[int(cam_offs[1]) + 2] = [np.nan, 1.0]
    assert_pairwise_equal(cuda, pts, cam_offs, F, pairs, S, C, options=argmin_path)


def test_pairwise_wide_views_edge_cases(cuda, argmin_path):
    """Views of 769..1024 columns (C3's shape: several column chunks per
    wave, the lazy argmin's chunk recovery) with degenerate lines, NaN / inf / huge centroids and a column
    count that leaves the last wave's lanes partly empty."""
    from bpc_baseline_amd.synth import make_scenes
    b = make_scenes(3, 3, 900, seed=77)
    pts = b.pts.copy()
    o1 = int(b.cam_offs[1])
    pts[o1 + 5] = [np.nan, 3.0]          # a NaN column (scene 0, camera 1)
    pts[o1 + 700] = [np.inf, 1.0]
    pts[7] = [1e300, -1e300]            # a wild row (scene 0, camera 0)
    pts[int(b.cam_offs[4]) + 3] = [2.0 ** 41, 7.0]
    F = b.F.copy()
    F[3, 0:6] = 0.0                     # scene 1, pair (0,1): degenerate row lines
    F[5, [0, 1, 3, 4, 6, 7]] = 0.0      # scene 1, pair (1,2): degenerate column lines
    assert_pairwise_equal(cuda, pts, b.cam_offs, F, b.pairs, 3, 3, options=argmin_path)


def test_pairwise_ties_and_duplicates(cuda, argmin_path):
    """Duplicate detections give exact ties across lanes and chunks: lowest index wins."""
    from bpc_baseline_amd.synth import make_scenes
    b = make_scenes(2, 3, 600, seed=3)
    pts = b.pts.copy()
    # cam 1 of scene 0: copy column 3 into columns 300 and 517 (other chunk / other lane)
    o = b.cam_offs[1]
    pts[o + 300] = pts[o + 3]
    pts[o + 517] = pts[o + 3]
    pts[o + 4] = pts[o + 3]
    assert_pairwise_equal(cuda, pts, b.cam_offs, b.F, b.pairs, 2, 3, options=argmin_path)


@pytest.mark.parametrize("n", [256, 512, 1024, 600, 1000])
def test_pairwise_row_minimum_ties(cuda, n, argmin_path):
    """Exact ties AT the row minimum in clean views (the lazy path's case):
    a row's winning column is duplicated inside its own 4-column lane group
    (lower and higher q), in the same lane of another chunk, and in another
    lane -- np.argmin's lowest index must win every time."""
    from bpc_baseline_amd.synth import make_scenes
    b = make_scenes(2, 3, n, seed=11 + n)
    pts = b.pts.copy()
    _, ra, _, _, _ = O.pairwise(pts, b.cam_offs, b.F, b.pairs, 2, 3, want_dist=False)
    ro = np.concatenate([[0], np.cumsum([n] * 6)])
    for s_, p_, row in ((0, 0, 0), (0, 2, 5), (1, 1, 17), (1, 0, n - 1)):
        cam_b = int(b.pairs[p_][1])
        j0 = int(ra[ro[s_ * 3 + p_] + row])
        ob = int(b.cam_offs[s_ * 3 + cam_b])
        for j in {j0 ^ 1, j0 ^ 3, (j0 + 256) % n, (j0 + 4 * 7 + 1) % n, (j0 + 300) % n}:
            pts[ob + j] = pts[ob + j0]
    assert_pairwise_equal(cuda, pts, b.cam_offs, b.F, b.pairs, 2, 3, options=argmin_path)


@pytest.mark.parametrize("row_align", [4, 32, 256])
def test_pairwise_pitched_layout(cuda, row_align):
    """mvm_pairwise_residual_argmin_pitched: row i of matrix (s, p) at
    dist_offs[sp] + i * roundup(n_b, row_align).  Ragged IPD-like counts
    (700..1024 and a few small views): every residual and argmin equal to the
    oracle, every padding column +inf (clean views: the kernel writes whole
    pitched rows), and nothing written past a matrix's pitched extent."""
    from bpc_baseline_amd import ops
    rng = np.random.default_rng(row_align)
    S, C = 5, 4
    cnt = rng.integers(700, 1025, size=(S, C))
    cnt[1, 2], cnt[3, 0], cnt[4, 1] = 33, 1, 255
    cam_offs = np.zeros(S * C + 1, np.int64)
    np.cumsum(cnt.reshape(-1), out=cam_offs[1:])
    from bpc_baseline_amd.synth import make_scenes
    b = make_scenes(S, C, 1024, seed=row_align)
    pts = np.concatenate([b.pts[int(b.cam_offs[v]):int(b.cam_offs[v]) + int(cnt.reshape(-1)[v])]
                          for v in range(S * C)])
    plan = ops.PairwisePlan(cam_offs, S, C, b.pairs, device=cuda, row_align=row_align)
    assert plan.row_align == row_align and np.all(plan.ld % row_align == 0)
    assert np.all(plan.dist_offs_host % row_align == 0)
    guard = plan.dist_size + 64
    dist = torch.full((guard,), -7.0, dtype=torch.float32, device=cuda)
    am = torch.empty(plan.n_rows, dtype=torch.int32, device=cuda)
    mv = torch.empty(plan.n_rows, dtype=torch.float32, device=cuda)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(cuda)
    ops.pairwise_residual_argmin(t(pts), t(cam_offs), t(b.F), plan, out=(dist, am, mv))
    torch.cuda.synchronize()
    rd, ra, rm, _, _ = O.pairwise(pts, cam_offs, b.F, b.pairs, S, C)
    assert np.array_equal(_bits(plan.compact(dist).cpu().numpy()), _bits(rd))
    assert np.array_equal(am.cpu().numpy(), ra) and np.array_equal(_bits(mv.cpu().numpy()), _bits(rm))
    h = dist.cpu().numpy()
    for sp in range(plan.na.size):
        o, na, nb, ld = (int(x) for x in (plan.dist_offs_host[sp], plan.na[sp], plan.nb[sp],
                                           plan.ld[sp]))
        pad = h[o:o + na * ld].reshape(na, ld)[:, nb:]
        assert np.all(np.isposinf(pad)), f"matrix {sp}: padding not +inf"
    assert np.all(h[plan.dist_size:] == -7.0)


def test_pairwise_argmin_only(cuda, argmin_path):
    from bpc_baseline_amd.synth import make_scenes
    b = make_scenes(2, 4, 200, seed=9)
    d, a, m = run_pairwise(cuda, b.pts, b.cam_offs, b.F, b.pairs, 2, 4, want_dist=False,
                           options=argmin_path)
    _, ra, rm, _, _ = O.pairwise(b.pts, b.cam_offs, b.F, b.pairs, 2, 4, want_dist=False)
    assert d.size == 0
    assert np.array_equal(a, ra) and np.array_equal(_bits(m), _bits(rm))


# --------------------------------------------------------------- cube ----
# largest view each forced lane shape holds (3 k: 192 at one row per
# instruction; 5 k: 160 at two; 8 k at two rows: 256)
KPL_MAX_VIEW = {"fused_kpl3": 192, "fused_kpl5": 160, "fused_rows2_kpl8": 256, "fused_tile32_kpl5": 160}


@pytest.fixture(params=["default", "small", "fused", "fused_rows2", "fused_rows1", "fused_kpl4",
                        "fused_rows1_kpl4", "fused_kpl3", "fused_kpl5", "fused_rows2_kpl8", "fused_tile32",
                        "fused_tile32_kpl5", "fused_rows8_tile16", "fused_rows4", "workspace",
                        "generic"])
def cube_path(request):
    """mvm_options of each cube kernel: the small-scene kernel (views of < 64
    detections), the fused tiled kernel (pair residuals computed in the
    prologue; up to 256, then its k-chunked form) with four / two / one
    (i, j) rows per wave instruction (eight up to 32: rows8_tile16 with tiles of
    16 i rows, the default 32; rows4 the four-row form there) -- 3 k per lane where the view fits them
    (the default), or 4 forced (kpl4), or 3 forced (kpl3: fewer rows per
    instruction where the view needs them; views of <= 192 only), or 5 / 8
    forced (the split forms' wide lanes: views of <= 160 / <= 256), tiles of
    32 i rows (tile32: the split forms; one row per instruction keeps 16) -- the
    tiled kernel over the fp64 workspace (beyond 256: the generic kernel) and
    the generic kernel."""
    return request.param, {"default": {}, "small": {"cube_kernel": "small"},
                           "fused": {"cube_kernel": "fused"},
                           "fused_rows2": {"cube_kernel": "fused", "cube_rows_per_instr": 2},
                           "fused_rows1": {"cube_kernel": "fused", "cube_rows_per_instr": 1},
                           "fused_kpl4": {"cube_kernel": "fused", "cube_cols_per_lane": 4},
                           "fused_rows1_kpl4": {"cube_kernel": "fused", "cube_rows_per_instr": 1,
                                                "cube_cols_per_lane": 4},
                           "fused_kpl3": {"cube_kernel": "fused", "cube_cols_per_lane": 3},
                           "fused_kpl5": {"cube_kernel": "fused", "cube_cols_per_lane": 5},
                           "fused_rows2_kpl8": {"cube_kernel": "fused", "cube_rows_per_instr": 2,
                                                "cube_cols_per_lane": 8},
                           "fused_tile32": {"cube_kernel": "fused", "cube_tile_rows": 32},
                           "fused_rows8_tile16": {"cube_kernel": "fused", "cube_rows_per_instr": 8,
                                                  "cube_tile_rows": 16},
                           "fused_rows4": {"cube_kernel": "fused", "cube_rows_per_instr": 4},
                           "fused_tile32_kpl5": {"cube_kernel": "fused", "cube_tile_rows": 32,
                                                 "cube_cols_per_lane": 5},
                           "workspace": {"cube_kernel": "workspace"},
                           "generic": {"cube_kernel": "generic"}}[request.param]


def test_cube_golden_batched(cuda, golden, cube_path):
    """All reference compute_cost_matrix cubes in ONE ragged batched launch."""
    g = golden("a3_cost_cubes.npz")
    names = list(g["names"])
    path, opts = cube_path
    if path == "small":           # keep the batch inside the small kernel's range
        names = [n for n in names if max(len(g[f"{n}_p{v}"]) for v in (1, 2, 3)) <= 64]
        assert len(names) >= 8
    views, Fs = [], []
    for n in names:
        views += [g[f"{n}_p1"], g[f"{n}_p2"], g[f"{n}_p3"]]
        Fs.append(g[f"{n}_F"])
    cam_offs = np.zeros(len(views) + 1, np.int64)
    np.cumsum([len(v) for v in views], out=cam_offs[1:])
    c, a, _ = run_cube(cuda, np.concatenate(views), cam_offs, np.concatenate(Fs), len(names),
                       options=opts)
    co = ro = 0
    for n in names:
        ref = g[f"{n}_cube"]
        N, M, P = ref.shape
        got = c[co:co + ref.size]
        assert np.array_equal(_bits(got), _bits(ref.reshape(-1))), f"cube {n}"
        assert np.array_equal(a[ro:ro + N * M], g[f"{n}_argmin"]), f"argmin {n}"
        co += ref.size
        ro += N * M


def test_cube_golden_mid_sizes(cuda, golden, cube_path):
    """The reference's own cubes at the fused kernel's lane / tile boundaries
    (views of 47/48: 3 k per lane with a partial last lane, 48-wide j tiles;
    97: 4 k per lane, rows off 16 bytes; 150: 3 k per lane at one row per
    instruction; 250: rows off 16 bytes at one row per instruction), each in
    its own launch so each takes its size's kernel, on every cube path."""
    g = golden("a3b_cost_cubes_mid.npz")
    path, opts = cube_path
    for n in g["names"]:
        p = [g[f"{n}_p{k}"] for k in (1, 2, 3)]
        if max(len(x) for x in p) > KPL_MAX_VIEW.get(path, 1 << 30):
            continue                                  # views the forced lane shape cannot hold
        cam_offs = np.array([0, len(p[0]), len(p[0]) + len(p[1]), sum(len(x) for x in p)], np.int64)
        c, a, _ = run_cube(cuda, np.concatenate(p), cam_offs, g[f"{n}_F"], 1, options=opts)
        assert np.array_equal(_bits(c), _bits(g[f"{n}_cube"].reshape(-1))), f"cube {n}"
        assert np.array_equal(a, g[f"{n}_argmin"]), f"argmin {n}"


@pytest.mark.parametrize("S,n,ragged", [(3, 64, False), (1, 300, False), (4, 45, True), (2, 256, False),
                                        (300, 24, False), (40, 64, True), (7, 1, False),
                                        (2, 512, False), (3, 333, True), (1, 770, False), (2, 200, False),
                                        (2, 384, False), (20, 96, False), (6, 100, True), (5, 128, False),
                                        (9, 77, True), (4, 68, False), (3, 160, False),
                                        (2, 192, False), (3, 48, False), (3, 150, True),
                                        (4, 190, True), (5, 47, True), (3, 93, False)])
def test_cube_synthetic_vs_oracle(cuda, S, n, ragged, cube_path):
    from bpc_baseline_amd.synth import make_scenes
    if n > KPL_MAX_VIEW.get(cube_path[0], 1 << 30):
        pytest.skip("views the forced lane shape cannot hold")
    b = make_scenes(S, 3, n, seed=7 * n + S, ragged=ragged)
    c, a, m = run_cube(cuda, b.pts, b.cam_offs, b.F, S, options=cube_path[1])
    rc, ra, rm, _, _ = O.cube(b.pts, b.cam_offs, b.F, S)
    bad = np.nonzero(_bits(c) != _bits(rc))[0]
    assert bad.size == 0, f"{bad.size} cube mismatches"
    assert np.array_equal(a, ra)
    assert np.array_equal(_bits(m), _bits(rm))


def test_deterministic_repeat(cuda):
    from bpc_baseline_amd.synth import make_scenes
    b = make_scenes(4, 4, 700, seed=1)
    r1 = run_pairwise(cuda, b.pts, b.cam_offs, b.F, b.pairs, 4, 4)
    r2 = run_pairwise(cuda, b.pts, b.cam_offs, b.F, b.pairs, 4, 4)
    for x, y in zip(r1, r2):
        assert np.array_equal(np.asarray(x).view(np.uint8), np.asarray(y).view(np.uint8))


def test_launches_capture_into_a_hip_graph(cuda):
    """The C ABI enqueues work only (no allocation, copy or sync inside), so a
    step of launches can be captured into a hipGraph (torch.cuda.CUDAGraph on
    ROCm) and replayed; replay reproduces the eager results bit for bit."""
    from bpc_baseline_amd import ops
    from bpc_baseline_amd.synth import make_scenes
    b = make_scenes(6, 4, 200, seed=12)
    c = make_scenes(4, 3, 40, seed=13)
    pp = ops.PairwisePlan(b.cam_offs, b.n_scenes, b.n_cams, b.pairs, device=cuda)
    tp = ops.TripletPlan(c.cam_offs, c.n_scenes, device=cuda)
    t = lambda a: torch.from_numpy(a).to(cuda)
    bp, bc, bF = t(b.pts), t(b.cam_offs), t(b.F)
    cp, cc, cF = t(c.pts), t(c.cam_offs), t(c.F)
    dist = torch.empty(pp.dist_size, dtype=torch.float32, device=cuda)
    am = torch.empty(pp.n_rows, dtype=torch.int32, device=cuda)
    mv = torch.empty(pp.n_rows, dtype=torch.float32, device=cuda)
    cube = torch.empty(tp.n_cube, dtype=torch.float32, device=cuda)
    cam = torch.empty(tp.n_rows, dtype=torch.int32, device=cuda)
    cmv = torch.empty(tp.n_rows, dtype=torch.float32, device=cuda)

    def step():
        ops.pairwise_residual_argmin(bp, bc, bF, pp, out=(dist, am, mv))
        ops.triplet_cost_argmin(cp, cc, cF, tp, out=(cube, cam, cmv))

    s = torch.cuda.Stream(cuda)
    s.wait_stream(torch.cuda.current_stream(cuda))
    with torch.cuda.stream(s):
        step()                                   # warm-up on the side stream
    torch.cuda.current_stream(cuda).wait_stream(s)
    ref = [x.clone() for x in (dist, am, cube, cam)]
    for x in (dist, am, cube, cam):
        x.zero_()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        step()
    g.replay()
    torch.cuda.synchronize(cuda)
    for x, r in zip((dist, am, cube, cam), ref):
        assert torch.equal(x.view(torch.int32) if x.dtype == torch.float32 else x,
                           r.view(torch.int32) if r.dtype == torch.float32 else r)


@pytest.mark.parametrize("n", [520, 256, 100, 60])
def test_cube_row_minimum_ties_across_chunks(cuda, cube_path, n):
    """A row's winning k duplicated in its own lane group, in another lane and
    (views of more than 256) in the same lane of the next 256-chunk and in the
    ragged tail chunk; the lowest k must win (the chunked kernel keeps the
    earliest chunk).  n = 100 runs the two-rows-per-wave kernel, with rows in
    both halves of a wave (wave rows 0..3 and 4..7); n = 256 runs the fused
    kernel's full-tile loop, whose in-lane first index comes from lane masks
    (k0 ^ 1, k0 ^ 2, k0 ^ 3: every q position of the winner's lane)."""
    from bpc_baseline_amd.synth import make_scenes
    if n > KPL_MAX_VIEW.get(cube_path[0], 1 << 30):
        pytest.skip("views the forced lane shape cannot hold")
    b = make_scenes(1, 3, n, seed=21)
    pts = b.pts.copy()
    _, ra, _, _, _ = O.cube(pts, b.cam_offs, b.F, 1, want_cube=False)
    o3 = int(b.cam_offs[2])
    for row in (0, 77, 6 * n + 5):
        k0 = int(ra[row])
        for k in {k0 ^ 1, k0 ^ 2, k0 ^ 3, (k0 + 256) % n, (k0 + 260) % n, n - 3} - {k0}:
            pts[o3 + k] = pts[o3 + k0]
    c, a, m = run_cube(cuda, pts, b.cam_offs, b.F, 1, options=cube_path[1])
    rc, ra, rm, _, _ = O.cube(pts, b.cam_offs, b.F, 1)
    assert np.array_equal(_bits(c), _bits(rc))
    assert np.array_equal(a, ra)
    assert np.array_equal(_bits(m), _bits(rm))
