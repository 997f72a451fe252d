"""Host-side logic (CPU): plans, synthetic generator, sharding, input
validation, the 'no CPU path' contract, and the float32-exactness claim of
the kernel's exponent-decrement halving."""
import math
import os

import numpy as np
import pytest
import torch

from oracle import oracle as O


def test_pairwise_plan_offsets_match_oracle():
    from bpc_baseline_amd import ops
    from bpc_baseline_amd.synth import make_scenes
    b = make_scenes(7, 4, 33, seed=2, ragged=True)
    plan = ops.PairwisePlan(b.cam_offs, b.n_scenes, b.n_cams, b.pairs, device="cpu", row_align=1)
    doff, roff = O.pairwise_offsets(b.cam_offs, b.n_scenes, b.n_cams, b.pairs)
    assert np.array_equal(plan.dist_offs_host, doff) and np.array_equal(plan.row_offs_host, roff)
    assert plan.n_dist == plan.dist_size == b.n_residual_pairs()
    assert plan.max_n == int(b.counts().max())


@pytest.mark.parametrize("row_align", ["auto", 4, 32, 256])
def test_pairwise_plan_pitched_rows(row_align):
    """Pitched plans: ld = roundup(n_b, row_align); matrices back to back with
    n_a * ld floats each; "auto" pitches to 32 floats (128-byte lines) when a
    count is not a multiple of 32 and is unpitched otherwise; matrix() and
    compact() read the unpitched values back."""
    from bpc_baseline_amd import ops
    from bpc_baseline_amd.synth import make_scenes
    b = make_scenes(3, 4, 33, seed=2, ragged=True)
    plan = ops.PairwisePlan(b.cam_offs, b.n_scenes, b.n_cams, b.pairs, device="cpu",
                            row_align=row_align)
    ra = 32 if row_align == "auto" else row_align
    assert plan.row_align == ra
    assert np.array_equal(plan.ld, (plan.nb + ra - 1) // ra * ra)
    assert np.array_equal(np.diff(plan.dist_offs_host), plan.na * plan.ld)
    assert plan.n_dist == b.n_residual_pairs() and plan.dist_size == int(plan.dist_offs_host[-1])
    flat = O.pairwise(b.pts, b.cam_offs, b.F, b.pairs, b.n_scenes, b.n_cams)[0]
    # lay the oracle's values out pitched (padding = +inf), read them back
    pitched = np.full(plan.dist_size, np.inf, np.float32)
    o = 0
    for sp in range(plan.na.size):
        na, nb, ld, d0 = (int(x) for x in (plan.na[sp], plan.nb[sp], plan.ld[sp],
                                           plan.dist_offs_host[sp]))
        pitched[d0:d0 + na * ld].reshape(na, ld)[:, :nb] = flat[o:o + na * nb].reshape(na, nb)
        got = plan.matrix(torch.from_numpy(pitched), sp // 6, sp % 6).numpy()
        assert np.array_equal(got, flat[o:o + na * nb].reshape(na, nb))
        o += na * nb
    assert np.array_equal(plan.compact(torch.from_numpy(pitched)).numpy(), flat)
    u = ops.PairwisePlan(np.array([0, 64, 96], np.int64), 1, 2, [[0, 1]], device="cpu",
                         row_align="auto")
    assert u.row_align == 1 and u.dist_size == u.n_dist == 64 * 32
    # the default is the unpitched contract (matrices back to back) even for
    # ragged counts: pitching is opt-in
    d = ops.PairwisePlan(b.cam_offs, b.n_scenes, b.n_cams, b.pairs, device="cpu")
    assert d.row_align == 1 and d.dist_size == d.n_dist
    with pytest.raises(ValueError):
        ops.PairwisePlan(b.cam_offs, b.n_scenes, b.n_cams, b.pairs, device="cpu", row_align=48)


def test_triplet_plan_offsets():
    from bpc_baseline_amd import ops
    from bpc_baseline_amd.synth import make_scenes
    b = make_scenes(5, 3, 20, seed=3, ragged=True)
    plan = ops.TripletPlan(b.cam_offs, b.n_scenes, device="cpu")
    coff, roff = O.cube_offsets(b.cam_offs, b.n_scenes)
    assert np.array_equal(plan.cube_offs_host, coff) and np.array_equal(plan.row_offs_host, roff)
    assert plan.workspace.numel() >= plan.workspace_bytes


def test_synth_is_deterministic_and_shardable():
    from bpc_baseline_amd.synth import make_scenes
    full = make_scenes(6, 3, 16, seed=11)
    tail = make_scenes(3, 3, 16, seed=11, first_scene=3)
    assert np.array_equal(full.F[3 * 3:], tail.F)
    assert np.array_equal(full.pts[full.cam_offs[9]:], tail.pts)
    again = make_scenes(6, 3, 16, seed=11)
    assert np.array_equal(full.pts, again.pts)


def test_synth_centroids_are_half_integers():
    """_detect truncates box corners to int and averages (process_pose.py:134-136)."""
    from bpc_baseline_amd.synth import make_scenes, make_capture
    b = make_scenes(3, 4, 50, seed=5)
    assert np.all(2 * b.pts == np.round(2 * b.pts))
    _, _, dets = make_capture(np.random.default_rng(0), 3, 5)
    for d in dets[0]:
        x1, y1, x2, y2 = d["bbox"]
        assert all(isinstance(v, int) for v in d["bbox"])
        assert d["bb_center"] == (0.5 * (x1 + x2), 0.5 * (y1 + y2))


def test_synth_true_matches_have_low_cost():
    """Sanity of the synthetic rig: real objects match below the reference's
    threshold of 30 px while clutter does not."""
    from bpc_baseline_amd.synth import make_scenes
    b = make_scenes(1, 3, 64, seed=8)
    _, am, mv, _, _ = O.cube(b.pts, b.cam_offs, b.F, 1)
    assert np.sum(mv < 30) >= 16
    assert np.median(mv) > 30


def test_shard_range_partitions():
    from bpc_baseline_amd.distributed import shard_range
    for n in (0, 1, 7, 10000, 10001):
        for w in (1, 2, 3, 8):
            parts = [shard_range(n, r, w) for r in range(w)]
            assert parts[0][0] == 0 and parts[-1][1] == n
            assert all(parts[i][1] == parts[i + 1][0] for i in range(w - 1))
            sizes = [b - a for a, b in parts]
            assert max(sizes) - min(sizes) <= 1


def test_ops_reject_cpu_tensors():
    """The matcher has no CPU path: host tensors are refused loudly."""
    from bpc_baseline_amd import ops
    plan = ops.PairwisePlan(np.array([0, 1, 2], np.int64), 1, 2, [[0, 1]], device="cpu")
    with pytest.raises(ValueError, match="GPU"):
        ops.pairwise_residual_argmin(torch.zeros(2, 2, dtype=torch.float64),
                                     torch.tensor([0, 1, 2]), torch.zeros(9, dtype=torch.float64),
                                     plan)


def test_pipeline_ops_reject_cpu_tensors():
    from bpc_baseline_amd import ops
    with pytest.raises(ValueError, match="GPU"):
        ops.pack_detections(torch.zeros(2, 4), torch.ones(2), torch.zeros(2),
                            torch.tensor([0, 2]), 0.1)
    with pytest.raises(ValueError, match="GPU"):
        ops.triangulate_dlt(torch.zeros(1, 3, 3, 4, dtype=torch.float64),
                            torch.zeros(1, 3, 2, dtype=torch.float64))


@pytest.mark.skipif(torch.cuda.is_available(), reason="checks the no-GPU failure mode")
def test_dropin_fails_loudly_without_gpu():
    from bpc_baseline_amd.inference import epipolar_matching as em
    with pytest.raises(RuntimeError, match="GPU"):
        em.epipolar_error((1.0, 2.0), (3.0, 4.0), np.eye(3))
    d = [{"bb_center": (1.0, 2.0), "bbox": (0, 0, 2, 4)}]
    with pytest.raises(RuntimeError, match="GPU"):
        em.compute_cost_matrix(d, d, d, np.eye(3), np.eye(3), np.eye(3))


def test_dropin_empty_view_returns_zero_cube():
    """N == 0 (or M, P): the reference loop never runs -> zeros((N, M, P)) float32.
    Needs no GPU (matches the reference exactly without launching)."""
    from bpc_baseline_amd.inference import epipolar_matching as em
    d = [{"bb_center": (1.0, 2.0), "bbox": (0, 0, 2, 4)}] * 3
    c = em.compute_cost_matrix([], d, d, np.eye(3), np.eye(3), np.eye(3))
    assert c.shape == (0, 3, 3) and c.dtype == np.float32
    c = em.compute_cost_matrix(d, d, [], np.eye(3), np.eye(3), np.eye(3))
    assert c.shape == (3, 3, 0)


def _half_for_f32_np(s):
    """numpy emulation of the kernel's half_for_f32 (mvm_kernels.hip)."""
    b = s.view(np.uint64)
    hi = (b >> np.uint64(32)).astype(np.int64)
    hi = np.maximum(hi - 0x00100000, 0).astype(np.uint64)
    return ((hi << np.uint64(32)) | (b & np.uint64(0xFFFFFFFF))).view(np.float64)


def test_exponent_halving_is_exact_after_f32_cast():
    """float32(half_for_f32(s)) == float32(0.5 * s) for every s >= +0 finite:
    random mantissas over all binades, every binade boundary, subnormals, 0."""
    rng = np.random.default_rng(0)
    exps = np.arange(-1074, 1024)
    mant = rng.uniform(1.0, 2.0, size=exps.size * 64)
    s = np.ldexp(mant, np.repeat(exps, 64))
    s = s[np.isfinite(s)]
    edges = np.ldexp(1.0, np.arange(-1074, 1023)).astype(np.float64)
    extra = np.concatenate([edges, np.nextafter(edges, 0), np.nextafter(edges, np.inf),
                            [0.0, 5e-324, 2.2250738585072014e-308, 4.450147717014403e-308,
                             np.finfo(np.float64).max / 4]])
    s = np.concatenate([s, extra]).astype(np.float64)
    with np.errstate(over="ignore", under="ignore"):
        want = (0.5 * s).astype(np.float32)
        got = _half_for_f32_np(s.copy()).astype(np.float32)
    assert np.array_equal(want.view(np.int32), got.view(np.int32))


def _third_fast_ok_np(q0):
    """numpy emulation of third_fast_ok (mvm_kernels.hip)."""
    b = q0.view(np.uint64)
    lo = (b & np.uint64(0xFFFFFFFF)).astype(np.uint32)
    hi = (b >> np.uint64(32)).astype(np.uint32)
    low29 = lo & np.uint32(0x1FFFFFFF)
    with np.errstate(over="ignore"):
        near = (low29 - np.uint32((1 << 28) - 3)) <= np.uint32(6)
        in_range = ((hi >> np.uint32(20)) - np.uint32(1023 - 126)) <= np.uint32(252)
    return ~near & in_range


def _third_fast_ok_spec(q0):
    """The rule as first written: |low 29 mantissa bits - 2^28| <= 3 is near a
    float32 midpoint; the exponent must put q0 in [2^-126, 2^127)."""
    b = q0.view(np.uint64)
    lo = (b & np.uint64(0xFFFFFFFF)).astype(np.int64)
    e = (b >> np.uint64(52)).astype(np.int64)              # sign + exponent
    near = np.abs((lo & 0x1FFFFFFF) - (1 << 28)) <= 3
    in_range = (e >= 1023 - 126) & (e <= 1023 + 126)
    return ~near & in_range


def test_third_fast_ok_bit_form_equals_spec():
    """The kernel's wrap-around form of the check equals the spec on random bit
    patterns, every low-29 value around 2^28 and the exponent window edges."""
    rng = np.random.default_rng(1)
    bits = rng.integers(0, 2 ** 63, 2_000_000, dtype=np.uint64)
    bits[::2] |= np.uint64(1) << np.uint64(63)                    # negatives too
    lows = np.arange((1 << 28) - 40, (1 << 28) + 40, dtype=np.uint64)
    exps = np.array([0, 1, 896, 897, 898, 1149, 1150, 1151, 2046, 2047], dtype=np.uint64)
    grid = (exps[:, None] << np.uint64(52)) | lows[None, :] | (np.uint64(0x5A5A5) << np.uint64(29))
    q0 = np.concatenate([bits, grid.reshape(-1), grid.reshape(-1) | (np.uint64(1) << np.uint64(63))])
    q0 = q0.view(np.float64)
    assert np.array_equal(_third_fast_ok_np(q0.copy()), _third_fast_ok_spec(q0.copy()))


def test_fast_division_by_three_rule():
    """The cube kernel's float32(RN(x/3)) shortcut: wherever third_fast_ok
    accepts q0 = x * RN(1/3), float32(q0) == float32(x / 3).  Random values over
    many binades plus adversarial x placed within +-3 ulps of 3 * (float32
    rounding midpoint)."""
    rng = np.random.default_rng(7)
    third = np.float64(1.0) / np.float64(3.0)
    x = np.concatenate([np.exp(rng.uniform(np.log(1e-40), np.log(1e40), 1_000_000)),
                        rng.uniform(0, 30000, 1_000_000), [0.0, 3.0, 9999.0, 29997.0]])
    f = rng.uniform(0.01, 5000, 200_000).astype(np.float32)
    mid = (f.astype(np.float64) + np.nextafter(f, np.float32(np.inf)).astype(np.float64)) / 2
    adv = mid * 3
    x = np.concatenate([x] + [adv + k * np.spacing(adv) for k in range(-3, 4)])
    q0 = x * third
    ok = _third_fast_ok_np(q0.copy())
    with np.errstate(over="ignore", under="ignore"):
        a = (x / 3.0).astype(np.float32).view(np.int32)
        b = q0.astype(np.float32).view(np.int32)
    assert not np.any((a != b) & ok)
    assert ok[1_000_000:2_000_000].mean() > 0.999   # realistic costs take the fast path


def _markstein_third(s: float) -> float:
    """third_q (mvm_kernels.hip) with exact fma emulation: q0 = RN(s * RN(1/3)),
    r = fma(-q0, 3, s), q1 = fma(r, RN(1/3), q0).  float(Fraction) and float
    '/' are correctly rounded in CPython, so each fma is one rounding."""
    from fractions import Fraction
    y = 1.0 / 3.0
    q0 = s * y
    r = float(Fraction(s) - 3 * Fraction(q0))
    return float(Fraction(r) * Fraction(y) + Fraction(q0))


def test_markstein_division_by_three_is_correctly_rounded():
    """The cube kernels' default RN(s / 3): one Markstein correction of the
    product equals the IEEE division bit for bit -- random values over every
    binade (subnormals included), binade edges, and s next to 3 * (midpoint
    of two consecutive doubles), where the plain product is most often off."""
    import struct
    rng = np.random.default_rng(21)
    xs = list(rng.integers(1, 0x7FEFFFFFFFFFFFFF, 6000, dtype=np.int64).view(np.float64))
    xs += list(rng.uniform(0, 30000, 6000)) + [0.0, 3.0, 9999.0, 29997.0, 5e-324, 1.7976931348623157e308]
    for e in range(-1074, 1024, 7):
        b = struct.unpack("<q", struct.pack("<d", math.ldexp(1.0, e)))[0]
        xs += [struct.unpack("<d", struct.pack("<q", b + d))[0] for d in (-1, 0, 1)]
    for _ in range(3000):
        e = int(rng.integers(-1000, 1000))
        k = (1 << 52) | int(rng.integers(0, 1 << 52))
        s0 = 3.0 * math.ldexp(float(k), e - 52) + math.ldexp(1.5, e - 52)
        b = struct.unpack("<q", struct.pack("<d", s0))[0]
        xs += [struct.unpack("<d", struct.pack("<q", b + d))[0] for d in range(-2, 3)]
    corrected = 0
    for s in xs:
        s = float(s)
        if not (s >= 0.0) or math.isinf(s):
            continue
        q1 = _markstein_third(s)
        assert q1 == s / 3.0 and math.copysign(1.0, q1) == 1.0, s
        corrected += (s * (1.0 / 3.0)) != s / 3.0
    assert corrected > 1000          # the plain product is off often enough to matter


def test_markstein_division_by_three_c_sweep(tmp_path):
    """tools/probes/third_markstein.c: the same identity on ~2e7 inputs with the
    C library's fma (skipped without a C compiler)."""
    import shutil
    import subprocess
    cc = shutil.which("gcc") or shutil.which("cc")
    if cc is None:
        pytest.skip("no C compiler")
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = str(tmp_path / "third_markstein")
    subprocess.run([cc, "-O2", "-ffp-contract=off", "-o", exe,
                    os.path.join(repo, "tools", "probes", "third_markstein.c"), "-lm"], check=True)
    r = subprocess.run([exe, "2000000"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and " 0 mismatches" in r.stdout, r.stdout


def test_batched_fundamental_matrices_bit_equal():
    """§8f #2: batched F == the per-pair restatement of compute_fundamental_matrix,
    bit for bit on this host (same numpy/BLAS kernels, matrix by matrix)."""
    from bpc_baseline_amd.synth import make_rig
    from bpc_baseline_amd.inference.utils.camera_utils import (
        camera_pairs, fundamental_matrices, fundamental_matrices_batched)
    rng = np.random.default_rng(3)
    rigs = [make_rig(rng, 4) for _ in range(50)]
    Ks = np.stack([np.stack(k) for k, _ in rigs])
    RTs = np.stack([np.stack(r) for _, r in rigs])
    pairs = camera_pairs(4)
    ref = np.concatenate([fundamental_matrices(list(k), list(r), pairs) for k, r in zip(Ks, RTs)])
    got = fundamental_matrices_batched(Ks, RTs, pairs)
    assert np.array_equal(ref.view(np.int64), got.view(np.int64))


def test_batched_fundamental_matrices_vs_reference(golden):
    from bpc_baseline_amd.inference.utils.camera_utils import fundamental_matrices_batched
    g = golden("a6_fundamental.npz")
    RT = np.zeros((len(g["R"]), 2, 4, 4))
    RT[..., :3, :3], RT[..., :3, 3], RT[..., 3, 3] = g["R"], g["t"], 1.0
    got = fundamental_matrices_batched(g["K"], RT, np.array([[0, 1]]))
    np.testing.assert_allclose(got.reshape(-1, 3, 3), g["F"], rtol=1e-12, atol=1e-18)


def test_capture_cameras_equals_per_capture(tmp_path, capsys):
    """Batched camera ingestion == Capture.from_dir's per-capture Ks / RTs."""
    import json
    from bpc_baseline_amd.inference.utils.camera_utils import (calc_pose_matrix, capture_cameras,
                                                                load_camera_params)
    rng = np.random.default_rng(4)
    cams = ["cam1", "cam2", "cam3"]
    for cam in cams:
        recs = {str(i): {"cam_K": rng.uniform(-2000, 4000, 9).tolist(),
                         "cam_R_w2c": rng.normal(size=9).tolist(),
                         "cam_t_w2c": rng.uniform(-2000, 2000, 3).tolist()} for i in range(7)}
        (tmp_path / f"scene_camera_{cam}.json").write_text(json.dumps(recs))
    params = load_camera_params(str(tmp_path), cams)
    assert "Loading camera parameters from:" in capsys.readouterr().out   # as the reference
    ids = [5, 0, 3]
    Ks, RTs = capture_cameras(str(tmp_path), cams, ids)
    for s, im in enumerate(ids):
        for c, cam in enumerate(cams):
            assert np.array_equal(Ks[s, c], params[cam]["K"][im]) and Ks.dtype == np.float32
            ref = calc_pose_matrix(params[cam]["R"][im], params[cam]["t"][im])
            assert np.array_equal(RTs[s, c], ref) and RTs.dtype == ref.dtype


def test_numpy_port_agrees_in_float32():
    """The vectorised NumPy restatement (bench.py's numpy CPU baseline) has no
    FMA, so only float32 agreement with the bit-exact C oracle is expected."""
    from bpc_baseline_amd.synth import make_scenes
    from oracle import numpy_port as NP
    from oracle import oracle as O
    b = make_scenes(4, 4, 120, seed=5)
    d, a = NP.pairwise(b.pts, b.cam_offs, b.F, b.pairs, 4, 4)
    rd, ra, _, _, _ = O.pairwise(b.pts, b.cam_offs, b.F, b.pairs, 4, 4)
    assert d.size == rd.size > 300000
    assert np.mean(d.view(np.int32) == rd.view(np.int32)) > 0.9999
    assert np.mean(a == ra) > 0.999


def test_reference_loop_restatement_is_bit_exact(golden):
    """oracle/reference_loop.py (the reference's per-pair NumPy cost model, timed
    by bench.py) reproduces the reference's own outputs bit for bit."""
    from oracle import reference_loop as RL
    z = golden("a1_epipolar_error.npz")
    got = np.array([RL.residual(z["p1"][k], z["p2"][k], np.asarray(z["F"][k]).reshape(3, 3))
                    for k in range(len(z["e"]))])
    assert np.array_equal(got.view(np.int64), np.asarray(z["e"], np.float64).view(np.int64))
    g = golden("a3_cost_cubes.npz")
    for n in ("c4", "c537", "degen", "dup"):
        F12, F13, F23 = (np.asarray(f, np.float64).reshape(3, 3) for f in g[f"{n}_F"])
        c = RL.cube(g[f"{n}_p1"], g[f"{n}_p2"], g[f"{n}_p3"], F12, F13, F23)
        assert np.array_equal(c.view(np.int32), g[f"{n}_cube"].view(np.int32)), n


@pytest.mark.parametrize("mode", ["static", "mixed", "distinct", "single"])
def test_rig_matrices_dedupe_bit_equal(mode):
    """match_captures' F/P: one evaluation per distinct rig, bit-equal to
    evaluating every capture (static rig, a few rigs, all distinct, S = 1)."""
    from bpc_baseline_amd.synth import make_rig
    from bpc_baseline_amd.inference.batch_match import projection_matrices, rig_matrices
    from bpc_baseline_amd.inference.utils.camera_utils import camera_pairs, fundamental_matrices_batched
    rng = np.random.default_rng(4)
    S = 1 if mode == "single" else 64
    rigs = [make_rig(rng, 3) for _ in range(S if mode == "distinct" else 3)]
    idx = {"static": np.zeros(S, int), "mixed": rng.integers(0, 3, S),
           "distinct": np.arange(S), "single": np.zeros(S, int)}[mode]
    Ks = np.stack([np.stack(rigs[i][0]) for i in idx]).astype(np.float32)
    RTs = np.stack([np.stack(rigs[i][1]) for i in idx]).astype(np.float64)
    F, P = rig_matrices(Ks, RTs)
    assert np.array_equal(F.view(np.int64), fundamental_matrices_batched(Ks, RTs, camera_pairs(3)).view(np.int64))
    assert np.array_equal(P.view(np.int64), projection_matrices(Ks, RTs).view(np.int64))


def test_bench_output_slots():
    """bench.py gives each launch of the timed steps its own output allocation
    as far as HBM holds them with 8 GiB to spare, never fewer than one."""
    import bench
    gib = 1 << 30
    assert bench.output_slots(10 * 20, 25 * gib, 287 * gib) == 11   # C3 on one MI355X
    assert bench.output_slots(10, 25 * gib, 150 * gib) == 5
    assert bench.output_slots(10, 25 * gib, 20 * gib) == 1
    assert bench.output_slots(4 * 20, 17 * gib, 287 * gib) == 16    # the C2 cube
    assert bench.output_slots(20, gib, 287 * gib) == 20             # C2: one per step
    assert bench.output_slots(1, gib, 287 * gib) == 1


def test_bench_launch_split():
    """Launches of at most --chunk scenes, at least --min-launches of them,
    sizes within one scene: configs[3] (1,250 scenes per rank) runs 5 x 250,
    so only a fifth of a step's association gather is left unoverlapped."""
    import bench

    def sizes(n, c, m):
        b = bench.launch_bounds(n, c, m)
        assert b[0][0] == 0 and b[-1][1] == n
        assert all(b[k][1] == b[k + 1][0] for k in range(len(b) - 1))
        return [s1 - s0 for s0, s1 in b]

    assert sizes(10000, 1000, 1) == [1000] * 10     # C3, one GPU
    assert sizes(1250, 1000, 5) == [250] * 5         # configs[3]
    assert sizes(5000, 1000, 5) == [1000] * 5        # two GPUs
    assert sizes(2500, 1000, 5) == [500] * 5         # four GPUs
    assert sizes(1000, 1000, 1) == [1000]            # C2
    assert sizes(3, 1000, 5) == [1, 1, 1]            # fewer scenes than launches
    assert sizes(12, 8, 5) == [3, 3, 2, 2, 2]
    # N > 1: a short last launch (its gather piece is the one left exposed)
    def tapered(n, c, m):
        b = bench.launch_bounds(n, c, m, 0.25)
        assert b[0][0] == 0 and b[-1][1] == n
        assert all(b[k][1] == b[k + 1][0] for k in range(len(b) - 1))
        return [s1 - s0 for s0, s1 in b]
    assert tapered(1250, 1000, 5) == [238, 238, 238, 237, 237, 62]   # configs[3]
    assert tapered(5000, 1000, 5) == [950] * 5 + [250]                # two GPUs
    assert tapered(3, 1000, 5) == [1, 1, 1]                           # one scene per launch
    assert tapered(6, 1000, 5) == [1, 1, 1, 1, 1, 1]
    assert max(tapered(10000, 1000, 5)) <= 1000
    for n, c, m in ((1250, 1000, 8), (7, 2, 3), (10001, 1000, 5), (1, 1, 1)):
        z = sizes(n, c, m)
        assert max(z) <= c and max(z) - min(z) <= 1 and len(z) >= min(m, n)


def test_bench_rejects_fewer_scenes_than_ranks(monkeypatch):
    """Strong scaling with fewer scenes than ranks would leave a rank with no
    launch while the others wait in its collectives: bench.py refuses it."""
    import sys
    import bench
    from bpc_baseline_amd import distributed

    class Env:
        rank, world, local_rank, initialised, backend = 0, 8, 0, False, None
        device = "cpu"

    monkeypatch.setattr(bench, "init_from_env", lambda: Env())
    monkeypatch.setenv("WORLD_SIZE", "8")      # as a rank of an 8-rank launch
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "8", "--scenes", "4"])
    with pytest.raises(SystemExit, match="every rank needs at least one scene"):
        bench.main()
    assert distributed.shard_range(4, 7, 8) == (4, 4)


def test_capture_session_cache_bounds(monkeypatch):
    """The drop-in's slot cache: capacity classes (next power of two, >= 8),
    LRU eviction by count AND bytes, a slot above the byte cap used uncached,
    and clear() releasing the thread's slots (no unbounded pinned /
    device memory in a long-lived service)."""
    from bpc_baseline_amd.inference import capture_session as cs
    assert [cs._cap(n) for n in (0, 1, 8, 9, 24, 64, 65)] == [8, 8, 8, 16, 32, 64, 128]

    class Fake:
        def __init__(self, nbytes):
            self.nbytes = nbytes

    cs.clear()
    monkeypatch.setattr(cs, "_MAX_BYTES", 1000)
    monkeypatch.setattr(cs, "_MAX_SLOTS", 3)
    for k in range(5):                                   # count bound
        cs._lookup("cube", ("c", k), lambda: Fake(10))
    assert cs.cache_info()["cube"] == {"slots": 3, "bytes": 30}
    assert ("c", 4) in cs._cache("cube") and ("c", 0) not in cs._cache("cube")
    a = cs._lookup("cube", ("c", 2), lambda: Fake(10))  # a hit moves to the end
    assert list(cs._cache("cube"))[-1] == ("c", 2) and a is cs._cache("cube")[("c", 2)]
    cs._lookup("cube", ("big", 0), lambda: Fake(980))   # byte bound evicts the oldest
    assert cs.cache_info()["cube"]["bytes"] <= 1000
    huge = cs._lookup("cube", ("huge", 0), lambda: Fake(5000))
    assert huge.nbytes == 5000 and ("huge", 0) not in cs._cache("cube")
    cs.clear()
    assert cs.cache_info() == {"cube": {"slots": 0, "bytes": 0}, "lsap": {"slots": 0, "bytes": 0}}


def test_rig_workers_equal_rig_matrices():
    """F and P computed by the worker processes (shared memory, slices of the
    batch per worker) equal rig_matrices in the calling process bit for bit:
    a static rig, mixed rigs, all distinct, a batch larger than the slots
    (the slot grows), an empty batch, and submit-before-collect pipelining."""
    from bpc_baseline_amd.synth import make_rig
    from bpc_baseline_amd.inference.rig_workers import RigWorkers
    from bpc_baseline_amd.inference.utils.camera_utils import rig_matrices
    rng = np.random.default_rng(12)

    def batch(S, n_rigs):
        rigs = [make_rig(rng, 3) for _ in range(n_rigs)]
        idx = rng.integers(0, n_rigs, S)
        Ks = np.stack([np.stack(rigs[i][0]) for i in idx]).astype(np.float32)
        RTs = np.stack([np.stack(rigs[i][1]) for i in idx]).astype(np.float64)
        return Ks, RTs

    empty = (np.zeros((0, 3, 3, 3), np.float32), np.zeros((0, 3, 4, 4), np.float64))
    batches = [batch(40, 1), batch(64, 5), batch(300, 300), batch(7, 7), empty]
    with RigWorkers(3) as rw:
        rw.submit(*batches[0])
        for k, (Ks, RTs) in enumerate(batches):
            F, P = rw.result()
            if k + 1 < len(batches):
                rw.submit(*batches[k + 1])
            if Ks.shape[0] == 0:
                assert F.shape == (0, 9) and P.shape == (0, 3, 3, 4)
                continue
            Fr, Pr = rig_matrices(Ks, RTs)
            assert np.array_equal(F.view(np.int64), Fr.view(np.int64)), k
            assert np.array_equal(P.view(np.int64), Pr.view(np.int64)), k


def test_lsap_slot_capacity_covers_every_shape():
    """A capacity-class assignment slot's workspace covers every shape of its
    class, tall (transposed copy) and wide alike (mvm_lsap_plan_ex sizes)."""
    import ctypes
    from bpc_baseline_amd import _native
    lib = _native.load()

    def plan(r, c):
        ws = np.zeros(2, np.int64)
        out = np.zeros(2, np.int64)
        ra, ca = np.array([r], np.int64), np.array([c], np.int64)
        return lib.mvm_lsap_plan_ex(1, ra.ctypes.data, ca.ctypes.data, _native.MVM_F32,
                                    ws.ctypes.data, out.ctypes.data)

    for rcap, ccap in ((8, 8), (64, 8), (8, 64), (512, 64), (16, 16)):
        cap = max(plan(min(rcap, ccap), ccap), plan(rcap, min(ccap, rcap - 1)) if rcap > 1 else 0)
        worst = max(plan(r, c) for r in range(1, rcap + 1) for c in range(1, ccap + 1))
        assert worst <= cap, (rcap, ccap, worst, cap)


def test_rig_workers_tickets_and_drain():
    """A result() with another job's ticket raises; drain() collects a job in
    flight so the pool takes the next submit."""
    from bpc_baseline_amd.synth import make_rig
    from bpc_baseline_amd.inference.rig_workers import RigWorkers
    from bpc_baseline_amd.inference.utils.camera_utils import rig_matrices
    rng = np.random.default_rng(3)
    Ks, RTs = make_rig(rng, 3)
    Ks = np.stack([np.stack(Ks)] * 4).astype(np.float32)
    RTs = np.stack([np.stack(RTs)] * 4)
    with RigWorkers(2) as rw:
        t1 = rw.submit(Ks, RTs)
        with pytest.raises(RuntimeError, match="collect the previous result first"):
            rw.submit(Ks, RTs)
        with pytest.raises(RuntimeError, match="not the one in flight"):
            rw.result(t1 + 1)
        rw.drain()                                  # the abandoned job
        t2 = rw.submit(Ks, RTs)
        F, P = rw.result(t2)
        Fr, _ = rig_matrices(Ks, RTs)
        assert np.array_equal(F.view(np.int64), Fr.view(np.int64))
        rw.drain()                                  # nothing in flight: no-op


def test_capture_stream_abandoned_then_reused(monkeypatch):
    """A consumer that breaks out of match_capture_stream leaves the next
    batch's F/P job in flight; the stream collects it, so a second stream on
    the same thread's pool runs (batch_match.py:204).  Threads get
    their own pools.  match_captures is replaced by a host stand-in that
    returns the F it was given (the device chain is covered by -m gpu)."""
    import threading
    import torch
    from bpc_baseline_amd.inference import batch_match as bm
    from bpc_baseline_amd.synth import make_rig
    from bpc_baseline_amd.inference.utils.camera_utils import rig_matrices
    monkeypatch.setattr(bm, "match_captures", lambda *a, F=None, proj=None, **k: F)
    rng = np.random.default_rng(9)

    def batch(S):
        rigs = [make_rig(rng, 3) for _ in range(S)]
        Ks = np.stack([np.stack(r[0]) for r in rigs]).astype(np.float32)
        RTs = np.stack([np.stack(r[1]) for r in rigs])
        return (torch.zeros(1), None, None, torch.zeros(3 * S + 1, dtype=torch.int64), Ks, RTs)

    batches = [batch(5), batch(6), batch(7)]
    for F in bm.match_capture_stream(batches, rig_workers=2):
        break                                       # batch 1's job is in flight here
    got = list(bm.match_capture_stream(batches, rig_workers=2))
    for b, F in zip(batches, got):
        assert np.array_equal(F.numpy().view(np.int64), rig_matrices(b[4], b[5])[0].view(np.int64))
    with pytest.raises(ZeroDivisionError):
        for F in bm.match_capture_stream(batches, rig_workers=2):
            1 / 0                                   # an exception in the consumer
    assert len(list(bm.match_capture_stream(batches, rig_workers=2))) == 3
    # another thread gets its own pool, and the pool is closed when that
    # thread ends (no worker processes left behind per thread)
    seen = []

    def other():
        p = bm.rig_worker_pool(2)
        seen.append((p, list(p.procs)))
    th = threading.Thread(target=other)
    th.start()
    th.join()
    import gc
    gc.collect()
    pool, procs = seen[0]
    assert pool is not bm.rig_worker_pool(2)
    assert not pool.procs and all(pr.poll() is not None for pr in procs)
