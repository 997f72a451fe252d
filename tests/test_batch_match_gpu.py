"""Batched device pipeline (pack -> cube -> assignment -> select + DLT) equals
the reference's per-capture _detect/_match/PosePrediction outputs."""
import numpy as np
import pytest
import torch

from oracle import lsap, pipeline
from oracle import oracle as cube_oracle

pytestmark = pytest.mark.gpu
DLT_RTOL, DLT_ATOL = 1e-10, 1e-9


def _run(cuda, per_image, Ks, RTs, **kw):
    from bpc_baseline_amd.inference.batch_match import match_captures
    boxes = np.concatenate([b for b, _, _ in per_image]).astype(np.float32).reshape(-1, 4)
    conf = np.concatenate([c for _, c, _ in per_image]).astype(np.float32)
    cls = np.concatenate([k for _, _, k in per_image]).astype(np.float32)
    offs = np.zeros(len(per_image) + 1, np.int64)
    np.cumsum([b.shape[0] for b, _, _ in per_image], out=offs[1:])
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(cuda)
    return match_captures(t(boxes), t(conf), t(cls), t(offs), Ks, RTs, **kw), (boxes, conf, cls, offs)


def test_batch_equals_reference_match(cuda, golden):
    """All a7 captures (incl. one with an empty view) in one batch."""
    z = golden("a7_match.npz")
    n = int(z["n"])
    per_image, Ks, RTs = [], [], []
    for c in range(n):
        for cam in range(3):
            b = z[f"m{c}_boxes{cam}"]
            per_image.append((b, np.ones(len(b)), np.zeros(len(b))))
        Ks.append(z[f"m{c}_K"])
        RTs.append(z[f"m{c}_RT"])
    res, _ = _run(cuda, per_image, np.stack(Ks), np.stack(RTs))
    for c in range(n):
        preds = res.predictions(c)
        assert len(preds) == z[f"m{c}_t"].shape[0]
        for q, (bx, cent, t) in enumerate(preds):
            np.testing.assert_array_equal(bx, z[f"m{c}_boxes"][q])
            np.testing.assert_array_equal(cent, z[f"m{c}_centroids"][q])
            np.testing.assert_allclose(t, z[f"m{c}_t"][q], rtol=DLT_RTOL, atol=DLT_ATOL)


def _oracle_capture(boxes, conf, cls, offs, K, RT, conf_thresh, thr):
    """Per-capture chain on the CPU restatements: _detect packing, F, cube,
    scipy-identical assignment, threshold, stable sort, DLT."""
    from bpc_baseline_amd.inference.utils.camera_utils import camera_pairs, fundamental_matrices
    bbox, cent, o = pipeline.detect_pack(boxes, conf, cls, offs, conf_thresh)
    F = fundamental_matrices(list(K), list(RT), camera_pairs(3))
    counts = np.diff(o)
    if np.any(counts == 0):
        return []
    cube = cube_oracle.cube(cent, o, F, 1)[0].reshape(counts)
    matches = lsap.match_objects(cube, thr)
    matches = sorted(matches, key=lambda m: cube[m])
    P = np.stack([K[v] @ RT[v][:3] for v in range(3)])
    out = []
    for i, j, k in matches:
        rows = o[:3] + np.array([i, j, k])
        X = pipeline.triangulate(P[None], cent[rows][None])[0]
        out.append((bbox[rows], cent[rows], X))
    return out


@pytest.mark.parametrize("sizes", ["ipd", "large", "c2"])
def test_batch_vs_oracle_synthetic(cuda, sizes):
    """ipd: views of 0-40 detections (the small cube kernel, the one-wave
    assignment); large: 0-100 (the tiled cube kernels -- with empty views
    among them -- and the wider assignment classes, the candidate-list one
    with the 8-row minima read back from the cube); c2: 130-256 (the fused
    kernel writing the 8-row minima, the candidate-list assignment reducing
    them)."""
    from bpc_baseline_amd.synth import make_capture
    rng = np.random.default_rng({"ipd": 11, "large": 12, "c2": 13}[sizes])
    S = {"ipd": 120, "large": 30, "c2": 5}[sizes]
    choices, probs = {"ipd": ([0, 1, 2, 6, 12, 24, 40], [.04, .06, .1, .3, .3, .1, .1]),
                      "large": ([0, 1, 24, 45, 64, 100], [.1, .05, .15, .25, .25, .2]),
                      "c2": ([130, 160, 200, 256], [.25, .25, .25, .25])}[sizes]
    per_image, Ks, RTs = [], [], []
    for s in range(S):
        counts = list(rng.choice(choices, 3, p=probs))
        K, RT, dets = make_capture(rng, 3, counts, duplicates=int(s % 7 == 0))
        for cam in range(3):
            b = np.asarray([d["bbox"] for d in dets[cam]], np.float64).reshape(-1, 4)
            b = b + rng.uniform(0, 0.999, b.shape)              # fractional parts: int() truncates
            conf = rng.uniform(0.2, 1.0, len(b))
            cls = np.zeros(len(b))
            # detector clutter the filter must drop
            nj = int(rng.integers(0, 4))
            jb = rng.uniform(0, 2000, (nj, 4))
            jc = np.where(rng.random(nj) < 0.5, rng.uniform(0, 0.09, nj), 0.9)
            jk = np.where(jc > 0.5, 1.0, 0.0)
            per = rng.permutation(len(b) + nj)
            per_image.append((np.concatenate([b, jb])[per], np.concatenate([conf, jc])[per],
                              np.concatenate([cls, jk])[per]))
        Ks.append(np.stack(K))
        RTs.append(np.stack(RT))
    Ks, RTs = np.stack(Ks), np.stack(RTs)
    res, (boxes, conf, cls, offs) = _run(cuda, per_image, Ks, RTs, conf_thresh=0.1,
                                         matching_threshold=30)
    total = 0
    for s in range(S):
        o = offs[3 * s:3 * s + 4]
        ref = _oracle_capture(boxes[o[0]:o[3]], conf[o[0]:o[3]], cls[o[0]:o[3]], o - o[0],
                              Ks[s], RTs[s], 0.1, 30)
        got = res.predictions(s)
        assert len(got) == len(ref), s
        for (gb, gc, gt), (rb, rc, rt) in zip(got, ref):
            np.testing.assert_array_equal(gb, rb)
            np.testing.assert_array_equal(gc, rc)
            np.testing.assert_allclose(gt, rt, rtol=DLT_RTOL, atol=DLT_ATOL)
        total += len(ref)
    assert total > 2 * S     # the synthetic objects are actually recovered
    if sizes != "ipd":
        return
    # a static rig: F and P passed in give the same results
    from bpc_baseline_amd.inference.batch_match import match_captures, projection_matrices
    from bpc_baseline_amd.inference.utils.camera_utils import camera_pairs, fundamental_matrices_batched
    Fd = torch.from_numpy(fundamental_matrices_batched(Ks, RTs, camera_pairs(3))).to(cuda)
    Pd = torch.from_numpy(projection_matrices(Ks, RTs)).to(cuda)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(cuda)
    res2 = match_captures(t(boxes), t(conf), t(cls), t(offs), Ks, RTs, F=Fd, proj=Pd)
    assert np.array_equal(res2.count, res.count)
    for s in range(S):       # rows past count[s] are unused capacity
        o, k = int(res.offs[s]), int(res.count[s])
        assert torch.equal(res2.match[o:o + k], res.match[o:o + k])
        assert torch.equal(res2.X[o:o + k], res.X[o:o + k])


def test_capture_stream_equals_per_batch(cuda):
    """match_capture_stream (host F/P of batch b+1 on a worker thread) gives
    each batch exactly what match_captures gives it; an empty stream yields
    nothing."""
    from bpc_baseline_amd.inference.batch_match import match_capture_stream, match_captures
    from bpc_baseline_amd.synth import make_detector_batch
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(cuda)
    batches = []
    for seed, (S, n) in enumerate(((40, 12), (7, 30), (25, 5))):
        b = make_detector_batch(S, n, seed=seed)
        batches.append((t(b.boxes), t(b.conf), t(b.cls), t(b.img_offs), b.Ks, b.RTs))
    got = list(match_capture_stream(iter(batches), matching_threshold=30))
    assert len(got) == len(batches)
    for bt, r in zip(batches, got):
        ref = match_captures(*bt, matching_threshold=30)
        assert np.array_equal(r.count, ref.count) and np.array_equal(r.offs, ref.offs)
        for s in range(len(r.count)):
            o, k = int(r.offs[s]), int(r.count[s])
            assert torch.equal(r.match[o:o + k], ref.match[o:o + k])
            assert torch.equal(r.X[o:o + k], ref.X[o:o + k])
    assert list(match_capture_stream([])) == []
    with pytest.raises(TypeError):
        next(match_capture_stream(batches, F=None))


def test_batch_threshold_inf_and_empty(cuda, golden):
    """threshold=inf keeps every assignment; an all-empty batch is a no-op."""
    z = golden("a3_cost_cubes.npz")
    name = "c24"
    per_image = []
    for v in (1, 2, 3):
        q = z[f"{name}_p{v}"]
        x1, y1 = np.floor(q[:, 0]) - 3.0, np.floor(q[:, 1]) - 2.0
        b = np.stack([x1, y1, 2.0 * q[:, 0] - x1, 2.0 * q[:, 1] - y1], 1)
        per_image.append((b, np.ones(len(b)), np.zeros(len(b))))
    # the pipeline derives F from the rig, so check the selection against
    # match_objects on the cube the pipeline itself built
    from bpc_baseline_amd.synth import make_rig
    K, RT = make_rig(np.random.default_rng(5), 3)
    res, _ = _run(cuda, per_image, np.stack(K)[None], np.stack(RT)[None],
                  matching_threshold=np.inf, keep_cube=True)
    cube = res.cube.cpu().numpy().reshape(24, 24, 24)
    ref = sorted(lsap.match_objects(cube, np.inf), key=lambda m: cube[m])
    got = res.match[:int(res.count[0])].cpu().numpy()
    np.testing.assert_array_equal(got, np.asarray(ref).reshape(-1, 3))
    empty = [(np.zeros((0, 4)), np.zeros(0), np.zeros(0))] * 6
    res, _ = _run(cuda, empty, np.stack([np.stack(K)] * 2), np.stack([np.stack(RT)] * 2))
    assert list(res.count) == [0, 0]
