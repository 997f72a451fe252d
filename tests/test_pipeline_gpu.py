"""On-device detection packing (mvm_pack_detections) and batched DLT
(mvm_triangulate_dlt) against the reference's outputs (a7/a8/a9 fixtures) and
the CPU restatement (oracle/pipeline.py) at batch sizes."""
import numpy as np
import pytest
import torch

from oracle import pipeline

pytestmark = pytest.mark.gpu

# Jacobi vs LAPACK: both backward stable; the smallest right singular vector
# agrees to ~1e-12 relative on these systems (oracle emulation: <= 8e-13)
DLT_RTOL, DLT_ATOL = 1e-10, 1e-9


def _pack(cuda, boxes, conf, cls, in_offs, thresh):
    from bpc_baseline_amd import ops
    t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a, dt)).to(cuda)
    pts, offs, bbox, counts, status = ops.pack_detections(
        t(np.asarray(boxes).reshape(-1, 4), np.float32), t(conf, np.float32), t(cls, np.float32),
        t(in_offs, np.int64), thresh)
    offs = offs.cpu().numpy()
    n = int(offs[-1])
    return pts[:n].cpu().numpy(), bbox[:n].cpu().numpy(), offs, counts.cpu().numpy(), int(status.item())


def test_pack_matches_reference_detect(cuda, golden):
    z = golden("a8_detect.npz")
    for c in range(int(z["n"])):
        pts, bbox, offs, counts, st = _pack(cuda, z[f"d{c}_boxes"], z[f"d{c}_conf"], z[f"d{c}_cls"],
                                            z[f"d{c}_in_offs"], float(z[f"d{c}_thresh"]))
        assert st == 0
        np.testing.assert_array_equal(offs, z[f"d{c}_out_offs"])
        np.testing.assert_array_equal(counts, np.diff(z[f"d{c}_out_offs"]))
        np.testing.assert_array_equal(bbox, z[f"d{c}_bbox"])
        np.testing.assert_array_equal(pts, z[f"d{c}_center"])


def test_pack_batch_vs_oracle(cuda):
    rng = np.random.default_rng(7)
    n_img = 30000
    counts = rng.choice([0, 1, 5, 63, 64, 65, 255, 256, 257, 600], n_img,
                        p=[.1, .2, .3, .1, .05, .05, .05, .05, .05, .05])
    in_offs = np.zeros(n_img + 1, np.int64)
    np.cumsum(counts, out=in_offs[1:])
    n = int(in_offs[-1])
    boxes = rng.uniform(-5, 4000, (n, 4)).astype(np.float32)
    boxes[rng.random((n, 4)) < 0.1] = np.float32(-0.5)
    conf = rng.random(n).astype(np.float32)
    conf[rng.random(n) < 0.05] = np.float32(0.3)
    cls = rng.integers(0, 3, n).astype(np.float32)
    pts, bbox, offs, cnt, st = _pack(cuda, boxes, conf, cls, in_offs, 0.3)
    rb, rc, ro = pipeline.detect_pack(boxes, conf, cls, in_offs, 0.3)
    assert st == 0
    np.testing.assert_array_equal(offs, ro)
    np.testing.assert_array_equal(bbox, rb)
    np.testing.assert_array_equal(pts, rc)


def test_pack_empty_and_bad_boxes(cuda):
    pts, bbox, offs, cnt, st = _pack(cuda, np.zeros((0, 4)), np.zeros(0), np.zeros(0),
                                     np.zeros(4, np.int64), 0.1)
    assert st == 0 and list(offs) == [0, 0, 0, 0] and pts.shape == (0, 2)
    boxes = np.array([[1, 2, 3, 4], [np.nan, 0, 1, 1], [0, 0, 3e9, 1], [np.inf, 0, 0, 0]], np.float32)
    conf = np.array([0.9, 0.9, 0.9, 0.01], np.float32)
    _, bbox, offs, _, st = _pack(cuda, boxes, conf, np.zeros(4), np.array([0, 4]), 0.1)
    assert st == 1 and int(offs[-1]) == 3          # the low-confidence inf box is dropped
    np.testing.assert_array_equal(bbox[0], [1, 2, 3, 4])


def test_pack_feeds_matcher(cuda, golden):
    """Packed centres are the matcher's CSR input: the cube built from them
    equals the reference's cube built from _detect's dicts (a3 inputs)."""
    from bpc_baseline_amd import ops
    z = golden("a3_cost_cubes.npz")
    name = "c16"
    p = [z[f"{name}_p{v}"] for v in (1, 2, 3)]
    # rebuild integer boxes whose centre is the stored half-integer centre
    def box(q):
        x1, y1 = np.floor(q[:, 0]) - 3.0, np.floor(q[:, 1]) - 2.0
        return np.stack([x1, y1, 2.0 * q[:, 0] - x1, 2.0 * q[:, 1] - y1], 1)
    boxes = np.concatenate([box(q) for q in p]).astype(np.float32)
    in_offs = np.array([0, len(p[0]), len(p[0]) + len(p[1]), sum(len(q) for q in p)], np.int64)
    assert np.all(np.abs(boxes - np.trunc(boxes)) == 0)
    n = boxes.shape[0]
    pts, offs, _, counts, st = ops.pack_detections(
        torch.from_numpy(boxes).to(cuda), torch.ones(n, device=cuda), torch.zeros(n, device=cuda),
        torch.from_numpy(in_offs).to(cuda), 0.1)
    np.testing.assert_array_equal(pts.cpu().numpy(), np.concatenate(p))
    plan = ops.TripletPlan(offs.cpu().numpy(), 1, device=cuda)
    F = torch.from_numpy(np.ascontiguousarray(z[f"{name}_F"], np.float64).reshape(-1)).to(cuda)
    cube, argmin, _ = ops.triplet_cost_argmin(pts, offs, F, plan)
    np.testing.assert_array_equal(cube.cpu().numpy().reshape(z[f"{name}_cube"].shape), z[f"{name}_cube"])


def _dlt(cuda, proj, pts, set_of_point=None):
    from bpc_baseline_amd import ops
    sp = None if set_of_point is None else torch.from_numpy(set_of_point.astype(np.int32)).to(cuda)
    return ops.triangulate_dlt(torch.from_numpy(np.ascontiguousarray(proj)).to(cuda),
                               torch.from_numpy(np.ascontiguousarray(pts)).to(cuda), sp).cpu().numpy()


def test_dlt_matches_reference(cuda, golden):
    z = golden("a9_triangulate.npz")
    for V in (2, 3, 4, 8):
        X = _dlt(cuda, z[f"v{V}_proj"], z[f"v{V}_pts"])
        np.testing.assert_allclose(X, z[f"v{V}_X"], rtol=DLT_RTOL, atol=DLT_ATOL)


def test_dlt_matches_pose_predictions(cuda, golden):
    z = golden("a7_match.npz")
    for c in range(int(z["n"])):
        cent = z[f"m{c}_centroids"]
        if cent.shape[0] == 0:
            continue
        P = np.stack([z[f"m{c}_K"][v] @ z[f"m{c}_RT"][v][:3] for v in range(3)])[None]
        X = _dlt(cuda, P, cent, np.zeros(cent.shape[0]))
        np.testing.assert_allclose(X, z[f"m{c}_t"], rtol=DLT_RTOL, atol=DLT_ATOL)


def test_dlt_batch_vs_oracle(cuda):
    from bpc_baseline_amd.synth import make_rig
    rng = np.random.default_rng(3)
    n_sets, n = 50, 20000
    P = np.empty((n_sets, 3, 3, 4))
    for s in range(n_sets):
        Ks, RTs = make_rig(rng, 3)
        P[s] = np.stack([Ks[v] @ RTs[v][:3] for v in range(3)])
    set_of_point = rng.integers(0, n_sets, n)
    Xw = np.concatenate([rng.uniform(-250, 250, (n, 2)), rng.uniform(-80, 80, (n, 1)), np.ones((n, 1))], 1)
    uvw = np.einsum("nvij,nj->nvi", P[set_of_point], Xw)
    uv = np.round(2 * (uvw[..., :2] / uvw[..., 2:3] + rng.normal(0, 1.5, (n, 3, 2)))) / 2
    X = _dlt(cuda, P, uv, set_of_point)
    sample = rng.choice(n, 2000, replace=False)
    ref = pipeline.triangulate(P[set_of_point[sample]], uv[sample])
    np.testing.assert_allclose(X[sample], ref, rtol=DLT_RTOL, atol=DLT_ATOL)
    # and the triangulated points are near the true ones (noise ~1.5 px)
    assert np.median(np.abs(X - Xw[:, :3])) < 5.0


def test_dlt_rejects_bad_views(cuda):
    from bpc_baseline_amd import ops
    from bpc_baseline_amd._native import MvmError
    with pytest.raises((MvmError, ValueError)):
        ops.triangulate_dlt(torch.zeros((1, 1, 3, 4), dtype=torch.float64, device=cuda),
                            torch.zeros((1, 1, 2), dtype=torch.float64, device=cuda))
