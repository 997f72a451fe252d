"""Pin the CPU restatement of _detect's packing and of triangulate_multi_view
(oracle/pipeline.py) against the reference's own outputs (a8, a9 fixtures)."""
import numpy as np

from oracle import pipeline


def test_detect_pack_matches_reference(golden):
    z = golden("a8_detect.npz")
    for c in range(int(z["n"])):
        bbox, center, offs = pipeline.detect_pack(z[f"d{c}_boxes"], z[f"d{c}_conf"], z[f"d{c}_cls"],
                                                  z[f"d{c}_in_offs"], float(z[f"d{c}_thresh"]))
        np.testing.assert_array_equal(offs, z[f"d{c}_out_offs"])
        np.testing.assert_array_equal(bbox, z[f"d{c}_bbox"])
        assert center.dtype == np.float64
        np.testing.assert_array_equal(center, z[f"d{c}_center"])


def test_detect_fixture_covers_edges(golden):
    """The fixture exercises what the kernel must get right: confidences equal
    to the float32 threshold and one ulp below, negative fractional coordinates
    (int() truncates toward zero), empty images, foreign classes."""
    z = golden("a8_detect.npz")
    seen_eq = seen_below = seen_neg = seen_empty = seen_cls = False
    for c in range(int(z["n"])):
        t32 = np.float32(float(z[f"d{c}_thresh"]))
        conf, boxes, cls = z[f"d{c}_conf"], z[f"d{c}_boxes"], z[f"d{c}_cls"]
        seen_eq |= bool(np.any(conf == t32))
        seen_below |= bool(np.any(conf == np.nextafter(t32, np.float32(-1))))
        seen_neg |= bool(np.any((boxes < 0) & (boxes > -1)))
        seen_empty |= bool(np.any(np.diff(z[f"d{c}_in_offs"]) == 0))
        seen_cls |= bool(np.any(cls != 0))
    assert seen_eq and seen_below and seen_neg and seen_empty and seen_cls


def test_triangulate_matches_reference(golden):
    z = golden("a9_triangulate.npz")
    for V in (2, 3, 4, 8):
        X = pipeline.triangulate(z[f"v{V}_proj"], z[f"v{V}_pts"])
        np.testing.assert_allclose(X, z[f"v{V}_X"], rtol=1e-12, atol=1e-9)


def test_triangulate_matches_match_fixture(golden):
    """PosePrediction.t of the reference's _match runs (a7)."""
    z = golden("a7_match.npz")
    for c in range(int(z["n"])):
        cent = z[f"m{c}_centroids"]
        if cent.shape[0] == 0:
            continue
        P = np.stack([z[f"m{c}_K"][v] @ z[f"m{c}_RT"][v][:3] for v in range(3)])
        proj = np.broadcast_to(P, (cent.shape[0], 3, 3, 4))
        X = pipeline.triangulate(proj, cent)
        np.testing.assert_allclose(X, z[f"m{c}_t"], rtol=1e-12, atol=1e-9)
