"""Matching stage of ``bpc/inference/process_pose.py`` on the MI355X matcher.

Mirrors the part of the reference's pose pipeline that the hot path serves:

* ``PoseEstimatorParams`` (process_pose.py:32-38) -- same fields/defaults;
* ``PosePrediction`` (process_pose.py:79-94) -- same attributes; DLT
  triangulation of the matched centroids;
* ``match_detections(capture, detections, params)`` -- the body of
  ``PoseEstimator._match`` (process_pose.py:144-188): F12/F13/F23 on the
  host, the empty-view guard, the cost cube on the GPU, the same stats and
  five random samples printed from the GLOBAL ``np.random`` (so the caller's
  RNG stream advances exactly as with the reference), Hungarian matching
  with ``matching_threshold``, stable sort by cost;
* ``detect_capture`` / ``MatcherMixin._detect`` -- ``PoseEstimator._detect``
  (process_pose.py:116-142) with the box filtering, int truncation and
  centres done on the GPU (``mvm_pack_detections``); returns the same
  ``{idx: [{'bbox', 'bb_center'}, ...]}`` mapping, which also carries the
  packed device centroids so ``_match`` skips the host -> device copy;
* ``MatcherMixin._match`` -- a drop-in method for ``PoseEstimator``;
* ``install_into_reference()`` -- rebinds the reference modules' names to
  this implementation (the reference binds them at import time,
  process_pose.py:24-26), so the Inference Notebook runs unchanged.

The YOLO network itself, the ResNet rotation head and image I/O stay in the
reference (out of scope: SURVEY §2).
"""
from __future__ import annotations

import sys
from dataclasses import dataclass
from typing import Dict, List, Optional

import numpy as np
import torch

from .. import ops
from .capture_session import cube_slot
from .epipolar_matching import _device, compute_cost_matrix, match_objects, triangulate_multi_view
from .utils.camera_utils import compute_fundamental_matrix

__all__ = ["PoseEstimatorParams", "PosePrediction", "PackedDetections", "pack_detector_outputs",
           "detect_capture", "match_detections", "MatcherMixin", "install_into_reference"]


@dataclass
class PoseEstimatorParams:
    """Same fields and defaults as the reference (process_pose.py:32-38)."""
    yolo_model_path: str = "yolo11-detection-obj11.pt"
    pose_model_path: str = "best_model.pth"
    matching_threshold: int = 30
    yolo_conf_thresh: float = 0.1
    rotation_mode: Optional[str] = None


class PosePrediction:
    """One matched object: per-camera boxes/centroids + triangulated centre
    (process_pose.py:79-94)."""

    def __init__(self, detections, capture):
        self.boxes = np.array([d["bbox"] for d in detections])
        self.centroids = np.array([d["bb_center"] for d in detections])
        self.capture = capture
        self.t = self.triangulate()

    def triangulate(self) -> np.ndarray:
        proj = [self.capture.Ks[k] @ self.capture.RTs[k][:3] for k in range(len(self.boxes))]
        return triangulate_multi_view(proj, self.centroids)


class PackedDetections(dict):
    """``_detect``'s result, ``{idx: [{'bbox': (x1, y1, x2, y2), 'bb_center':
    (cx, cy)}, ...]}`` (process_pose.py:133-141: Python ints / floats), plus
    the packed device copy the matcher reads directly:

    ``pts`` f64 [n, 2] and ``cam_offs`` i64 [n_img + 1] on the GPU (rows past
    ``cam_offs[-1]`` are unused capacity), ``cam_offs_host`` numpy."""

    pts: torch.Tensor
    cam_offs: torch.Tensor
    cam_offs_host: np.ndarray


def pack_detector_outputs(per_image, conf_thresh: float) -> PackedDetections:
    """Pack per-image detector outputs ``[(xyxy [n, 4], conf [n], cls [n]), ...]``
    (torch tensors, any device, as YOLO's ``results.boxes`` holds them) on the
    GPU with ``_detect``'s rules (process_pose.py:130-136)."""
    dev = _device()
    boxes = torch.cat([torch.as_tensor(b).reshape(-1, 4).to(dev, torch.float32) for b, _, _ in per_image]
                      + [torch.zeros((0, 4), device=dev)])
    conf = torch.cat([torch.as_tensor(c).reshape(-1).to(dev, torch.float32) for _, c, _ in per_image]
                     + [torch.zeros(0, device=dev)])
    cls = torch.cat([torch.as_tensor(k).reshape(-1).to(dev, torch.float32) for _, _, k in per_image]
                    + [torch.zeros(0, device=dev)])
    offs = np.zeros(len(per_image) + 1, np.int64)
    np.cumsum([int(torch.as_tensor(c).numel()) for _, c, _ in per_image], out=offs[1:])
    pts, cam_offs, bbox, _, status = ops.pack_detections(boxes, conf, cls,
                                                         torch.from_numpy(offs).to(dev), conf_thresh)
    off_h = cam_offs.cpu().numpy()
    if int(status.item()) != 0:
        raise ValueError("cannot convert a non-finite or out-of-range box coordinate to int")
    n = int(off_h[-1])
    bbox_h = bbox[:n].cpu().numpy().tolist()
    pts_h = pts[:n].cpu().numpy().tolist()
    out = PackedDetections()
    for k in range(len(per_image)):
        out[k] = [{"bbox": tuple(bbox_h[q]), "bb_center": tuple(pts_h[q])}
                  for q in range(int(off_h[k]), int(off_h[k + 1]))]
    out.pts, out.cam_offs, out.cam_offs_host = pts, cam_offs, off_h
    return out


def detect_capture(yolo, capture, conf_thresh: float, *, imgsz: int = 1280,
                   verbose: bool = True) -> PackedDetections:
    """``PoseEstimator._detect`` (process_pose.py:116-142): run the detector on
    every image, then pack all images' boxes on the GPU in one launch."""
    per_image = []
    for image in capture.images:
        if verbose:
            print(f"Processing image shape: {image.shape}")
        res = yolo(image, imgsz=imgsz)[0]
        per_image.append((res.boxes.xyxy, res.boxes.conf, res.boxes.cls))
    return pack_detector_outputs(per_image, conf_thresh)


def _packed_cube(det: PackedDetections, F12, F13, F23) -> np.ndarray:
    """The cost cube straight from the packed device centroids of images 0-2
    (only F travels host -> device; capture_session's cached slot)."""
    N, M, P = (int(c) for c in np.diff(det.cam_offs_host[:4]))
    slot = cube_slot(N, M, P, det.pts.device)
    return slot.run(None, (F12, F13, F23), pts=det.pts, cam_offs=det.cam_offs[:4], counts=(N, M, P))


def match_detections(capture, detections: Dict[int, list], params=None, *,
                     verbose: bool = True) -> List[PosePrediction]:
    """``PoseEstimator._match`` (process_pose.py:144-188) on the GPU matcher."""
    threshold = (params.matching_threshold if params is not None
                 else PoseEstimatorParams().matching_threshold)
    out: List[PosePrediction] = []
    d1, d2, d3 = detections[0], detections[1], detections[2]
    K1, K2, K3 = capture.Ks
    (R1, R2, R3) = (rt[:3, :3] for rt in capture.RTs)
    (t1, t2, t3) = (rt[:3, 3] for rt in capture.RTs)
    F12 = compute_fundamental_matrix(K1, R1, t1, K2, R2, t2)
    F13 = compute_fundamental_matrix(K1, R1, t1, K3, R3, t3)
    F23 = compute_fundamental_matrix(K2, R2, t2, K3, R3, t3)

    if len(d1) == 0 or len(d2) == 0 or len(d3) == 0:
        if verbose:
            print("\nAt least one camera has zero detections => no matching.")
        return out

    if isinstance(detections, PackedDetections) and hasattr(detections, "pts"):
        cost = _packed_cube(detections, F12, F13, F23)        # no host -> device copy
    else:
        cost = compute_cost_matrix(d1, d2, d3, F12, F13, F23)
    N, M, P = cost.shape
    # the reference prints stats and samples with the global RNG; keep the
    # RNG consumption identical even when quiet (the text is built only to print)
    lines = ["\n--- Cost Matrix Stats ---", f"Shape: {cost.shape}",
             f"Min: {cost.min():.4f}, Max: {cost.max():.4f}, Mean: {cost.mean():.4f}",
             "\nRandom samples from cost_matrix:"] if verbose else []
    for _ in range(min(5, N * M * P)):
        i = np.random.randint(0, N)
        j = np.random.randint(0, M)
        k = np.random.randint(0, P)
        if verbose:
            lines.append(f"  cost_matrix[{i},{j},{k}] = {cost[i, j, k]:.4f}")
    if verbose:
        print("\n".join(lines))

    matches = match_objects(cost, threshold=threshold)
    for i, j, k in sorted(matches, key=lambda m: cost[m[0], m[1], m[2]]):
        out.append(PosePrediction([d1[i], d2[j], d3[k]], capture))
    return out


class MatcherMixin:
    """Mix into (or monkey-patch onto) the reference ``PoseEstimator``:
    ``_detect``'s packing and ``_match`` then run on the MI355X; the YOLO
    and pose networks are unchanged."""

    def _detect(self, capture):
        return detect_capture(self.yolo, capture, self.params.yolo_conf_thresh)

    def _match(self, capture, detections):
        return match_detections(capture, detections, getattr(self, "params", None))


def install_into_reference(verbose: bool = False) -> List[str]:
    """Rebind the reference's matcher names to this implementation.

    ``bpc.inference.process_pose`` binds ``compute_cost_matrix``,
    ``match_objects`` and ``triangulate_multi_view`` by name at import time
    (process_pose.py:24), so the module attributes are replaced in every
    already-imported reference module.  ``PoseEstimator._detect`` and
    ``_match`` (the two calls the Inference Notebook makes) are replaced by
    MatcherMixin's, so the packed device centroids flow from one to the other.
    Returns the patched qualified names.
    """
    from . import epipolar_matching as ours
    names = ["epipolar_error", "epipolar_error_full", "compute_cost_matrix", "match_objects",
             "triangulate_multi_view"]
    patched = []
    for mod_name in ("bpc.inference.epipolar_matching", "bpc.inference.process_pose"):
        mod = sys.modules.get(mod_name)
        if mod is None:
            continue
        for n in names:
            if hasattr(mod, n):
                setattr(mod, n, getattr(ours, n))
                patched.append(f"{mod_name}.{n}")
    est = getattr(sys.modules.get("bpc.inference.process_pose"), "PoseEstimator", None)
    if est is not None:
        for n in ("_detect", "_match"):
            setattr(est, n, getattr(MatcherMixin, n))
            patched.append(f"bpc.inference.process_pose.PoseEstimator.{n}")
    if verbose:
        print("bpc_baseline_amd: patched " + ", ".join(patched))
    return patched
