"""PyTorch custom ops over the C ABI (``torch.ops.mvmatch.*``).

Each op is a thin shim: it validates dtypes/devices/shapes, then calls the
corresponding ``include/mvmatch.h`` entry point on the tensors' device
pointers and the current HIP stream.  Nothing here computes on the host.

Ops (all ``*_out`` ops write caller-allocated tensors, like the C ABI):
  mvmatch::pairwise_residual_argmin_out   e_ab (f32) + per-row argmin/min
  mvmatch::pairwise_residual_f64_out      e_ab kept in float64 (uniform layout)
  mvmatch::triplet_cost_argmin_out        3-camera cube + per-(i,j) argmin

Plans (``PairwisePlan`` / ``TripletPlan``) hold the host-side offset tables
(prefix sums of the per-view detection counts) and their device copies; a
plan is reusable for every batch with the same counts.

Kernel-path choices (``include/mvmatch.h`` ``mvm_options``) are explicit:
the high-level functions take ``options=dict(...)`` (field names of
``_native.MvmOptions``) and the ops an ``opts`` list of the field values; by
default (None) the library's compiled-in defaults apply.  The choices never
change results -- the parity tests run every path.
"""
from __future__ import annotations

import ctypes
from typing import List, Optional, Tuple

import numpy as np
import torch
from torch import Tensor

from . import _native

__all__ = [
    "PairwisePlan", "TripletPlan",
    "pairwise_residual_argmin", "pairwise_residual_f64", "triplet_cost_argmin",
    "hbm_write_probe", "LsapPlan", "linear_sum_assignment_batched",
    "pack_detections", "triangulate_dlt", "select_triangulate",
    "triplet_minima", "linear_sum_assignment_resid", "select_triangulate_resid",
    "cube_free_scenes", "sparse_class_bounds", "lsap_sparse_stats",
]


def _h2d_int64(arrays: List[np.ndarray], device: torch.device) -> List[Tensor]:
    """Host int64 arrays -> device tensors with ONE copy: concatenated into a
    pinned staging buffer and copied without blocking (a plan's offsets used
    to cost one synchronous pageable copy each).  Returns views of the one
    device buffer, in order."""
    flat = np.concatenate([np.ascontiguousarray(a, dtype=np.int64).reshape(-1) for a in arrays])
    host = torch.from_numpy(flat)
    if device.type == "cuda":
        dev = host.pin_memory().to(device, non_blocking=True)
    else:
        dev = host.to(device)
    out, o = [], 0
    for a in arrays:
        out.append(dev[o:o + a.size])
        o += a.size
    return out


def _opts_list(options: Optional[dict]) -> Optional[List[int]]:
    """options dict -> the op's ``opts`` list (mvm_options fields after ``size``)."""
    o = _native.make_options(**(options or {}))
    return None if o is None else [int(getattr(o, n)) for n in _native.OPTION_FIELDS]


def _opts_ref(opts: Optional[List[int]]):
    """The op's ``opts`` list -> a pointer to an mvm_options (None = defaults)."""
    if opts is None:
        return None
    if len(opts) != len(_native.OPTION_FIELDS):
        raise ValueError(f"opts: expected {len(_native.OPTION_FIELDS)} values, got {len(opts)}")
    return ctypes.byref(_native.make_options(**dict(zip(_native.OPTION_FIELDS, opts))))


def _p(t: Optional[Tensor]):
    if t is None or t.numel() == 0:
        return None
    return ctypes.c_void_p(t.data_ptr())


def _stream(t: Tensor):
    return ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


def _require(t: Tensor, name: str, dtype: torch.dtype, device: torch.device) -> None:
    if t.dtype != dtype:
        raise ValueError(f"{name}: expected {dtype}, got {t.dtype}")
    if t.device != device:
        raise ValueError(f"{name}: expected device {device}, got {t.device}")
    if not t.is_contiguous():
        raise ValueError(f"{name}: must be contiguous")


def _check_inputs(pts: Tensor, cam_offs: Tensor, F: Tensor, n_views: int, n_mats: int) -> None:
    if pts.device.type != "cuda":
        raise ValueError("pts must be a GPU tensor (the matcher has no CPU path)")
    dev = pts.device
    _require(pts, "pts", torch.float64, dev)
    _require(cam_offs, "cam_offs", torch.int64, dev)
    _require(F, "F", torch.float64, dev)
    if pts.dim() != 2 or pts.shape[1] != 2:
        raise ValueError(f"pts: expected [n, 2], got {tuple(pts.shape)}")
    if cam_offs.numel() != n_views + 1:
        raise ValueError(f"cam_offs: expected {n_views + 1} entries, got {cam_offs.numel()}")
    if F.numel() != n_mats * 9:
        raise ValueError(f"F: expected {n_mats} 3x3 matrices, got {F.numel()} values")


# ------------------------------------------------------------------ ops ----
@torch.library.custom_op("mvmatch::pairwise_residual_argmin_out",
                         mutates_args=("dist", "argmin", "minval"))
def pairwise_residual_argmin_out(pts: Tensor, cam_offs: Tensor, F: Tensor, pair_a: List[int],
                                 pair_b: List[int], n_scenes: int, n_cams: int, max_n: int,
                                 dist_offs: Tensor, row_offs: Tensor, dist: Tensor,
                                 argmin: Tensor, minval: Tensor,
                                 opts: Optional[List[int]] = None, row_align: int = 1) -> None:
    n_pairs = len(pair_a)
    _check_inputs(pts, cam_offs, F, n_scenes * n_cams, n_scenes * n_pairs)
    for t, n, dt in ((dist_offs, "dist_offs", torch.int64), (row_offs, "row_offs", torch.int64),
                     (dist, "dist", torch.float32), (argmin, "argmin", torch.int32),
                     (minval, "minval", torch.float32)):
        _require(t, n, dt, pts.device)
    pa = (ctypes.c_int32 * n_pairs)(*pair_a)
    pb = (ctypes.c_int32 * n_pairs)(*pair_b)
    st = _native.load().mvm_pairwise_residual_argmin_pitched(
        _p(pts), _p(cam_offs), _p(F), pa, pb, n_scenes, n_cams, n_pairs, max_n, row_align,
        _p(dist_offs), _p(row_offs), _p(dist), _p(argmin), _p(minval), _opts_ref(opts),
        _stream(pts))
    _native.check("mvm_pairwise_residual_argmin_pitched", st)


@pairwise_residual_argmin_out.register_fake
def _(pts, cam_offs, F, pair_a, pair_b, n_scenes, n_cams, max_n, dist_offs, row_offs, dist,
      argmin, minval, opts=None, row_align=1):
    return None


@torch.library.custom_op("mvmatch::pairwise_residual_f64_out", mutates_args=("e",))
def pairwise_residual_f64_out(pts: Tensor, cam_offs: Tensor, F: Tensor, pair_a: List[int],
                              pair_b: List[int], n_scenes: int, n_cams: int, max_n: int,
                              mat_stride: int, ld: int, e: Tensor) -> None:
    n_pairs = len(pair_a)
    _check_inputs(pts, cam_offs, F, n_scenes * n_cams, n_scenes * n_pairs)
    _require(e, "e", torch.float64, pts.device)
    if e.numel() < n_scenes * n_pairs * mat_stride:
        raise ValueError("e: too small for n_scenes * n_pairs * mat_stride")
    pa = (ctypes.c_int32 * n_pairs)(*pair_a)
    pb = (ctypes.c_int32 * n_pairs)(*pair_b)
    st = _native.load().mvm_pairwise_residual_f64(
        _p(pts), _p(cam_offs), _p(F), pa, pb, n_scenes, n_cams, n_pairs, max_n, mat_stride,
        ld, _p(e), _stream(pts))
    _native.check("mvm_pairwise_residual_f64", st)


@pairwise_residual_f64_out.register_fake
def _(pts, cam_offs, F, pair_a, pair_b, n_scenes, n_cams, max_n, mat_stride, ld, e):
    return None


@torch.library.custom_op("mvmatch::triplet_cost_argmin_out",
                         mutates_args=("cube", "argmin", "minval", "workspace"))
def triplet_cost_argmin_out(pts: Tensor, cam_offs: Tensor, F: Tensor, n_scenes: int, max_n: int,
                            cube_offs: Tensor, row_offs: Tensor, cube: Tensor, argmin: Tensor,
                            minval: Tensor, workspace: Tensor,
                            opts: Optional[List[int]] = None) -> None:
    _check_inputs(pts, cam_offs, F, n_scenes * 3, n_scenes * 3)
    for t, n, dt in ((cube_offs, "cube_offs", torch.int64), (row_offs, "row_offs", torch.int64),
                     (cube, "cube", torch.float32), (argmin, "argmin", torch.int32),
                     (minval, "minval", torch.float32), (workspace, "workspace", torch.uint8)):
        _require(t, n, dt, pts.device)
    ws_bytes = workspace.numel()
    st = _native.load().mvm_triplet_cost_argmin_ex(
        _p(pts), _p(cam_offs), _p(F), n_scenes, max_n, _p(cube_offs), _p(row_offs), _p(cube),
        _p(argmin), _p(minval), _p(workspace), ws_bytes, _opts_ref(opts), _stream(pts))
    _native.check("mvm_triplet_cost_argmin_ex", st)


@triplet_cost_argmin_out.register_fake
def _(pts, cam_offs, F, n_scenes, max_n, cube_offs, row_offs, cube, argmin, minval, workspace,
      opts=None):
    return None


@torch.library.custom_op("mvmatch::triplet_cost_bmin8_out",
                         mutates_args=("cube", "argmin", "minval", "bmin8", "workspace"))
def triplet_cost_bmin8_out(pts: Tensor, cam_offs: Tensor, F: Tensor, n_scenes: int, max_n: int,
                           cube_offs: Tensor, row_offs: Tensor, cube: Tensor, argmin: Tensor,
                           minval: Tensor, bmin8: Tensor, bmin8_offs: Tensor, workspace: Tensor,
                           opts: Optional[List[int]] = None) -> None:
    """triplet_cost_argmin_out + the 8-row minima the assignment reduces
    (mvm_triplet_cost_argmin_bmin8)."""
    _check_inputs(pts, cam_offs, F, n_scenes * 3, n_scenes * 3)
    for t, n, dt in ((cube_offs, "cube_offs", torch.int64), (row_offs, "row_offs", torch.int64),
                     (cube, "cube", torch.float32), (argmin, "argmin", torch.int32),
                     (minval, "minval", torch.float32), (bmin8, "bmin8", torch.int16),
                     (bmin8_offs, "bmin8_offs", torch.int64), (workspace, "workspace", torch.uint8)):
        _require(t, n, dt, pts.device)
    st = _native.load().mvm_triplet_cost_argmin_bmin8(
        _p(pts), _p(cam_offs), _p(F), n_scenes, max_n, _p(cube_offs), _p(row_offs), _p(cube),
        _p(argmin), _p(minval), _p(bmin8), _p(bmin8_offs), _p(workspace), workspace.numel(),
        _opts_ref(opts), _stream(pts))
    _native.check("mvm_triplet_cost_argmin_bmin8", st)


@triplet_cost_bmin8_out.register_fake
def _(pts, cam_offs, F, n_scenes, max_n, cube_offs, row_offs, cube, argmin, minval, bmin8, bmin8_offs,
      workspace, opts=None):
    return None


@torch.library.custom_op("mvmatch::lsap_solve_bmin8_out",
                         mutates_args=("workspace", "row_ind", "col_ind", "status"))
def lsap_solve_bmin8_out(cost: Tensor, cost_offs: Tensor, dims: Tensor, ws_offs: Tensor,
                         out_offs: Tensor, workspace: Tensor, row_ind: Tensor, col_ind: Tensor,
                         status: Tensor, bmin8: Tensor, bmin8_offs: Tensor, segs: Tensor,
                         long_min: int, long_max: int, short_max: int,
                         opts: Optional[List[int]] = None) -> None:
    """lsap_solve_out taking a cube's 8-row minima (mvm_lsap_solve_ex3)."""
    dev = cost.device
    if dev.type != "cuda" or cost.dtype != torch.float32:
        raise ValueError("cost must be a float32 GPU tensor")
    for t, n, dt in ((cost_offs, "cost_offs", torch.int64), (dims, "dims", torch.int64),
                     (ws_offs, "ws_offs", torch.int64), (out_offs, "out_offs", torch.int64),
                     (workspace, "workspace", torch.uint8), (row_ind, "row_ind", torch.int64),
                     (col_ind, "col_ind", torch.int64), (status, "status", torch.int32),
                     (bmin8, "bmin8", torch.int16), (bmin8_offs, "bmin8_offs", torch.int64),
                     (segs, "segs", torch.int64)):
        _require(t, n, dt, dev)
    st = _native.load().mvm_lsap_solve_ex3(_p(cost), _native.MVM_F32, _p(cost_offs), _p(dims),
                                           status.numel(), _p(ws_offs), _p(out_offs), _p(workspace),
                                           workspace.numel(), _p(row_ind), _p(col_ind), _p(status),
                                           long_min, long_max, short_max, _p(bmin8), _p(bmin8_offs),
                                           _p(segs), _opts_ref(opts), _stream(cost))
    _native.check("mvm_lsap_solve_ex3", st)


@lsap_solve_bmin8_out.register_fake
def _(cost, cost_offs, dims, ws_offs, out_offs, workspace, row_ind, col_ind, status, bmin8, bmin8_offs,
      segs, long_min, long_max, short_max, opts=None):
    return None


@torch.library.custom_op("mvmatch::lsap_solve_out",
                         mutates_args=("workspace", "row_ind", "col_ind", "status"))
def lsap_solve_out(cost: Tensor, cost_offs: Tensor, dims: Tensor, ws_offs: Tensor,
                   out_offs: Tensor, workspace: Tensor, row_ind: Tensor, col_ind: Tensor,
                   status: Tensor, long_min: int = 1, long_max: int = 2 ** 62,
                   opts: Optional[List[int]] = None, short_max: int = -1) -> None:
    dev = cost.device
    if dev.type != "cuda":
        raise ValueError("cost must be a GPU tensor (the matcher has no CPU path)")
    if cost.dtype not in (torch.float32, torch.float64):
        raise ValueError(f"cost: expected float32 or float64, got {cost.dtype}")
    for t, n, dt in ((cost, "cost", cost.dtype), (cost_offs, "cost_offs", torch.int64),
                     (dims, "dims", torch.int64), (ws_offs, "ws_offs", torch.int64),
                     (out_offs, "out_offs", torch.int64), (workspace, "workspace", torch.uint8),
                     (row_ind, "row_ind", torch.int64), (col_ind, "col_ind", torch.int64),
                     (status, "status", torch.int32)):
        _require(t, n, dt, dev)
    n = status.numel()
    dtype = _native.MVM_F64 if cost.dtype == torch.float64 else _native.MVM_F32
    st = _native.load().mvm_lsap_solve_ex2(_p(cost), dtype, _p(cost_offs), _p(dims), n, _p(ws_offs),
                                           _p(out_offs), _p(workspace), workspace.numel(),
                                           _p(row_ind), _p(col_ind), _p(status), long_min,
                                           long_max, long_max if short_max < 0 else short_max,
                                           _opts_ref(opts), _stream(cost))
    _native.check("mvm_lsap_solve_ex2", st)


@lsap_solve_out.register_fake
def _(cost, cost_offs, dims, ws_offs, out_offs, workspace, row_ind, col_ind, status, long_min=1,
      long_max=2 ** 62, opts=None, short_max=-1):
    return None


@torch.library.custom_op("mvmatch::triplet_minima_out", mutates_args=("bmin8", "resid"))
def triplet_minima_out(pts: Tensor, cam_offs: Tensor, F: Tensor, n_scenes: int, max_n: int,
                       bmin8: Tensor, bmin8_offs: Tensor, bm32: Tensor, bm32_offs: Tensor,
                       resid: Tensor, opts: Optional[List[int]] = None) -> None:
    """The cube's 8-row minima, the assignment's 32-column block minima and
    every scene's fp64 pair residuals, no cube (mvm_triplet_minima, ABI 7)."""
    _check_inputs(pts, cam_offs, F, n_scenes * 3, n_scenes * 3)
    for t, n, dt in ((bmin8, "bmin8", torch.int16), (bmin8_offs, "bmin8_offs", torch.int64),
                     (bm32, "bm32", torch.int16), (bm32_offs, "bm32_offs", torch.int64),
                     (resid, "resid", torch.uint8)):
        _require(t, n, dt, pts.device)
    st = _native.load().mvm_triplet_minima(_p(pts), _p(cam_offs), _p(F), n_scenes, max_n, _p(bmin8),
                                           _p(bmin8_offs), _p(bm32), _p(bm32_offs), _p(resid),
                                           resid.numel(), _opts_ref(opts), _stream(pts))
    _native.check("mvm_triplet_minima", st)


@triplet_minima_out.register_fake
def _(pts, cam_offs, F, n_scenes, max_n, bmin8, bmin8_offs, bm32, bm32_offs, resid, opts=None):
    return None


@torch.library.custom_op("mvmatch::lsap_solve_resid_out",
                         mutates_args=("workspace", "row_ind", "col_ind", "status"))
def lsap_solve_resid_out(dims: Tensor, ws_offs: Tensor, out_offs: Tensor, workspace: Tensor,
                         row_ind: Tensor, col_ind: Tensor, status: Tensor, bmin8: Tensor,
                         bmin8_offs: Tensor, bm32: Tensor, bm32_offs: Tensor, segs: Tensor,
                         resid: Tensor, max_n: int, long_min: int, long_max: int, short_max: int,
                         opts: Optional[List[int]] = None) -> None:
    """The assignment of every flattened cube of a triplet_minima batch, from
    its 8-row minima and pair residuals (mvm_lsap_solve_resid, ABI 7)."""
    dev = dims.device
    if dev.type != "cuda":
        raise ValueError("dims must be a GPU tensor (the matcher has no CPU path)")
    for t, n, dt in ((dims, "dims", torch.int64), (ws_offs, "ws_offs", torch.int64),
                     (out_offs, "out_offs", torch.int64), (workspace, "workspace", torch.uint8),
                     (row_ind, "row_ind", torch.int64), (col_ind, "col_ind", torch.int64),
                     (status, "status", torch.int32), (bmin8, "bmin8", torch.int16),
                     (bmin8_offs, "bmin8_offs", torch.int64), (bm32, "bm32", torch.int16),
                     (bm32_offs, "bm32_offs", torch.int64), (segs, "segs", torch.int64),
                     (resid, "resid", torch.uint8)):
        _require(t, n, dt, dev)
    st = _native.load().mvm_lsap_solve_resid(_p(dims), status.numel(), _p(ws_offs), _p(out_offs),
                                             _p(workspace), workspace.numel(), _p(row_ind), _p(col_ind),
                                             _p(status), long_min, long_max, short_max, _p(bmin8),
                                             _p(bmin8_offs), _p(bm32), _p(bm32_offs), _p(segs), _p(resid),
                                             max_n, _opts_ref(opts), _stream(dims))
    _native.check("mvm_lsap_solve_resid", st)


@lsap_solve_resid_out.register_fake
def _(dims, ws_offs, out_offs, workspace, row_ind, col_ind, status, bmin8, bmin8_offs, bm32, bm32_offs,
      segs, resid, max_n, long_min, long_max, short_max, opts=None):
    return None


@torch.library.custom_op("mvmatch::pack_detections_out",
                         mutates_args=("counts", "cam_offs", "pts", "boxes_out", "status"))
def pack_detections_out(boxes: Tensor, conf: Tensor, cls: Tensor, img_offs: Tensor,
                        conf_thresh: float, class_id: float, counts: Tensor, cam_offs: Tensor,
                        pts: Tensor, boxes_out: Tensor, status: Tensor) -> None:
    dev = boxes.device
    if dev.type != "cuda":
        raise ValueError("boxes must be a GPU tensor (the packer has no CPU path)")
    n_img = counts.numel()
    n = boxes.shape[0] if boxes.dim() == 2 else -1
    if boxes.dim() != 2 or boxes.shape[1] != 4:
        raise ValueError("boxes must be [n, 4] (xyxy)")
    for t, name, dt, numel in ((boxes, "boxes", torch.float32, 4 * n), (conf, "conf", torch.float32, n),
                               (cls, "cls", torch.float32, n), (img_offs, "img_offs", torch.int64, n_img + 1),
                               (counts, "counts", torch.int32, n_img),
                               (cam_offs, "cam_offs", torch.int64, n_img + 1),
                               (pts, "pts", torch.float64, 2 * n),
                               (boxes_out, "boxes_out", torch.int32, 4 * n), (status, "status", torch.int32, 1)):
        _require(t, name, dt, dev)
        if t.numel() < numel:
            raise ValueError(f"{name} holds {t.numel()} elements, needs {numel}")
    st = _native.load().mvm_pack_detections(_p(boxes), _p(conf), _p(cls), _p(img_offs), n_img,
                                            float(conf_thresh), float(class_id), _p(counts),
                                            _p(cam_offs), _p(pts), _p(boxes_out), _p(status),
                                            _stream(boxes))
    _native.check("mvm_pack_detections", st)


@pack_detections_out.register_fake
def _(boxes, conf, cls, img_offs, conf_thresh, class_id, counts, cam_offs, pts, boxes_out, status):
    return None


@torch.library.custom_op("mvmatch::triangulate_dlt_out", mutates_args=("X",))
def triangulate_dlt_out(proj: Tensor, set_of_point: Optional[Tensor], pts2d: Tensor,
                        X: Tensor) -> None:
    dev = pts2d.device
    if dev.type != "cuda":
        raise ValueError("pts2d must be a GPU tensor (the triangulator has no CPU path)")
    if pts2d.dim() != 3 or pts2d.shape[2] != 2:
        raise ValueError("pts2d must be [n_points, n_views, 2]")
    n_points, n_views = int(pts2d.shape[0]), int(pts2d.shape[1])
    _require(pts2d, "pts2d", torch.float64, dev)
    _require(proj, "proj", torch.float64, dev)
    _require(X, "X", torch.float64, dev)
    if proj.dim() != 4 or tuple(proj.shape[1:]) != (n_views, 3, 4):
        raise ValueError("proj must be [n_sets, n_views, 3, 4]")
    if X.numel() < 3 * n_points:
        raise ValueError("X must hold [n_points, 3]")
    if set_of_point is None:
        if proj.shape[0] < n_points:
            raise ValueError("without set_of_point, proj needs one set per point")
    else:
        _require(set_of_point, "set_of_point", torch.int32, dev)
        if set_of_point.numel() != n_points:
            raise ValueError("set_of_point must have n_points entries")
    st = _native.load().mvm_triangulate_dlt(_p(proj), _p(set_of_point), _p(pts2d), n_points,
                                            n_views, _p(X), _stream(pts2d))
    _native.check("mvm_triangulate_dlt", st)


@triangulate_dlt_out.register_fake
def _(proj, set_of_point, pts2d, X):
    return None


@torch.library.custom_op("mvmatch::select_triangulate_out",
                         mutates_args=("match", "cost", "X", "count"))
def select_triangulate_out(cube: Tensor, cube_offs: Tensor, cam_offs: Tensor, lsap_offs: Tensor,
                           row_ind: Tensor, col_ind: Tensor, pts: Tensor, proj: Tensor,
                           threshold: float, match: Tensor, cost: Tensor, X: Tensor,
                           count: Tensor) -> None:
    dev = cube.device
    if dev.type != "cuda":
        raise ValueError("cube must be a GPU tensor (the matcher has no CPU path)")
    n_scenes = count.numel()
    for t, name, dt, numel in ((cube, "cube", torch.float32, 0),
                               (cube_offs, "cube_offs", torch.int64, n_scenes + 1),
                               (cam_offs, "cam_offs", torch.int64, 3 * n_scenes + 1),
                               (lsap_offs, "lsap_offs", torch.int64, n_scenes + 1),
                               (row_ind, "row_ind", torch.int64, 0), (col_ind, "col_ind", torch.int64, 0),
                               (pts, "pts", torch.float64, 0), (proj, "proj", torch.float64, 36 * n_scenes),
                               (match, "match", torch.int32, 3 * row_ind.numel()),
                               (cost, "cost", torch.float32, row_ind.numel()),
                               (X, "X", torch.float64, 3 * row_ind.numel()),
                               (count, "count", torch.int32, 0)):
        _require(t, name, dt, dev)
        if numel and t.numel() != numel and name in ("cube_offs", "cam_offs", "lsap_offs", "proj"):
            raise ValueError(f"{name} holds {t.numel()} elements, expected {numel}")
        if numel and t.numel() < numel:
            raise ValueError(f"{name} holds {t.numel()} elements, needs {numel}")
    if col_ind.numel() != row_ind.numel():
        raise ValueError("row_ind / col_ind differ in length")
    st = _native.load().mvm_select_triangulate(
        _p(cube), _p(cube_offs), _p(cam_offs), _p(lsap_offs), _p(row_ind), _p(col_ind), _p(pts),
        _p(proj), n_scenes, float(threshold), _p(match), _p(cost), _p(X), _p(count), _stream(cube))
    _native.check("mvm_select_triangulate", st)


@select_triangulate_out.register_fake
def _(cube, cube_offs, cam_offs, lsap_offs, row_ind, col_ind, pts, proj, threshold, match, cost,
      X, count):
    return None


@torch.library.custom_op("mvmatch::select_triangulate_resid_out",
                         mutates_args=("match", "cost", "X", "count"))
def select_triangulate_resid_out(resid: Tensor, max_n: int, cam_offs: Tensor, lsap_offs: Tensor,
                                 row_ind: Tensor, col_ind: Tensor, pts: Tensor, proj: Tensor,
                                 threshold: float, match: Tensor, cost: Tensor, X: Tensor,
                                 count: Tensor) -> None:
    """select_triangulate_out with each assigned entry recomputed from a
    triplet_minima batch's residuals (mvm_select_triangulate_resid, ABI 7)."""
    dev = pts.device
    if dev.type != "cuda":
        raise ValueError("pts must be a GPU tensor (the matcher has no CPU path)")
    n_scenes = count.numel()
    for t, name, dt, numel in ((resid, "resid", torch.uint8, 0),
                               (cam_offs, "cam_offs", torch.int64, 3 * n_scenes + 1),
                               (lsap_offs, "lsap_offs", torch.int64, n_scenes + 1),
                               (row_ind, "row_ind", torch.int64, 0), (col_ind, "col_ind", torch.int64, 0),
                               (pts, "pts", torch.float64, 0), (proj, "proj", torch.float64, 36 * n_scenes),
                               (match, "match", torch.int32, 3 * row_ind.numel()),
                               (cost, "cost", torch.float32, row_ind.numel()),
                               (X, "X", torch.float64, 3 * row_ind.numel()),
                               (count, "count", torch.int32, 0)):
        _require(t, name, dt, dev)
        if numel and t.numel() != numel and name in ("cam_offs", "lsap_offs", "proj"):
            raise ValueError(f"{name} holds {t.numel()} elements, expected {numel}")
        if numel and t.numel() < numel:
            raise ValueError(f"{name} holds {t.numel()} elements, needs {numel}")
    if col_ind.numel() != row_ind.numel():
        raise ValueError("row_ind / col_ind differ in length")
    st = _native.load().mvm_select_triangulate_resid(
        _p(resid), max_n, _p(cam_offs), _p(lsap_offs), _p(row_ind), _p(col_ind), _p(pts), _p(proj),
        n_scenes, float(threshold), _p(match), _p(cost), _p(X), _p(count), _stream(pts))
    _native.check("mvm_select_triangulate_resid", st)


@select_triangulate_resid_out.register_fake
def _(resid, max_n, cam_offs, lsap_offs, row_ind, col_ind, pts, proj, threshold, match, cost, X, count):
    return None


# ---------------------------------------------------------------- plans ----
class PairwisePlan:
    """Offsets of every (scene, pair) residual matrix and argmin row block.

    Built on the host from ``cam_offs`` (the per-view counts are host
    knowledge: they come from the detector), copied once to ``device``.

    ``row_align``: rows of matrix (s, p) are ``ld = roundup(n_b, row_align)``
    floats apart (include/mvmatch.h, mvm_pairwise_residual_argmin_pitched).
    1 (the default) is the unpitched layout: matrices back to back, rows of
    n_b floats.  "auto" (what the bench and the batch paths ask for) pitches
    rows to 128-byte lines (32 floats) when some view's count is not a
    multiple of 32 -- the ragged views real detectors produce, whose unpitched
    rows would start mid-line, ~1.4x slower per byte -- and keeps the
    unpitched layout otherwise (then the two are the same).  ``matrix()``
    returns the (n_a, n_b) view of a matrix either way; ``compact()`` the
    unpitched flat layout.
    """

    def __init__(self, cam_offs: np.ndarray, n_scenes: int, n_cams: int, pairs,
                 device: torch.device | str = "cuda", row_align=1):
        cam_offs = np.asarray(cam_offs, dtype=np.int64)
        pairs = np.asarray(pairs, dtype=np.int32).reshape(-1, 2)
        counts = np.diff(cam_offs).reshape(n_scenes, n_cams)
        na = counts[:, pairs[:, 0]].reshape(-1)
        nb = counts[:, pairs[:, 1]].reshape(-1)
        if row_align == "auto":
            row_align = 32 if (nb % 32).any() else 1
        row_align = int(row_align)
        if row_align < 1 or row_align > 256 or row_align & (row_align - 1):
            raise ValueError(f"row_align {row_align}: a power of two in [1, 256]")
        ld = (nb + row_align - 1) // row_align * row_align
        dist_offs = np.zeros(na.size + 1, np.int64)
        row_offs = np.zeros(na.size + 1, np.int64)
        np.cumsum(na * ld, out=dist_offs[1:])
        np.cumsum(na, out=row_offs[1:])
        self.n_scenes, self.n_cams = int(n_scenes), int(n_cams)
        self.pairs = pairs
        self.pair_a = [int(a) for a in pairs[:, 0]]
        self.pair_b = [int(b) for b in pairs[:, 1]]
        self.max_rows = int(na.max()) if na.size else 0
        self.max_cols = int(nb.max()) if nb.size else 0
        self.max_n = max(self.max_rows, self.max_cols)
        self.na, self.nb, self.ld = na, nb, ld
        self.row_align = row_align
        self.n_dist = int((na * nb).sum())      # residuals (pairs)
        self.dist_size = int(dist_offs[-1])     # floats of the (pitched) output
        self.n_rows = int(row_offs[-1])
        self.dist_offs_host, self.row_offs_host = dist_offs, row_offs
        self.device = torch.device(device)
        self.dist_offs, self.row_offs = _h2d_int64([dist_offs, row_offs], self.device)

    def matrix(self, dist: Tensor, scene: int, pair: int) -> Tensor:
        """(n_a, n_b) view of the (scene, pair) residual matrix inside ``dist``
        (strided when the rows are pitched)."""
        sp = scene * len(self.pair_a) + pair
        o = int(self.dist_offs_host[sp])
        na, nb, ld = int(self.na[sp]), int(self.nb[sp]), int(self.ld[sp])
        return dist[o:o + na * ld].view(na, ld)[:, :nb]

    def compact(self, dist: Tensor) -> Tensor:
        """The residuals in the unpitched layout (matrices back to back, rows
        of n_b): ``dist`` itself when the plan is unpitched, else a copy."""
        if self.dist_size == self.n_dist:
            return dist[:self.n_dist]
        parts = [self.matrix(dist, sp // len(self.pair_a), sp % len(self.pair_a)).reshape(-1)
                 for sp in range(self.na.size)]
        return torch.cat(parts) if parts else dist[:0]


def pairwise_residual_argmin(pts: Tensor, cam_offs: Tensor, F: Tensor, plan: PairwisePlan, *,
                             want_dist: bool = True,
                             out: Optional[Tuple[Tensor, Tensor, Tensor]] = None,
                             options: Optional[dict] = None):
    """-> (dist f32 [plan.dist_size], argmin i32 [plan.n_rows], minval f32 [plan.n_rows]).
    ``dist`` has the plan's (possibly pitched) layout: ``plan.matrix()`` /
    ``plan.compact()`` read it.  ``options``: mvm_options fields, e.g.
    ``{"pairwise_argmin": "eager"}``."""
    dev = pts.device
    if out is None:
        dist = torch.empty(plan.dist_size if want_dist else 0, dtype=torch.float32, device=dev)
        argmin = torch.empty(plan.n_rows, dtype=torch.int32, device=dev)
        minval = torch.empty(plan.n_rows, dtype=torch.float32, device=dev)
    else:
        dist, argmin, minval = out
    if not (options or {}).get("pairwise_xcd_fronts"):
        # the library's default front count is sized from the padded bound
        # (scenes x pairs x max rows x max columns); the plan knows the bytes
        # this launch really writes: 4 fronts per XCD from 8 GB
        options = dict(options or {})
        options["pairwise_xcd_fronts"] = 4 if (dist.numel() and 4.0 * plan.dist_size >= 8e9) else 1
    torch.ops.mvmatch.pairwise_residual_argmin_out(
        pts, cam_offs, F, plan.pair_a, plan.pair_b, plan.n_scenes, plan.n_cams, plan.max_n,
        plan.dist_offs, plan.row_offs, dist, argmin, minval, _opts_list(options), plan.row_align)
    return dist, argmin, minval


def pairwise_residual_f64(pts: Tensor, cam_offs: Tensor, F: Tensor, plan: PairwisePlan):
    """fp64 residual matrices -> Tensor [S*P, max_rows, ld] (padding unspecified)."""
    ld = (max(plan.max_cols, 1) + 3) // 4 * 4
    rows = max(plan.max_rows, 1)
    e = torch.zeros(plan.n_scenes * len(plan.pair_a) * rows * ld, dtype=torch.float64,
                    device=pts.device)
    torch.ops.mvmatch.pairwise_residual_f64_out(
        pts, cam_offs, F, plan.pair_a, plan.pair_b, plan.n_scenes, plan.n_cams, plan.max_n,
        rows * ld, ld, e)
    return e.view(plan.n_scenes * len(plan.pair_a), rows, ld)


class TripletPlan:
    """Offsets + workspace for batched 3-camera cubes (cam_offs has S*3+1 entries)."""

    def __init__(self, cam_offs: np.ndarray, n_scenes: int, device: torch.device | str = "cuda"):
        cam_offs = np.asarray(cam_offs, dtype=np.int64)
        counts = np.diff(cam_offs).reshape(n_scenes, 3)
        rows = counts[:, 0] * counts[:, 1]
        cube_offs = np.zeros(n_scenes + 1, np.int64)
        row_offs = np.zeros(n_scenes + 1, np.int64)
        np.cumsum(rows * counts[:, 2], out=cube_offs[1:])
        np.cumsum(rows, out=row_offs[1:])
        self.n_scenes = int(n_scenes)
        self.counts = counts
        self.max_n = int(counts.max()) if counts.size else 0
        self.n_cube = int(cube_offs[-1])
        self.n_rows = int(row_offs[-1])
        self.cube_offs_host, self.row_offs_host = cube_offs, row_offs
        self.device = torch.device(device)
        self.cube_offs, self.row_offs = _h2d_int64([cube_offs, row_offs], self.device)
        self.workspace_bytes = int(_native.load().mvm_triplet_workspace_bytes(self.n_scenes,
                                                                               self.max_n))
        # the cube's 8-row minima for the assignment (mvm_triplet_cost_argmin_bmin8):
        # N * ceil(M/8) rows of P 16-bit keys per scene, scenes 4 keys aligned
        # (the kernel's 8-byte stores)
        bm8 = np.zeros(n_scenes + 1, np.int64)
        np.cumsum((counts[:, 0] * ((counts[:, 1] + 7) // 8) * counts[:, 2] + 3) // 4 * 4, out=bm8[1:])
        self.bmin8_offs_host = bm8
        self.n_bmin8 = int(bm8[-1])
        # the cube-free path's 32-column block minima (mvm_triplet_minima): per
        # scene P rows of ceil(M/32) * roundup(N, 16) 16-bit keys (32-byte runs)
        b32 = np.zeros(n_scenes + 1, np.int64)
        np.cumsum(counts[:, 2] * ((counts[:, 1] + 31) // 32) * ((counts[:, 0] + 15) // 16 * 16), out=b32[1:])
        self.bm32_offs_host = b32
        self.n_bm32 = int(b32[-1])
        self.bmin8_offs, self.segs, self.bm32_offs = _h2d_int64(
            [bm8, np.ascontiguousarray(counts[:, 1]), b32], self.device)
        self.workspace = torch.empty(max(self.workspace_bytes, 16), dtype=torch.uint8,
                                     device=self.device)


def triplet_cost_argmin(pts: Tensor, cam_offs: Tensor, F: Tensor, plan: TripletPlan, *,
                        want_cube: bool = True,
                        out: Optional[Tuple[Tensor, Tensor, Tensor]] = None,
                        options: Optional[dict] = None, bmin8: Optional[Tensor] = None):
    """-> (cube f32 [plan.n_cube], argmin i32 [plan.n_rows], minval f32 [plan.n_rows]).
    ``options``: mvm_options fields, e.g. ``{"cube_kernel": "workspace"}``.
    ``bmin8`` (int16 [plan.n_bmin8]): also the 8-row minima that
    ``linear_sum_assignment_batched(..., bmin8=)`` reduces (needs the cube)."""
    dev = pts.device
    if out is None:
        cube = torch.empty(plan.n_cube if want_cube else 0, dtype=torch.float32, device=dev)
        argmin = torch.empty(plan.n_rows, dtype=torch.int32, device=dev)
        minval = torch.empty(plan.n_rows, dtype=torch.float32, device=dev)
    else:
        cube, argmin, minval = out
    if bmin8 is not None:
        torch.ops.mvmatch.triplet_cost_bmin8_out(
            pts, cam_offs, F, plan.n_scenes, plan.max_n, plan.cube_offs, plan.row_offs, cube, argmin,
            minval, bmin8, plan.bmin8_offs, plan.workspace, _opts_list(options))
        return cube, argmin, minval
    torch.ops.mvmatch.triplet_cost_argmin_out(
        pts, cam_offs, F, plan.n_scenes, plan.max_n, plan.cube_offs, plan.row_offs, cube, argmin,
        minval, plan.workspace, _opts_list(options))
    return cube, argmin, minval


def triplet_minima(pts: Tensor, cam_offs: Tensor, F: Tensor, plan: TripletPlan, *,
                   bmin8: Optional[Tensor] = None, bm32: Optional[Tensor] = None,
                   with_bmin8: bool = True, options: Optional[dict] = None):
    """Cube-free input of the assignment (mvm_triplet_minima, ABI 7): the
    cube's 8-row minima (int16 [plan.n_bmin8], the same bits
    ``triplet_cost_argmin(..., bmin8=)`` writes), the assignment's 32-column
    block minima (16-bit keys, int16 [plan.n_bm32]) and every scene's fp64 pair residuals,
    written into ``plan.workspace`` (which the default cube kernels do not
    use; a later cube launch on the plan with the workspace kernel would
    overwrite them).  -> (bmin8, bm32).  Views of at most 256 detections.
    ``with_bmin8=False``: no 8-row minima (bmin8 an empty tensor; the
    assignment then gathers whole 32-column candidate blocks)."""
    if not with_bmin8:
        bmin8 = torch.empty(0, dtype=torch.int16, device=pts.device)
    elif bmin8 is None:
        bmin8 = torch.empty(max(plan.n_bmin8, 1), dtype=torch.int16, device=pts.device)
    if bm32 is None:
        bm32 = torch.empty(max(plan.n_bm32, 8), dtype=torch.int16, device=pts.device)
    torch.ops.mvmatch.triplet_minima_out(pts, cam_offs, F, plan.n_scenes, plan.max_n, bmin8,
                                         plan.bmin8_offs, bm32, plan.bm32_offs, plan.workspace,
                                         _opts_list(options))
    return bmin8, bm32


def sparse_class_bounds() -> Tuple[int, int, int]:
    """(default lower bound of the long side, largest long side, largest
    short side) of the candidate-list assignment class (mvm_lsap_sparse_bounds)."""
    v = [ctypes.c_int32(0) for _ in range(3)]
    _native.load().mvm_lsap_sparse_bounds(*(ctypes.byref(x) for x in v))
    return tuple(int(x.value) for x in v)


def cube_free_scenes(counts: np.ndarray, min_cols: Optional[int] = None) -> np.ndarray:
    """Per scene of a (S, 3) count array: True where the cube-free association
    (triplet_minima -> linear_sum_assignment_resid -> select_triangulate_resid)
    can take it: an empty problem, or views of <= 256 detections whose
    flattened (N*M, P) problem is of the candidate-list class."""
    lo, hi, sh = sparse_class_bounds()
    lo = lo if min_cols is None else int(min_cols)
    c = np.asarray(counts, dtype=np.int64).reshape(-1, 3)
    nm, p = c[:, 0] * c[:, 1], c[:, 2]
    empty = (nm == 0) | (p == 0)
    lng, sht = np.maximum(nm, p), np.minimum(nm, p)
    ok = (c.max(axis=1) <= 256) & (lng >= lo) & (lng > 1024) & (lng <= hi) & (sht <= sh)
    return empty | ok


def hbm_write_probe(buf: Tensor) -> None:
    """Stream 16-byte nontemporal stores over ``buf`` (roofline reference)."""
    if buf.device.type != "cuda" or not buf.is_contiguous():
        raise ValueError("hbm_write_probe needs a contiguous GPU tensor")
    nbytes = buf.numel() * buf.element_size() // 16 * 16
    st = _native.load().mvm_hbm_write_probe(_p(buf), nbytes, _stream(buf))
    _native.check("mvm_hbm_write_probe", st)


class LsapPlan:
    """Workspace / output layout of a batch of assignment problems (host dims)
    whose costs are ``dtype`` (float32, or float64 as scipy assigns a float64
    matrix: the workspace holds transposed costs of that type)."""

    def __init__(self, rows, cols, device: torch.device | str = "cuda",
                 dtype: torch.dtype = torch.float32, resid: bool = False):
        rows = np.ascontiguousarray(rows, dtype=np.int64).reshape(-1)
        cols = np.ascontiguousarray(cols, dtype=np.int64).reshape(-1)
        if dtype not in (torch.float32, torch.float64):
            raise ValueError(f"LsapPlan: dtype must be float32 or float64, got {dtype}")
        if resid and dtype != torch.float32:
            raise ValueError("LsapPlan: the cube-free form assigns float32 cube entries")
        n = rows.size
        ws_offs = np.zeros(n + 1, np.int64)
        out_offs = np.zeros(n + 1, np.int64)
        if resid:      # cube-free (mvm_lsap_solve_resid): the candidate lists only
            fn = "mvm_lsap_plan_resid"
            total = _native.load().mvm_lsap_plan_resid(n, rows.ctypes.data, cols.ctypes.data,
                                                       ws_offs.ctypes.data, out_offs.ctypes.data)
        else:
            fn = "mvm_lsap_plan_ex"
            code = _native.MVM_F64 if dtype == torch.float64 else _native.MVM_F32
            total = _native.load().mvm_lsap_plan_ex(n, rows.ctypes.data, cols.ctypes.data, code,
                                                    ws_offs.ctypes.data, out_offs.ctypes.data)
        if total < 0:
            raise _native.MvmError(fn, -1, _native.load().mvm_last_error_string().decode())
        self.resid = bool(resid)
        self.ws_offs_host = ws_offs
        self.dtype = dtype
        self.n = n
        self.rows, self.cols = rows, cols
        self.out_offs_host = out_offs
        self.device = torch.device(device)
        self.dims, self.ws_offs, self.out_offs = _h2d_int64(
            [np.stack([rows, cols], axis=1).reshape(-1), ws_offs, out_offs], self.device)
        self.workspace = torch.empty(max(int(total), 16), dtype=torch.uint8, device=self.device)
        self.n_out = int(out_offs[-1])
        longs = np.maximum(rows, cols)[(rows > 0) & (cols > 0)]
        self.long_min = int(longs.min()) if longs.size else 0     # bounds for the launch
        self.long_max = int(longs.max()) if longs.size else 0
        shorts = np.minimum(rows, cols)[(rows > 0) & (cols > 0)]
        self.short_max = int(shorts.max()) if shorts.size else 0


def linear_sum_assignment_batched(cost: Tensor, cost_offs: Tensor, plan: LsapPlan, *,
                                  options: Optional[dict] = None,
                                  bmin8: Optional[Tuple[Tensor, Tensor, Tensor]] = None):
    """scipy.optimize.linear_sum_assignment for every problem of ``plan`` on the GPU.
    -> (row_ind i64 [n_out], col_ind i64 [n_out], status i32 [n]) device tensors.
    ``cost`` must have the plan's dtype.  ``bmin8`` = (keys, the TripletPlan's
    bmin8_offs, its segs) when the costs are the flattened cubes of a
    ``triplet_cost_argmin(..., bmin8=keys)`` call: the assignment then reduces
    those instead of reading every cost once more (same result)."""
    if cost.dtype != plan.dtype:
        raise ValueError(f"cost is {cost.dtype} but the plan was built for {plan.dtype}")
    dev = cost.device
    row_ind = torch.empty(max(plan.n_out, 1), dtype=torch.int64, device=dev)
    col_ind = torch.empty(max(plan.n_out, 1), dtype=torch.int64, device=dev)
    status = torch.empty(plan.n, dtype=torch.int32, device=dev)
    if bmin8 is not None and cost.dtype == torch.float32:
        torch.ops.mvmatch.lsap_solve_bmin8_out(cost, cost_offs, plan.dims, plan.ws_offs, plan.out_offs,
                                               plan.workspace, row_ind, col_ind, status, bmin8[0],
                                               bmin8[1], bmin8[2], plan.long_min, plan.long_max,
                                               plan.short_max, _opts_list(options))
        return row_ind[:plan.n_out], col_ind[:plan.n_out], status
    torch.ops.mvmatch.lsap_solve_out(cost, cost_offs, plan.dims, plan.ws_offs, plan.out_offs,
                                     plan.workspace, row_ind, col_ind, status, plan.long_min,
                                     plan.long_max, _opts_list(options), plan.short_max)
    return row_ind[:plan.n_out], col_ind[:plan.n_out], status


def lsap_sparse_stats(plan: LsapPlan, min_cols: Optional[int] = None) -> np.ndarray:
    """After a solve with ``plan``: per problem the candidate-list solver's
    counters (mvm_lsap_sparse_stats_offset) -- int64 [n, 4] = dense free-minimum
    scans, dense tie scans, overflowed lists, Dijkstra steps; -1 for problems
    outside the class (``min_cols``: its lower bound if not the default)."""
    lib = _native.load()
    lo, hi, sh = sparse_class_bounds()
    lo = lo if min_cols is None else int(min_cols)
    lng, sht = np.maximum(plan.rows, plan.cols), np.minimum(plan.rows, plan.cols)
    cls = (lng >= lo) & (lng > 1024) & (lng <= hi) & (sht >= 1) & (sht <= sh)
    out = np.full((plan.n, 4), -1, np.int64)
    if not cls.any():
        return out
    ps = np.nonzero(cls)[0]
    offs = np.array([plan.ws_offs_host[p] + lib.mvm_lsap_sparse_stats_offset(int(plan.rows[p]),
                                                                             int(plan.cols[p]))
                     for p in ps], np.int64)
    idx = torch.from_numpy((offs[:, None] // 4 + np.arange(4)).reshape(-1)).to(plan.workspace.device)
    words = plan.workspace[:plan.workspace.numel() // 4 * 4].view(torch.int32)
    out[ps] = words.index_select(0, idx).cpu().numpy().reshape(-1, 4)
    return out


def linear_sum_assignment_resid(plan: LsapPlan, tplan: TripletPlan, minima, *,
                                options: Optional[dict] = None):
    """linear_sum_assignment_batched of every flattened (N*M, P) cube of a
    ``triplet_minima(..., tplan)`` batch without the cubes (mvm_lsap_solve_resid):
    the same result (scipy's).  ``plan`` = LsapPlan(N*M, P, resid=True);
    ``minima`` = what triplet_minima returned (bmin8, bm32).
    -> (row_ind, col_ind, status) as linear_sum_assignment_batched; status 4:
    a problem outside the candidate-list class (cube_free_scenes)."""
    if not plan.resid:
        raise ValueError("linear_sum_assignment_resid needs LsapPlan(..., resid=True)")
    bmin8, bm32 = minima                  # what triplet_minima returned (bmin8 may be empty)
    dev = bm32.device
    row_ind = torch.empty(max(plan.n_out, 1), dtype=torch.int64, device=dev)
    col_ind = torch.empty(max(plan.n_out, 1), dtype=torch.int64, device=dev)
    status = torch.empty(plan.n, dtype=torch.int32, device=dev)
    torch.ops.mvmatch.lsap_solve_resid_out(plan.dims, plan.ws_offs, plan.out_offs, plan.workspace,
                                           row_ind, col_ind, status, bmin8, tplan.bmin8_offs, bm32,
                                           tplan.bm32_offs, tplan.segs, tplan.workspace, tplan.max_n,
                                           plan.long_min, plan.long_max, plan.short_max,
                                           _opts_list(options))
    return row_ind[:plan.n_out], col_ind[:plan.n_out], status


def pack_detections(boxes: Tensor, conf: Tensor, cls: Tensor, img_offs: Tensor,
                    conf_thresh: float, class_id: float = 0.0):
    """PoseEstimator._detect's box filtering + centres for a batch of images, on device.

    ``boxes`` f32 [n, 4] xyxy, ``conf``/``cls`` f32 [n] of all images
    concatenated, image k owning rows ``img_offs[k]:img_offs[k+1]`` (int64
    device tensor).  The threshold is rounded to float32 first, as numpy does
    when comparing a float32 array with a Python float (process_pose.py:130).
    -> (pts f64 [n, 2], cam_offs i64 [n_img+1], boxes_int i32 [n, 4],
    counts i32 [n_img], status i32 [1]) — rows past ``cam_offs[-1]`` are
    unused capacity; the matcher reads only the rows the offsets name.
    """
    dev = boxes.device
    n = int(boxes.shape[0])
    n_img = int(img_offs.numel()) - 1
    counts = torch.empty(max(n_img, 0), dtype=torch.int32, device=dev)
    cam_offs = torch.zeros(max(n_img, 0) + 1, dtype=torch.int64, device=dev)
    pts = torch.empty((n, 2), dtype=torch.float64, device=dev)
    boxes_out = torch.empty((n, 4), dtype=torch.int32, device=dev)
    status = torch.zeros(1, dtype=torch.int32, device=dev)
    thresh = float(np.float32(conf_thresh))
    torch.ops.mvmatch.pack_detections_out(boxes.contiguous(), conf.contiguous(), cls.contiguous(),
                                          img_offs, thresh, float(np.float32(class_id)), counts,
                                          cam_offs, pts, boxes_out, status)
    return pts, cam_offs, boxes_out, counts, status


def triangulate_dlt(proj: Tensor, pts2d: Tensor, set_of_point: Optional[Tensor] = None) -> Tensor:
    """triangulate_multi_view for every point at once -> X f64 [n_points, 3] (device)."""
    X = torch.empty((int(pts2d.shape[0]), 3), dtype=torch.float64, device=pts2d.device)
    torch.ops.mvmatch.triangulate_dlt_out(proj.contiguous(), set_of_point, pts2d.contiguous(), X)
    return X


def select_triangulate(cube: Tensor, cube_offs: Tensor, cam_offs: Tensor, lsap_offs: Tensor,
                       row_ind: Tensor, col_ind: Tensor, pts: Tensor, proj: Tensor,
                       threshold: float):
    """Filter + stable cost sort + DLT of every scene's assignment (device).
    -> (match i32 [cap, 3], cost f32 [cap], X f64 [cap, 3], count i32 [S]); scene
    s's matches are rows ``lsap_offs[s] : lsap_offs[s] + count[s]``."""
    dev = cube.device
    cap = int(row_ind.numel())
    n_scenes = int(lsap_offs.numel()) - 1
    match = torch.empty((cap, 3), dtype=torch.int32, device=dev)
    cost = torch.empty(cap, dtype=torch.float32, device=dev)
    X = torch.empty((cap, 3), dtype=torch.float64, device=dev)
    count = torch.empty(n_scenes, dtype=torch.int32, device=dev)
    torch.ops.mvmatch.select_triangulate_out(cube, cube_offs, cam_offs, lsap_offs, row_ind,
                                             col_ind, pts, proj.contiguous(), float(threshold),
                                             match, cost, X, count)
    return match, cost, X, count


def select_triangulate_resid(tplan: TripletPlan, cam_offs: Tensor, lsap_offs: Tensor,
                             row_ind: Tensor, col_ind: Tensor, pts: Tensor, proj: Tensor,
                             threshold: float):
    """select_triangulate for a ``triplet_minima(..., tplan)`` batch: each
    assigned entry recomputed from the residuals in ``tplan.workspace``."""
    dev = pts.device
    cap = int(row_ind.numel())
    n_scenes = int(lsap_offs.numel()) - 1
    match = torch.empty((cap, 3), dtype=torch.int32, device=dev)
    cost = torch.empty(cap, dtype=torch.float32, device=dev)
    X = torch.empty((cap, 3), dtype=torch.float64, device=dev)
    count = torch.empty(n_scenes, dtype=torch.int32, device=dev)
    torch.ops.mvmatch.select_triangulate_resid_out(tplan.workspace, tplan.max_n, cam_offs, lsap_offs,
                                                   row_ind, col_ind, pts, proj.contiguous(),
                                                   float(threshold), match, cost, X, count)
    return match, cost, X, count
