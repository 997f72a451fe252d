"""ctypes binding of the C ABI in include/mvmatch.h (libmvmatch.so).

The library is built in-tree by ``__graft_entry__.build()`` (hipcc,
--offload-arch=gfx950) into ``bpc_baseline_amd/lib/libmvmatch.so``.  There is
no fallback: if the library is missing or fails to load, importing the ops
raises, so the product path can never silently run anything but the HIP
kernels.
"""
from __future__ import annotations

import ctypes
import os
import re

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
# MVM_LIB_PATH: an alternative in-tree build for A/B timing (tools/ only; the
# library itself reads no environment)
LIB_PATH = os.environ.get("MVM_LIB_PATH") or os.path.join(PKG_DIR, "lib", "libmvmatch.so")
HEADER_PATH = os.path.join(os.path.dirname(PKG_DIR), "include", "mvmatch.h")

MVM_OK = 0
MVM_MAX_CAMS = 8
MVM_MAX_PAIRS = 28
MVM_F32, MVM_F64 = 0, 1

# enum values of include/mvmatch.h
PAIRWISE_ARGMIN = {"default": 0, "lazy_transposed": 1, "lazy_rows": 2, "eager": 3}
CUBE_KERNEL = {"default": 0, "small": 1, "fused": 2, "workspace": 3, "generic": 4}


class MvmOptions(ctypes.Structure):
    """``mvm_options`` (include/mvmatch.h): kernel-path selection; every field
    0 = the compiled-in default.  The choices never change results."""
    _fields_ = [(n, ctypes.c_int32) for n in (
        "size", "pairwise_argmin", "pairwise_rows_per_wave", "pairwise_row_groups",
        "cube_kernel", "cube_rows_per_instr", "lsap_wave_max_cols", "lsap_multi_g",
        "lsap_lds_max_cols", "lsap_lds_small_cols", "lsap_mid_max_cols", "lsap_reg_max_cols",
        "lsap_reg_threads", "lsap_mreg_max_cols", "pairwise_row_interleave",
        "cube_cols_per_lane", "pairwise_xcd_fronts", "lsap_sparse_min_cols",
        "lsap_sparse_blocks", "cube_tile_rows")]


OPTION_FIELDS = [n for n, _ in MvmOptions._fields_[1:]]


def make_options(**kw):
    """MvmOptions from keyword fields (names above; enum fields also accept the
    names in PAIRWISE_ARGMIN / CUBE_KERNEL).  No keywords -> None (defaults)."""
    if not kw:
        return None
    o = MvmOptions()
    o.size = ctypes.sizeof(MvmOptions)
    for k, v in kw.items():
        if k not in OPTION_FIELDS:
            raise ValueError(f"unknown mvm_options field {k!r}")
        if k == "pairwise_argmin" and isinstance(v, str):
            v = PAIRWISE_ARGMIN[v]
        if k == "cube_kernel" and isinstance(v, str):
            v = CUBE_KERNEL[v]
        setattr(o, k, int(v))
    return o


class MvmError(RuntimeError):
    """A non-zero status returned by the C ABI."""

    def __init__(self, fn: str, status: int, message: str):
        super().__init__(f"{fn} failed with status {status}: {message}")
        self.status = status


_vp = ctypes.c_void_p
_i32 = ctypes.c_int32
_i64 = ctypes.c_int64
_sz = ctypes.c_size_t

# name -> (restype, argtypes); kept in the order of include/mvmatch.h
SIGNATURES = {
    "mvm_version": (ctypes.c_char_p, []),
    "mvm_last_error_string": (ctypes.c_char_p, []),
    "mvm_status_string": (ctypes.c_char_p, [ctypes.c_int]),
    "mvm_options_init": (None, [_vp]),
    "mvm_pairwise_residual_argmin": (ctypes.c_int, [
        _vp, _vp, _vp, _vp, _vp,            # pts, cam_offs, F, pair_a (host), pair_b (host)
        _i32, _i32, _i32, _i32,             # n_scenes, n_cams, n_pairs, max_n
        _vp, _vp, _vp, _vp, _vp,            # dist_offs, row_offs, dist, argmin, minval
        _vp]),                              # stream
    "mvm_pairwise_residual_argmin_ex": (ctypes.c_int, [
        _vp, _vp, _vp, _vp, _vp,
        _i32, _i32, _i32, _i32,
        _vp, _vp, _vp, _vp, _vp,
        _vp, _vp]),                         # options (host), stream
    "mvm_pairwise_residual_argmin_pitched": (ctypes.c_int, [
        _vp, _vp, _vp, _vp, _vp,
        _i32, _i32, _i32, _i32, _i32,       # n_scenes, n_cams, n_pairs, max_n, row_align
        _vp, _vp, _vp, _vp, _vp,
        _vp, _vp]),                         # options (host), stream
    "mvm_pairwise_residual_f64": (ctypes.c_int, [
        _vp, _vp, _vp, _vp, _vp,
        _i32, _i32, _i32, _i32,
        _i64, _i64, _vp,                    # mat_stride, ld, e
        _vp]),
    "mvm_triplet_workspace_bytes": (_sz, [_i32, _i32]),
    "mvm_triplet_cost_argmin": (ctypes.c_int, [
        _vp, _vp, _vp, _i32, _i32,          # pts, cam_offs, F, n_scenes, max_n
        _vp, _vp, _vp, _vp, _vp,            # cube_offs, row_offs, cube, argmin, minval
        _vp, _sz, _vp]),                    # workspace, workspace_bytes, stream
    "mvm_triplet_cost_argmin_ex": (ctypes.c_int, [
        _vp, _vp, _vp, _i32, _i32,
        _vp, _vp, _vp, _vp, _vp,
        _vp, _sz, _vp, _vp]),               # workspace, bytes, options (host), stream
    "mvm_triplet_cost_argmin_bmin8": (ctypes.c_int, [
        _vp, _vp, _vp, _i32, _i32,
        _vp, _vp, _vp, _vp, _vp,
        _vp, _vp,                           # bmin8, bmin8_offs
        _vp, _sz, _vp, _vp]),               # workspace, bytes, options (host), stream
    "mvm_triplet_minima": (ctypes.c_int, [
        _vp, _vp, _vp, _i32, _i32,          # pts, cam_offs, F, n_scenes, max_n
        _vp, _vp, _vp, _vp,                 # bmin8, bmin8_offs, bm32, bm32_offs
        _vp, _sz, _vp, _vp]),               # resid, resid_bytes, options (host), stream
    "mvm_lsap_plan": (_i64, [_i32, _vp, _vp, _vp, _vp]),
    "mvm_lsap_plan_ex": (_i64, [_i32, _vp, _vp, _i32, _vp, _vp]),
    "mvm_lsap_solve": (ctypes.c_int, [
        _vp, _vp, _vp, _i32, _vp, _vp,      # cost, cost_offs, dims, n, ws_offs, out_offs
        _vp, _sz, _vp, _vp, _vp, _vp]),     # workspace, bytes, row_ind, col_ind, status, stream
    "mvm_lsap_solve_bounded": (ctypes.c_int, [
        _vp, _vp, _vp, _i32, _vp, _vp,
        _vp, _sz, _vp, _vp, _vp,
        _i64, _i64, _vp]),                  # long_min, long_max, stream
    "mvm_lsap_solve_ex": (ctypes.c_int, [
        _vp, _i32, _vp, _vp, _i32, _vp, _vp,   # cost, dtype, cost_offs, dims, n, ws_offs, out_offs
        _vp, _sz, _vp, _vp, _vp,            # workspace, bytes, row_ind, col_ind, status
        _i64, _i64, _vp, _vp]),             # long_min, long_max, options (host), stream
    "mvm_lsap_solve_ex2": (ctypes.c_int, [
        _vp, _i32, _vp, _vp, _i32, _vp, _vp,
        _vp, _sz, _vp, _vp, _vp,
        _i64, _i64, _i64, _vp, _vp]),       # long_min, long_max, short_max, options, stream
    "mvm_lsap_solve_ex3": (ctypes.c_int, [
        _vp, _i32, _vp, _vp, _i32, _vp, _vp,
        _vp, _sz, _vp, _vp, _vp,
        _i64, _i64, _i64,
        _vp, _vp, _vp, _vp, _vp]),          # bmin8, bmin8_offs, segs, options, stream
    "mvm_lsap_plan_resid": (_i64, [_i32, _vp, _vp, _vp, _vp]),
    "mvm_lsap_sparse_bounds": (None, [_vp, _vp, _vp]),
    "mvm_lsap_sparse_stats_offset": (_i64, [_i64, _i64]),
    "mvm_lsap_solve_resid": (ctypes.c_int, [
        _vp, _i32, _vp, _vp,                # dims, n, ws_offs, out_offs
        _vp, _sz, _vp, _vp, _vp,            # workspace, bytes, row_ind, col_ind, status
        _i64, _i64, _i64,                   # long_min, long_max, short_max
        _vp, _vp, _vp, _vp, _vp,            # bmin8, bmin8_offs, bm32, bm32_offs, segs
        _vp, _i32, _vp, _vp]),              # resid, max_n, options (host), stream
    "mvm_pack_detections": (ctypes.c_int, [
        _vp, _vp, _vp, _vp, _i32,           # boxes, conf, cls, img_offs, n_img
        ctypes.c_float, ctypes.c_float,     # conf_thresh, class_id
        _vp, _vp, _vp, _vp, _vp, _vp]),     # counts, cam_offs, pts, boxes_out, status, stream
    "mvm_triangulate_dlt": (ctypes.c_int, [
        _vp, _vp, _vp, _i32, _i32, _vp, _vp]),  # proj, set_of_point, pts2d, n_points, n_views, X, stream
    "mvm_select_triangulate": (ctypes.c_int, [
        _vp, _vp, _vp, _vp, _vp, _vp,       # cube, cube_offs, cam_offs, lsap_out_offs, row_ind, col_ind
        _vp, _vp, _i32, ctypes.c_double,    # pts, proj, n_scenes, threshold
        _vp, _vp, _vp, _vp, _vp]),          # match, cost, X, count, stream
    "mvm_select_triangulate_resid": (ctypes.c_int, [
        _vp, _i32, _vp, _vp, _vp, _vp,      # resid, max_n, cam_offs, lsap_out_offs, row_ind, col_ind
        _vp, _vp, _i32, ctypes.c_double,    # pts, proj, n_scenes, threshold
        _vp, _vp, _vp, _vp, _vp]),          # match, cost, X, count, stream
    "mvm_hbm_write_probe": (ctypes.c_int, [_vp, _sz, _vp]),
}

_lib = None


def header_symbols() -> list:
    """Function names declared in include/mvmatch.h (for the export test)."""
    with open(HEADER_PATH) as fh:
        text = fh.read()
    return re.findall(r"^\s*(?:const\s+)?[a-z_0-9]+\s*\*?\s*(mvm_[a-z_0-9]+)\s*\(", text, re.M)


def load(path: str = LIB_PATH):
    """Load libmvmatch.so once and attach the C signatures.  Raises if missing."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise ImportError(
            f"{path} not found: build the HIP library first "
            "(python -c 'import __graft_entry__ as g; g.build()')")
    lib = ctypes.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def check(fn_name: str, status: int) -> None:
    if status != MVM_OK:
        msg = load().mvm_last_error_string().decode(errors="replace")
        raise MvmError(fn_name, status, msg or load().mvm_status_string(status).decode())


def version() -> str:
    return load().mvm_version().decode()
