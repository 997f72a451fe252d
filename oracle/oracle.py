"""ctypes wrapper of the C restatement (mvm_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py, as the checker.  The product package
(bpc_baseline_amd) never imports this module.

Every function mirrors a reference symbol (see mvm_oracle.c for file:line).
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from typing import Optional, Tuple

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "libmvm_oracle.so")

_lib = None


def build() -> str:
    """Compile the C restatement with oracle/Makefile (gcc)."""
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        vp, d, i, i64 = ctypes.c_void_p, ctypes.c_double, ctypes.c_int, ctypes.c_int64
        L.mvm_oracle_epipolar_error.restype = d
        L.mvm_oracle_epipolar_error.argtypes = [vp, d, d, d, d]
        L.mvm_oracle_epipolar_error_full.restype = d
        L.mvm_oracle_epipolar_error_full.argtypes = [vp] * 6
        L.mvm_oracle_pairwise.restype = None
        L.mvm_oracle_pairwise.argtypes = [vp, vp, vp, vp, i, i, i, vp, vp, vp, vp, vp, i]
        L.mvm_oracle_cube.restype = None
        L.mvm_oracle_cube.argtypes = [vp, vp, vp, i, vp, vp, vp, vp, vp, i]
        L.mvm_oracle_residuals.restype = None
        L.mvm_oracle_residuals.argtypes = [vp, vp, vp, i, i, ctypes.c_int64, vp, i]
        L.mvm_oracle_max_threads.restype = i
        _lib = L
    return _lib


def _ptr(a: Optional[np.ndarray]):
    return None if a is None else a.ctypes.data


def epipolar_error(pt1, pt2, F) -> float:
    F = np.ascontiguousarray(F, dtype=np.float64).reshape(9)
    return lib().mvm_oracle_epipolar_error(_ptr(F), float(pt1[0]), float(pt1[1]),
                                           float(pt2[0]), float(pt2[1]))


def epipolar_error_full(pt1, pt2, pt3, F12, F13, F23) -> float:
    arrs = [np.ascontiguousarray(x, dtype=np.float64).reshape(-1) for x in (pt1, pt2, pt3, F12, F13, F23)]
    return lib().mvm_oracle_epipolar_error_full(*[_ptr(a) for a in arrs])


def pairwise_offsets(cam_offs: np.ndarray, n_scenes: int, n_cams: int, pairs: np.ndarray):
    """(dist_offs, row_offs) for every (scene, pair) in scene-major order."""
    counts = np.diff(cam_offs).reshape(n_scenes, n_cams)
    na = counts[:, pairs[:, 0]].reshape(-1)
    nb = counts[:, pairs[:, 1]].reshape(-1)
    dist_offs = np.zeros(len(na) + 1, np.int64)
    row_offs = np.zeros(len(na) + 1, np.int64)
    np.cumsum(na * nb, out=dist_offs[1:])
    np.cumsum(na, out=row_offs[1:])
    return dist_offs, row_offs


def pairwise(pts, cam_offs, F, pairs, n_scenes, n_cams, *, want_dist=True,
             nthreads: int = 0) -> Tuple[Optional[np.ndarray], np.ndarray, np.ndarray, np.ndarray, np.ndarray]:
    """-> (dist f32 flat, argmin i32, minv f32, dist_offs, row_offs)."""
    pts = np.ascontiguousarray(pts, np.float64)
    cam_offs = np.ascontiguousarray(cam_offs, np.int64)
    F = np.ascontiguousarray(F, np.float64)
    pairs = np.ascontiguousarray(pairs, np.int32)
    dist_offs, row_offs = pairwise_offsets(cam_offs, n_scenes, n_cams, pairs)
    dist = np.empty(int(dist_offs[-1]), np.float32) if want_dist else None
    argmin = np.empty(int(row_offs[-1]), np.int32)
    minv = np.empty(int(row_offs[-1]), np.float32)
    lib().mvm_oracle_pairwise(_ptr(pts), _ptr(cam_offs), _ptr(F), _ptr(pairs), n_scenes, n_cams,
                              len(pairs), _ptr(dist_offs), _ptr(row_offs), _ptr(dist),
                              _ptr(argmin), _ptr(minv), nthreads)
    return dist, argmin, minv, dist_offs, row_offs


def cube_offsets(cam_offs: np.ndarray, n_scenes: int):
    counts = np.diff(cam_offs).reshape(n_scenes, 3)
    rows = counts[:, 0] * counts[:, 1]
    cube_offs = np.zeros(n_scenes + 1, np.int64)
    row_offs = np.zeros(n_scenes + 1, np.int64)
    np.cumsum(rows * counts[:, 2], out=cube_offs[1:])
    np.cumsum(rows, out=row_offs[1:])
    return cube_offs, row_offs


def cube(pts, cam_offs, F, n_scenes, *, want_cube=True, nthreads: int = 0):
    """3-camera cost cubes -> (cube f32 flat, argmin i32, minv f32, cube_offs, row_offs).

    F is f64 [S*3, 9] ordered F12, F13, F23 per scene."""
    pts = np.ascontiguousarray(pts, np.float64)
    cam_offs = np.ascontiguousarray(cam_offs, np.int64)
    F = np.ascontiguousarray(F, np.float64)
    cube_offs, row_offs = cube_offsets(cam_offs, n_scenes)
    out = np.empty(int(cube_offs[-1]), np.float32) if want_cube else None
    argmin = np.empty(int(row_offs[-1]), np.int32)
    minv = np.empty(int(row_offs[-1]), np.float32)
    lib().mvm_oracle_cube(_ptr(pts), _ptr(cam_offs), _ptr(F), n_scenes, _ptr(cube_offs),
                          _ptr(row_offs), _ptr(out), _ptr(argmin), _ptr(minv), nthreads)
    return out, argmin, minv, cube_offs, row_offs


def max_threads() -> int:
    return int(lib().mvm_oracle_max_threads())


def residuals(pts, cam_offs, F, n_scenes: int, max_n: int, *, nthreads: int = 0) -> np.ndarray:
    """fp64 pair residuals of every 3-camera scene in the GPU cube-free layout
    (mvm_triplet_minima): f64 [S, 3, max_n, ld] = e12 [N][ld], e13T [P][ld],
    e23T [P][ld]; entries outside the views are NaN."""
    pts = np.ascontiguousarray(pts, np.float64)
    cam_offs = np.ascontiguousarray(cam_offs, np.int64)
    F = np.ascontiguousarray(F, np.float64)
    ld = (max_n + 3) // 4 * 4
    out = np.full((n_scenes, 3, max_n, ld), np.nan)
    lib().mvm_oracle_residuals(_ptr(pts), _ptr(cam_offs), _ptr(F), n_scenes, max_n, ld, _ptr(out),
                               nthreads)
    return out


def bmin8_keys(cube: np.ndarray) -> np.ndarray:
    """The 16-bit 8-row minima of one (N, M, P) float32 cube, as
    mvm_triplet_cost_argmin_bmin8 / mvm_triplet_minima write them: per (i,
    group of 8 j, k) the upper half of (bits | 0x80000000) of the group's
    minimum, 0 when any of the group is NaN -> uint16 [N, ceil(M/8), P]."""
    N, M, P = cube.shape
    g8 = (M + 7) // 8
    pad = np.full((N, g8 * 8, P), np.inf, np.float32)
    pad[:, :M] = cube
    key = pad.view(np.uint32) | np.uint32(0x80000000)
    key = np.where(np.isnan(pad), np.uint32(0), key)
    return (key.reshape(N, g8, 8, P).min(axis=2) >> 16).astype(np.uint16)


def bm32_keys(keys: np.ndarray, N: int, M: int, P: int) -> np.ndarray:
    """The 32-column block minima mvm_triplet_minima writes (include/mvmatch.h),
    from a scene's 8-row minima (bmin8_keys: uint16 [N, ceil(M/8), P]): per
    (k, block jt of 32 j, i) the block's smallest 16-bit key; rows i >= N
    0xFFFF -> uint16 [P, ceil(M/32), roundup(N, 16)]."""
    g8, bps, npad = (M + 7) // 8, (M + 31) // 32, (N + 15) // 16 * 16
    pad = np.full((N, bps * 4, P), 0xFFFF, np.uint16)
    pad[:, :g8] = keys
    h = pad.reshape(N, bps, 4, P).min(axis=2)                         # [N, bps, P]
    out = np.full((P, bps, npad), 0xFFFF, np.uint16)
    out[:, :, :N] = h.transpose(2, 1, 0)
    return out


