"""Cached launch state for the drop-in's one-capture calls.

The reference calls ``compute_cost_matrix`` and ``match_objects`` once per
capture with a few detections per view (the Inference Notebook's problems are
(4, 4, 4) and (2, 2, 2): process_pose.py:165,182).  At those sizes the kernels
take microseconds and a call's cost is its host<->device traffic: building a
plan, several pageable copies, allocating pinned staging, one synchronisation
per output.  A *slot* keeps, per problem shape, everything a call needs --
the plan's device offsets, device buffers, and pinned host staging in and out
-- so a call is: fill the pinned input, ONE host->device copy, the launch(es)
through the C ABI, ONE device->host copy, one stream synchronisation.

Slots are per thread (the reference is single-threaded; a thread never waits
on another's buffers) and per device, kept in a small LRU bounded by count
and bytes (``clear()`` releases them).  Small problems share capacity-class
slots: the per-call offsets travel in the staged copy, so a capture whose
detection counts differ from the last one's reuses the slot instead of
building plans and buffers (real captures change counts every time).
Results are identical to the general path: the same kernels run on the same
values.
"""
from __future__ import annotations

import ctypes
import threading
from collections import OrderedDict
from typing import Optional, Tuple

import numpy as np
import torch

from .. import _native, ops

__all__ = ["cube_slot", "lsap_slot", "CubeSlot", "LsapSlot", "clear", "cache_info"]

_MAX_SLOTS = 32               # per kind, per thread
_MAX_BYTES = 256 << 20        # device + pinned bytes per kind, per thread
_SMALL_CAP = 64               # views / sides up to this share capacity-class slots
_tls = threading.local()


def _cap(n: int) -> int:
    """Capacity class of a count: the next power of two, at least 8."""
    c = 8
    while c < n:
        c *= 2
    return c


def _cache(kind: str) -> "OrderedDict":
    c = getattr(_tls, kind, None)
    if c is None:
        c = OrderedDict()
        setattr(_tls, kind, c)
    return c


def _lookup(kind: str, key, make):
    """The slot for ``key`` (built on a miss), kept in the thread's LRU of at
    most _MAX_SLOTS slots and _MAX_BYTES bytes; a slot larger than the byte
    cap on its own is used once and not kept."""
    c = _cache(kind)
    slot = c.get(key)
    if slot is not None:
        c.move_to_end(key)
        return slot
    slot = make()
    if slot.nbytes > _MAX_BYTES:
        return slot
    c[key] = slot
    total = sum(x.nbytes for x in c.values())
    while len(c) > _MAX_SLOTS or total > _MAX_BYTES:
        _, old = c.popitem(last=False)
        total -= old.nbytes
    return slot


def clear() -> None:
    """Release every cached slot of the calling thread (device and pinned memory)."""
    for kind in ("cube", "lsap"):
        _cache(kind).clear()


def cache_info() -> dict:
    """Slots and bytes cached by the calling thread, per kind."""
    return {k: {"slots": len(_cache(k)), "bytes": sum(x.nbytes for x in _cache(k).values())}
            for k in ("cube", "lsap")}


def _vp(t: torch.Tensor, byte_offset: int = 0):
    return ctypes.c_void_p(t.data_ptr() + byte_offset)


class _Staging:
    """One pinned host buffer and its device twin, carved into typed regions
    (8-byte aligned): a call fills the host regions and moves them with ONE
    host->device copy."""

    def __init__(self, layout, dev):
        self.offs, o = {}, 0
        for name, dtype, n in layout:
            self.offs[name] = (o, dtype, n)
            o += (np.dtype(dtype).itemsize * n + 7) // 8 * 8
        self.nbytes = max(o, 8)
        self.host = torch.empty(self.nbytes, dtype=torch.uint8, pin_memory=True)
        self.dev = torch.empty(self.nbytes, dtype=torch.uint8, device=dev)
        hb = self.host.numpy()
        self.np = {k: hb[o:o + np.dtype(dt).itemsize * n].view(dt) for k, (o, dt, n) in self.offs.items()}

    def ptr(self, name: str):
        return _vp(self.dev, self.offs[name][0])

    def upload(self, upto: str = None, count: Optional[int] = None) -> None:
        """Copy the regions from the start through ``upto`` (all when None);
        ``count``: only the first ``count`` elements of ``upto`` itself."""
        if upto is None:
            n = self.nbytes
        else:
            o, dt, cap = self.offs[upto]
            n = o + np.dtype(dt).itemsize * (cap if count is None else min(int(count), cap))
        n = max(n, 1)
        self.dev[:n].copy_(self.host[:n], non_blocking=True)


class CubeSlot:
    """compute_cost_matrix of one capture whose views hold at most ``cap``
    detections: the offsets (cam_offs, cube_offs, row_offs) of each call's
    exact (N, M, P) travel with its centroids and F in the one staged copy, so
    every shape up to the capacity reuses the slot."""

    def __init__(self, cap: int, dev: torch.device):
        self.cap = cap
        self.stage = _Staging([("pts", np.float64, 6 * cap), ("F", np.float64, 27),
                               ("cam_offs", np.int64, 4), ("cube_offs", np.int64, 2),
                               ("row_offs", np.int64, 2)], dev)
        self.workspace_bytes = int(_native.load().mvm_triplet_workspace_bytes(1, cap))
        self.workspace = torch.empty(max(self.workspace_bytes, 16), dtype=torch.uint8, device=dev)
        self.cube = torch.empty(cap ** 3, dtype=torch.float32, device=dev)
        self.argmin = torch.empty(cap * cap, dtype=torch.int32, device=dev)
        self.minval = torch.empty(cap * cap, dtype=torch.float32, device=dev)
        self.h_cube = torch.empty(cap ** 3, dtype=torch.float32, pin_memory=True)
        self.h_cube_np = self.h_cube.numpy()
        self.nbytes = (2 * self.stage.nbytes + self.workspace.numel() + 8 * cap ** 3 + 8 * cap * cap)
        self.dev = dev

    def run(self, views, Fs, pts: Optional[torch.Tensor] = None,
            cam_offs: Optional[torch.Tensor] = None, counts=None) -> np.ndarray:
        """-> a fresh float32 (N, M, P) array (owned by the caller).  ``pts`` /
        ``cam_offs``: device centroids and offsets of packed detections, with
        ``counts`` = (N, M, P) (``views`` is then not read)."""
        N, M, P = (int(c) for c in counts) if counts is not None else (len(v) for v in views)
        st = self.stage
        if pts is None:
            o = 0
            for v, k in zip(views, (N, M, P)):
                st.np["pts"][o:o + 2 * k] = np.asarray(v, np.float64).reshape(-1)
                o += 2 * k
        for q, f in enumerate(Fs):
            st.np["F"][9 * q:9 * q + 9] = np.asarray(f, np.float64).reshape(-1)
        st.np["cam_offs"][:] = (0, N, N + M, N + M + P)
        st.np["cube_offs"][:] = (0, N * M * P)
        st.np["row_offs"][:] = (0, N * M)
        cs = torch.cuda.current_stream(self.dev)
        stream = ctypes.c_void_p(cs.cuda_stream)
        st.upload()
        p_ptr = st.ptr("pts") if pts is None else _vp(pts)
        c_ptr = st.ptr("cam_offs") if cam_offs is None else _vp(cam_offs)
        rc = _native.load().mvm_triplet_cost_argmin(
            p_ptr, c_ptr, st.ptr("F"), 1, max(N, M, P), st.ptr("cube_offs"), st.ptr("row_offs"),
            _vp(self.cube), _vp(self.argmin), _vp(self.minval), _vp(self.workspace),
            self.workspace.numel(), stream)
        _native.check("mvm_triplet_cost_argmin", rc)
        n = N * M * P
        self.h_cube[:n].copy_(self.cube[:n], non_blocking=True)
        cs.synchronize()
        return self.h_cube_np[:n].reshape(N, M, P).copy()


class LsapSlot:
    """linear_sum_assignment of one matrix of at most ``rcap`` x ``ccap``
    entries of dtype float32/float64: each call's dims and plan offsets
    (mvm_lsap_plan_ex on the host) travel with its costs in the one staged
    copy, so every shape up to the capacity reuses the slot."""

    def __init__(self, rcap: int, ccap: int, dtype: torch.dtype, dev: torch.device):
        self.rcap, self.ccap = rcap, ccap
        self.dtype = dtype
        self.code = _native.MVM_F64 if dtype == torch.float64 else _native.MVM_F32
        self.np_dtype = np.float64 if dtype == torch.float64 else np.float32
        self.stage = _Staging([("dims", np.int64, 2), ("ws_offs", np.int64, 2),
                               ("out_offs", np.int64, 2), ("cost_offs", np.int64, 1),
                               ("cost", self.np_dtype, rcap * ccap)], dev)
        # the workspace layout depends on the shape's regime (a tall matrix
        # keeps a transposed copy) and grows with the dims inside a regime:
        # the capacity is the larger of the two regimes' largest shapes
        self.ws_capacity = max(self._plan(min(rcap, ccap), ccap),
                               self._plan(rcap, min(ccap, rcap - 1)) if rcap > 1 else 0)
        self.workspace = torch.empty(max(self.ws_capacity, 16), dtype=torch.uint8, device=dev)
        k = min(rcap, ccap)
        # outputs packed as [row_ind (k) | col_ind (k) | status (int32 in one int64 slot)]
        self.d_out = torch.zeros(2 * k + 1, dtype=torch.int64, device=dev)
        self.h_out = torch.empty(2 * k + 1, dtype=torch.int64, pin_memory=True)
        self.h_out_np = self.h_out.numpy()
        self.nbytes = 2 * self.stage.nbytes + self.workspace.numel() + 16 * (2 * k + 1)
        self.dev = dev

    def _plan(self, rows: int, cols: int, ws=None, out=None) -> int:
        r = np.array([rows], np.int64)
        c = np.array([cols], np.int64)
        ws = np.zeros(2, np.int64) if ws is None else ws
        out = np.zeros(2, np.int64) if out is None else out
        total = _native.load().mvm_lsap_plan_ex(1, r.ctypes.data, c.ctypes.data, self.code,
                                                 ws.ctypes.data, out.ctypes.data)
        if total < 0:
            raise _native.MvmError("mvm_lsap_plan_ex", -1,
                                   _native.load().mvm_last_error_string().decode())
        return int(total)

    def run(self, cost: np.ndarray) -> Tuple[np.ndarray, np.ndarray, int]:
        """-> (row_ind, col_ind, status) as scipy returns them (status 0 = ok)."""
        rows, cols = cost.shape
        k = min(rows, cols)
        st = self.stage
        total = self._plan(rows, cols, st.np["ws_offs"], st.np["out_offs"])
        if total > self.ws_capacity:      # not expected (layouts grow with the dims)
            raise RuntimeError(f"LsapSlot: workspace {total} > capacity {self.ws_capacity}")
        st.np["dims"][:] = (rows, cols)
        st.np["cost_offs"][0] = 0
        np.copyto(st.np["cost"][:rows * cols], cost.reshape(-1))
        cs = torch.cuda.current_stream(self.dev)
        stream = ctypes.c_void_p(cs.cuda_stream)
        st.upload("cost", rows * cols)     # the cost region is last: skip its unused tail
        long_side = max(rows, cols)
        rc = _native.load().mvm_lsap_solve_ex(
            st.ptr("cost"), self.code, st.ptr("cost_offs"), st.ptr("dims"), 1, st.ptr("ws_offs"),
            st.ptr("out_offs"), _vp(self.workspace), self.workspace.numel(), _vp(self.d_out),
            _vp(self.d_out, 8 * k), _vp(self.d_out, 16 * k), long_side, long_side, None, stream)
        _native.check("mvm_lsap_solve_ex", rc)
        self.h_out[:2 * k + 1].copy_(self.d_out[:2 * k + 1], non_blocking=True)
        cs.synchronize()
        out = self.h_out_np
        status = int(out[2 * k:2 * k + 1].view(np.int32)[0])
        return out[:k].copy(), out[k:2 * k].copy(), status


def cube_slot(N: int, M: int, P: int, dev: torch.device) -> CubeSlot:
    """The slot for a capture of (N, M, P) detections: views up to _SMALL_CAP
    share their capacity class's slot; larger ones get a slot of their own size."""
    n = max(N, M, P)
    cap = _cap(n) if n <= _SMALL_CAP else n
    return _lookup("cube", (dev.index, cap), lambda: CubeSlot(cap, dev))


def lsap_slot(rows: int, cols: int, dtype: torch.dtype, dev: torch.device) -> LsapSlot:
    """The slot for a rows x cols assignment: capacity classes of both sides up
    to _SMALL_CAP^3 cost entries (the flattened cube of _SMALL_CAP views), the
    exact shape above."""
    rc, cc = _cap(rows), _cap(cols)
    if rc * cc > _SMALL_CAP ** 3:
        rc, cc = rows, cols
    return _lookup("lsap", (dev.index, rc, cc, dtype), lambda: LsapSlot(rc, cc, dtype, dev))
