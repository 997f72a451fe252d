"""Batched, device-resident matching of many 3-camera captures.

The reference processes one capture at a time through host Python:
``PoseEstimator._detect`` packs YOLO boxes into dicts (process_pose.py:116-142),
``_match`` builds F12/F13/F23, the cost cube, the assignment, the threshold
filter and the cost sort (:144-183), and ``PosePrediction`` triangulates each
match (:79-94).  ``match_captures`` runs the same steps for S captures at once
with every O(n) and larger step on the GPU:

  1. mvm_pack_detections      boxes/conf/cls -> half-integer centroids (CSR)
  2. host                     F (batched, bit-equal to compute_fundamental_matrix)
                              and P = K @ RT[:3]; O(1) per capture
  3. mvm_triplet_cost_argmin  the (N, M, P) cube of every capture (+ its 8-row
                              minima when an assignment is large: _bmin8)
  4. mvm_lsap_solve           scipy-identical assignment of every flattened cube
  5. mvm_select_triangulate   cost < threshold, stable sort by cost, DLT

The only device->host transfer before the results is the per-image kept
count (n_img int32, with the packing status), which sizes the cube and
assignment layouts; the results need one more (statuses + match counts).

Results equal, capture by capture, the reference's ``_match`` outputs fed with
``_detect``'s detections: match indices and order exactly, ``t`` to rounding
(tests/test_batch_match_gpu.py).
"""
from __future__ import annotations

import threading
import weakref
from dataclasses import dataclass
from typing import Iterable, Iterator, List, Optional, Sequence

import numpy as np
import torch

from .. import ops
from .utils.camera_utils import projection_matrices, rig_matrices

__all__ = ["MatchBatch", "match_capture_stream", "match_captures", "projection_matrices",
           "rig_matrices", "rig_worker_pool"]


@dataclass
class MatchBatch:
    """Device results of ``match_captures`` (scene s owns rows
    ``offs[s] : offs[s] + count[s]`` of match / cost / X)."""
    match: torch.Tensor          # int32 [cap, 3]   (i, j, k) per match
    cost: torch.Tensor           # float32 [cap]    cube value of the match
    X: torch.Tensor              # float64 [cap, 3] triangulated centre
    count: np.ndarray            # int32 [S]
    offs: np.ndarray             # int64 [S + 1]
    pts: torch.Tensor            # float64 [n, 2]   packed centroids
    boxes: torch.Tensor          # int32 [n, 4]     packed int boxes
    cam_offs: np.ndarray         # int64 [3S + 1]   CSR of pts / boxes
    cube: Optional[torch.Tensor] = None

    def host(self) -> dict:
        """One D2H copy of everything ``predictions`` reads."""
        if not hasattr(self, "_host"):
            self._host = {k: getattr(self, k).cpu().numpy() for k in ("match", "cost", "X", "pts", "boxes")}
        return self._host

    def predictions(self, s: int) -> List[tuple]:
        """Scene s as the reference's PosePrediction fields, in _match's order:
        list of (boxes int32 [3, 4], centroids f64 [3, 2], t f64 [3])."""
        o, n = int(self.offs[s]), int(self.count[s])
        h = self.host()
        rows = self.cam_offs[3 * s:3 * s + 3][None, :] + h["match"][o:o + n].astype(np.int64)
        return [(h["boxes"][rows[q]], h["pts"][rows[q]], h["X"][o + q]) for q in range(n)]


def match_captures(boxes: torch.Tensor, conf: torch.Tensor, cls: torch.Tensor,
                   img_offs: torch.Tensor, Ks: np.ndarray, RTs: np.ndarray, *,
                   conf_thresh: float = 0.1, matching_threshold: float = 30,
                   keep_cube: bool = False, timings: Optional[dict] = None,
                   F: Optional[torch.Tensor] = None,
                   proj: Optional[torch.Tensor] = None) -> MatchBatch:
    """Detect-packing + matching + triangulation of S 3-camera captures.

    ``boxes`` f32 [n, 4] xyxy, ``conf``/``cls`` f32 [n]: the detector outputs
    of the 3S images (capture s, camera c = image 3s + c) concatenated on the
    device; ``img_offs`` int64 [3S + 1] device.  ``Ks`` float32 [S, 3, 3, 3],
    ``RTs`` float64 [S, 3, 4, 4] (host).  Defaults are PoseEstimatorParams'
    (process_pose.py:36-37).

    ``F`` (f64 [S*3, 9], F12/F13/F23 per capture) and ``proj`` (f64 [S, 3, 3, 4])
    may be passed as device tensors when the rigs repeat across batches (a
    static camera rig): they are then not recomputed on the host.  They must
    be what ``fundamental_matrices_batched`` / ``projection_matrices`` return.
    """
    dev = boxes.device
    import time
    clock = [time.perf_counter()]

    def mark(name):                      # optional stage timings (synchronising)
        if timings is not None:
            torch.cuda.synchronize(dev)
            now = time.perf_counter()
            timings[name] = timings.get(name, 0.0) + now - clock[0]
            clock[0] = now

    n_img = int(img_offs.numel()) - 1
    if n_img % 3:
        raise ValueError("img_offs must describe 3 images per capture")
    S = n_img // 3
    Ks = np.asarray(Ks, dtype=np.float32).reshape(S, 3, 3, 3)
    RTs = np.asarray(RTs, dtype=np.float64).reshape(S, 3, 4, 4)

    pts, cam_offs, boxes_int, counts, status = ops.pack_detections(boxes, conf, cls, img_offs,
                                                                   conf_thresh)
    mark("pack")
    # host work while the packing runs: F and P for every capture (once per
    # distinct rig)
    if F is None or proj is None:
        F_h, P_h = rig_matrices(Ks, RTs)
        if F is None:
            F = torch.from_numpy(F_h).to(dev)
        if proj is None:
            proj = torch.from_numpy(P_h).to(dev)
    F_dev = F.reshape(-1)
    proj_dev = proj
    mark("F+P host")

    # one device -> host copy: the kept counts and the packing status
    ch = torch.cat([counts, status]).cpu().numpy().astype(np.int64)
    counts_host = ch[:-1]
    if ch[-1] != 0:
        raise ValueError("detector box with a non-finite or out-of-range coordinate")
    cam_offs_host = np.zeros(n_img + 1, np.int64)
    np.cumsum(counts_host, out=cam_offs_host[1:])
    mark("counts D2H")

    c3 = counts_host.reshape(S, 3)
    free = ops.cube_free_scenes(c3) if not keep_cube else np.zeros(S, bool)
    if free.all() or not free.any():
        res = _device_chain(pts, cam_offs, cam_offs_host, F_dev, proj_dev, S, float(matching_threshold),
                            bool(free.all()) and S > 0, keep_cube, mark)
    else:
        # a mixed batch: the scenes of the candidate-list class without the
        # cube, the others (small views: the dense assignment classes read
        # the cost) with it; each part is a contiguous sub-batch
        res = _split_chain(pts, cam_offs_host, F_dev, proj_dev, S, float(matching_threshold), free,
                           mark)
    match, cost, X, lstat, count, out_offs_host, cube = res
    # one device -> host copy: assignment statuses and match counts
    sc = torch.cat([lstat, count]).cpu().numpy()
    bad, count_h = sc[:S], sc[S:]
    if np.any(bad):
        raise ValueError(f"assignment failed for captures {np.nonzero(bad)[0][:8].tolist()} "
                         "(cost matrix contains invalid numeric entries or is infeasible)")
    mark("results D2H")
    return MatchBatch(match=match, cost=cost, X=X, count=count_h,
                      offs=out_offs_host, pts=pts, boxes=boxes_int, cam_offs=cam_offs_host,
                      cube=cube if keep_cube else None)


def _device_chain(pts, cam_offs, cam_offs_host, F_dev, proj_dev, S, threshold, cube_free, keep_cube,
                  mark):
    """Cube (or, cube_free, its 8-row minima + pair residuals) -> assignment ->
    select/DLT of S scenes whose CSR offsets are ``cam_offs`` (device) /
    ``cam_offs_host``.  -> (match, cost, X, status, count, out_offs_host, cube or None)."""
    dev = pts.device
    plan = ops.TripletPlan(cam_offs_host, S, device=dev)
    c3 = plan.counts
    mark("cube plan")
    if cube_free:
        # the assignment never reads a cube: the 32-column block minima its
        # candidate lists start from and the fp64 pair residuals it recomputes
        # its entries from (no 8-row minima: the lists gather
        # whole candidate blocks)
        minima = ops.triplet_minima(pts, cam_offs, F_dev, plan, with_bmin8=False)
        mark("cube")
        lplan = ops.LsapPlan(c3[:, 0] * c3[:, 1], c3[:, 2], device=dev, resid=True)
        mark("lsap plan")
        row_ind, col_ind, lstat = ops.linear_sum_assignment_resid(lplan, plan, minima)
        mark("lsap")
        match, cost, X, count = ops.select_triangulate_resid(plan, cam_offs, lplan.out_offs, row_ind,
                                                             col_ind, pts, proj_dev, threshold)
        mark("select")
        return match, cost, X, lstat, count, lplan.out_offs_host, None
    # flattened cubes of the candidate-list class: the cube kernel also writes
    # the 8-row minima that class reduces
    bm8 = None
    lo, hi, sh = ops.sparse_class_bounds()
    nm = c3[:, 0] * c3[:, 1]
    if S and bool(((nm >= lo) & (nm > 1024) & (nm <= hi) & (c3[:, 2] <= sh) & (nm > c3[:, 2])).any()):
        bm8 = torch.empty(max(plan.n_bmin8, 1), dtype=torch.int16, device=dev)
    cube, _, _ = ops.triplet_cost_argmin(pts, cam_offs, F_dev, plan, bmin8=bm8)
    mark("cube")
    lplan = ops.LsapPlan(nm, c3[:, 2], device=dev)
    mark("lsap plan")
    row_ind, col_ind, lstat = ops.linear_sum_assignment_batched(
        cube, plan.cube_offs[:-1].contiguous(), lplan,
        bmin8=(bm8, plan.bmin8_offs, plan.segs) if bm8 is not None else None)
    mark("lsap")
    match, cost, X, count = ops.select_triangulate(cube, plan.cube_offs, cam_offs, lplan.out_offs,
                                                   row_ind, col_ind, pts, proj_dev, threshold)
    mark("select")
    return match, cost, X, lstat, count, lplan.out_offs_host, (cube if keep_cube else None)


def _split_chain(pts, cam_offs_host, F_dev, proj_dev, S, threshold, free, mark):
    """_device_chain over the cube-free scenes and the others as two
    contiguous sub-batches (their centroids, F and P gathered on the device),
    merged back into the batch's scene order and assignment offsets."""
    dev = pts.device
    co = np.asarray(cam_offs_host, np.int64)
    c3 = np.diff(co).reshape(S, 3)
    caps = np.minimum(c3[:, 0] * c3[:, 1], c3[:, 2])
    out_offs = np.zeros(S + 1, np.int64)
    np.cumsum(caps, out=out_offs[1:])
    cap = int(out_offs[-1])
    match = torch.zeros((max(cap, 1), 3), dtype=torch.int32, device=dev)
    cost = torch.zeros(max(cap, 1), dtype=torch.float32, device=dev)
    X = torch.zeros((max(cap, 1), 3), dtype=torch.float64, device=dev)
    status = torch.zeros(S, dtype=torch.int32, device=dev)
    count = torch.zeros(S, dtype=torch.int32, device=dev)
    F3 = F_dev.reshape(S, 27)
    for part in (np.nonzero(free)[0], np.nonzero(~free)[0]):
        if part.size == 0:
            continue
        rows = np.concatenate([np.arange(co[3 * s], co[3 * s + 3]) for s in part]).astype(np.int64)
        sub_co = np.zeros(3 * part.size + 1, np.int64)
        np.cumsum(c3[part].reshape(-1), out=sub_co[1:])
        sel, idx, dst_rows, src_rows, sub_co_dev = ops._h2d_int64(
            [rows, part.astype(np.int64),
             np.concatenate([np.arange(out_offs[s], out_offs[s] + caps[s]) for s in part]).astype(np.int64),
             np.arange(int(caps[part].sum()), dtype=np.int64), sub_co], dev)
        sub_pts = pts.index_select(0, sel) if rows.size else pts[:0]
        m, c, x, st, n, _, _ = _device_chain(sub_pts, sub_co_dev, sub_co,
                                             F3.index_select(0, idx).reshape(-1),
                                             proj_dev.index_select(0, idx), part.size, threshold,
                                             bool(free[part[0]]), False, mark)
        if src_rows.numel():
            match.index_copy_(0, dst_rows, m.index_select(0, src_rows))
            cost.index_copy_(0, dst_rows, c.index_select(0, src_rows))
            X.index_copy_(0, dst_rows, x.index_select(0, src_rows))
        status.index_copy_(0, idx, st)
        count.index_copy_(0, idx, n)
    return match[:cap], cost[:cap], X[:cap], status, count, out_offs, None


def _rig_inputs(batch: Sequence):
    """(Ks f32 [S,3,3,3], RTs f64 [S,3,4,4]) of one ``match_capture_stream`` batch."""
    boxes, conf, cls, img_offs, Ks, RTs = batch
    S = (int(img_offs.numel()) - 1) // 3
    return (np.asarray(Ks, dtype=np.float32).reshape(S, 3, 3, 3),
            np.asarray(RTs, dtype=np.float64).reshape(S, 3, 4, 4))


_TLS = threading.local()


class _ThreadPools:
    """One thread's RigWorkers by size.  Its finalizer closes them when the
    thread ends (its thread-local storage, the only strong reference to this
    holder, is released) or at interpreter exit, whichever comes first: a
    service that starts a thread per request does not accumulate worker
    processes or shared-memory slots."""

    def __init__(self):
        self.by_n = {}
        weakref.finalize(self, _ThreadPools._close_all, self.by_n)

    @staticmethod
    def _close_all(by_n):
        for pool in list(by_n.values()):
            pool.close()
        by_n.clear()


def rig_worker_pool(n: int):
    """The calling thread's ``RigWorkers`` of ``n`` processes (started on first
    use, reused by every stream of that thread, closed when the thread ends or
    at exit).  Per thread: a pool has one job in flight, and two threads
    streaming at once must not share it."""
    from .rig_workers import RigWorkers
    holder = getattr(_TLS, "pools", None)
    if holder is None:
        holder = _TLS.pools = _ThreadPools()
    pool = holder.by_n.get(n)
    if pool is None or not pool.procs:      # first use, or closed
        pool = holder.by_n[n] = RigWorkers(n)
    return pool


def match_capture_stream(batches: Iterable[Sequence], *, rig_workers: int = 3,
                         **kwargs) -> Iterator[MatchBatch]:
    """``match_captures`` over a sequence of batches, pipelined: the host F and
    P of batch b+1 (``rig_matrices``: numpy, the same function, so the same
    bits) are computed by ``rig_workers`` worker PROCESSES
    (``rig_workers.RigWorkers``, shared memory) while the main process runs
    batch b's device chain -- off its GIL, which a worker thread was not
    (DESIGN.md §3.10).  ``rig_workers=0`` computes them inline.  Each batch is
    ``(boxes, conf, cls, img_offs, Ks, RTs)`` as ``match_captures`` takes them;
    ``kwargs`` are passed through (``F`` / ``proj`` are computed here).
    Results equal ``match_captures`` on each batch.
    """
    if "F" in kwargs or "proj" in kwargs:
        raise TypeError("match_capture_stream computes F and proj itself")
    it = iter(batches)
    cur = next(it, None)
    if cur is None:
        return
    pool = rig_worker_pool(rig_workers) if rig_workers > 0 else None
    try:
        ticket = pool.submit(*_rig_inputs(cur)) if pool is not None else None
        while cur is not None:
            F_h, P_h = pool.result(ticket) if pool is not None else rig_matrices(*_rig_inputs(cur))
            nxt = next(it, None)
            if nxt is not None and pool is not None:
                ticket = pool.submit(*_rig_inputs(nxt))   # batch b+1's F/P while batch b runs
            dev = cur[0].device
            yield match_captures(*cur, F=torch.from_numpy(F_h).to(dev),
                                 proj=torch.from_numpy(P_h).to(dev), **kwargs)
            cur = nxt
    finally:
        # a consumer that stops early (break, exception, the generator
        # collected) leaves batch b+1's job in flight: collect it, so the
        # thread's pool takes the next stream's submit
        if pool is not None:
            pool.drain()
