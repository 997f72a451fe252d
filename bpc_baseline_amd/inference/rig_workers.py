"""F and P of capture batches in worker PROCESSES (off the main process's GIL).

``match_captures`` needs, per capture, the three fundamental matrices
(camera_utils.py:23-46 of the reference, bit-identical only through numpy's
own BLAS calls) and the three projection matrices.  numpy issues one BLAS call
per 3x3 product, so for a batch of 1000 distinct rigs this is ~0.9 ms of host
time, most of it Python/numpy dispatch that holds the GIL -- a worker THREAD
overlaps little of it with the main thread's launches.

``RigWorkers`` runs ``rig_matrices`` (numpy, the same function, so the same
bits) in ``n`` child processes, each on a contiguous slice of the batch's
captures.  Inputs (Ks, RTs) and outputs (F, P) travel through shared memory;
a job is one short text line per worker over its stdin, answered on stdout.  ``submit`` returns at once;
``result`` waits and returns copies, so a pipeline can submit batch b+1
before it runs batch b.  Two shared-memory slots alternate, so one job may be
in flight while the previous job's result is read.  One job is in flight at a
time per pool: ``submit`` returns a ticket that ``result`` checks, and a lock
keeps two threads from interleaving the pool's state (each thread should hold
its own pool, as ``batch_match.rig_worker_pool`` gives it).
"""
from __future__ import annotations

import itertools
import threading
from multiprocessing import shared_memory
from typing import List, Optional, Tuple

import numpy as np

__all__ = ["RigWorkers"]


def _layout(S: int):
    """Byte offsets of Ks f32 [S,3,3,3], RTs f64 [S,3,4,4] | F f64 [S*3,9], P f64 [S,3,3,4]."""
    ks = S * 27 * 4
    rt_off = (ks + 63) // 64 * 64
    n_in = rt_off + S * 48 * 8
    f_bytes = S * 27 * 8
    p_off = (f_bytes + 63) // 64 * 64
    n_out = p_off + S * 36 * 8
    return rt_off, max(n_in, 8), p_off, max(n_out, 8)


def _views(S, shm_in, shm_out):
    rt_off, _, p_off, _ = _layout(S)
    Ks = np.ndarray((S, 3, 3, 3), np.float32, buffer=shm_in.buf, offset=0)
    RTs = np.ndarray((S, 3, 4, 4), np.float64, buffer=shm_in.buf, offset=rt_off)
    F = np.ndarray((S * 3, 9), np.float64, buffer=shm_out.buf, offset=0)
    P = np.ndarray((S, 3, 3, 4), np.float64, buffer=shm_out.buf, offset=p_off)
    return Ks, RTs, F, P


def _serve(inp, out) -> None:
    """Worker loop over text lines on stdin/stdout:
    "job IN OUT S I0 I1" -> F/P rows [I0, I1) of the slot, answered "ok" (or
    "err MESSAGE"); "forget NAME..." drops attached segments; EOF ends it."""
    from multiprocessing import resource_tracker
    from .utils.camera_utils import rig_matrices
    attached = {}

    def shm(name):
        if name not in attached:
            seg = shared_memory.SharedMemory(name=name)
            # the parent owns (and unlinks) the segment: do not let this
            # process's tracker unlink it when the worker exits
            resource_tracker.unregister(seg._name, "shared_memory")  # noqa: SLF001
            attached[name] = seg
        return attached[name]

    try:
        for line in inp:
            msg = line.split()
            if not msg:
                continue
            if msg[0] == "forget":            # the parent replaced a slot
                for name in msg[1:]:
                    seg = attached.pop(name, None)
                    if seg is not None:
                        seg.close()
                continue
            _, in_name, out_name, S, i0, i1 = msg
            S, i0, i1 = int(S), int(i0), int(i1)
            try:
                Ks, RTs, F, P = _views(S, shm(in_name), shm(out_name))
                if i1 > i0:
                    f, p = rig_matrices(Ks[i0:i1], RTs[i0:i1])
                    F[3 * i0:3 * i1] = f
                    P[i0:i1] = p
                    del f, p
                del Ks, RTs, F, P
                out.write("ok\n")
            except Exception as e:  # noqa: BLE001 -- reported to the parent
                out.write("err " + repr(e).replace("\n", " ") + "\n")
            out.flush()
    finally:
        for seg in attached.values():
            seg.close()


class _Slot:
    def __init__(self, S: int):
        _, n_in, _, n_out = _layout(S)
        self.S = S
        self.shm_in = shared_memory.SharedMemory(create=True, size=n_in)
        self.shm_out = shared_memory.SharedMemory(create=True, size=n_out)

    def close(self):
        for seg in (self.shm_in, self.shm_out):
            seg.close()
            seg.unlink()


class RigWorkers:
    """``n`` worker processes computing ``rig_matrices`` slices; see the module doc.

    Each worker is ``python -m bpc_baseline_amd.inference.rig_workers``, a
    child process that imports numpy and camera_utils only (no torch, no GPU,
    nothing of the parent's main module)."""

    def __init__(self, n: int = 2):
        import os
        import subprocess
        import sys
        root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        env = dict(os.environ)
        env["PYTHONPATH"] = root + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH") else "")
        env.setdefault("OMP_NUM_THREADS", "1")
        env.setdefault("OPENBLAS_NUM_THREADS", "1")
        self.procs = [subprocess.Popen([sys.executable, "-m", "bpc_baseline_amd.inference.rig_workers"],
                                       stdin=subprocess.PIPE, stdout=subprocess.PIPE, env=env,
                                       text=True, bufsize=1)
                      for _ in range(max(1, int(n)))]
        self.slots: List[Optional[_Slot]] = [None, None]
        self.next_slot = 0
        self.pending = None               # (ticket, slot index, S, workers used)
        self._tickets = itertools.count(1)
        self._lock = threading.Lock()

    def _send(self, w: int, line: str) -> None:
        self.procs[w].stdin.write(line + "\n")
        self.procs[w].stdin.flush()

    def _slot(self, S: int) -> int:
        k = self.next_slot
        self.next_slot ^= 1
        s = self.slots[k]
        if s is None or s.S < S:
            if s is not None:
                for w in range(len(self.procs)):
                    self._send(w, f"forget {s.shm_in.name} {s.shm_out.name}")
                s.close()
            self.slots[k] = _Slot(max(S, 1))
        return k

    def submit(self, Ks: np.ndarray, RTs: np.ndarray) -> int:
        """Start computing F/P of one batch (Ks f32 [S,3,3,3], RTs f64 [S,3,4,4]);
        returns the job's ticket."""
        with self._lock:
            return self._submit(Ks, RTs)

    def _submit(self, Ks, RTs) -> int:
        if not self.procs:
            raise RuntimeError("RigWorkers: closed")
        if self.pending is not None:
            raise RuntimeError("RigWorkers: collect the previous result first")
        Ks = np.asarray(Ks, dtype=np.float32)
        RTs = np.asarray(RTs, dtype=np.float64)
        S = int(Ks.shape[0])
        k = self._slot(S)
        slot = self.slots[k]
        Kv, Rv, _, _ = _views(slot.S, slot.shm_in, slot.shm_out)
        Kv[:S] = Ks.reshape(S, 3, 3, 3)
        Rv[:S] = RTs.reshape(S, 3, 4, 4)
        del Kv, Rv
        n = min(len(self.procs), max(S, 1))
        for w in range(n):
            i0, i1 = S * w // n, S * (w + 1) // n
            self._send(w, f"job {slot.shm_in.name} {slot.shm_out.name} {slot.S} {i0} {i1}")
        ticket = next(self._tickets)
        self.pending = (ticket, k, S, n)
        return ticket

    def result(self, ticket: Optional[int] = None) -> Tuple[np.ndarray, np.ndarray]:
        """-> (F f64 [S*3, 9], P f64 [S, 3, 3, 4]) of the submitted batch (copies).
        ``ticket`` (what ``submit`` returned), if given, must be the job in flight."""
        with self._lock:
            return self._result(ticket)

    def _result(self, ticket):
        if self.pending is None:
            raise RuntimeError("RigWorkers: nothing submitted")
        tk, k, S, n = self.pending
        if ticket is not None and ticket != tk:
            raise RuntimeError(f"RigWorkers: job {ticket} is not the one in flight ({tk})")
        self.pending = None
        replies = [self.procs[w].stdout.readline().strip() for w in range(n)]
        bad = [r for r in replies if r != "ok"]
        if bad:
            raise RuntimeError(f"RigWorkers: worker failed: {bad[0] or 'no reply (worker exited)'}")
        slot = self.slots[k]
        _, _, F, P = _views(slot.S, slot.shm_in, slot.shm_out)
        out = np.array(F[:3 * S]), np.array(P[:S])
        del F, P
        return out

    def drain(self) -> None:
        """Collect and drop the job in flight, if any (a consumer that stopped
        early leaves the pool ready for the next submit)."""
        with self._lock:
            if self.pending is not None:
                try:
                    self._result(None)
                except RuntimeError:
                    pass

    def close(self) -> None:
        self.drain()
        for p in self.procs:
            try:
                p.stdin.close()
            except OSError:
                pass
        for p in self.procs:
            try:
                p.wait(timeout=10)
            except Exception:  # noqa: BLE001
                p.kill()
            if p.stdout:
                p.stdout.close()
        self.procs = []
        for s in self.slots:
            if s is not None:
                s.close()
        self.slots = [None, None]

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


if __name__ == "__main__":
    import sys
    _serve(sys.stdin, sys.stdout)
