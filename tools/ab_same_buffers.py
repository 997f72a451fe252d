"""A/B of several in-tree builds of libmvmatch.so IN ONE PROCESS, each timed on
the SAME output buffers.  The launch time depends on where in HBM the output
lands (tools/probe_alloc.py: the same cube launch runs 2.38-2.45 ms on some
16.9 GB allocations and 2.95-2.99 ms on others), so builds compared in
separate processes are confounded by placement; here every build writes
every buffer, interleaved, and the table is per buffer.  The order of the
builds rotates every round: the build timed first on a buffer can differ from
the others by a few % for reasons of position alone.

python tools/ab_same_buffers.py --libs lib/a.so,lib/b.so [--workload cube|c3]
                                [--buffers 6] [--rounds 3]
Results of every build must be bit-identical (checked per buffer).
"""
import argparse
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bpc_baseline_amd import _native, ops  # noqa: E402
from bpc_baseline_amd.synth import make_scenes  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--libs", required=True)
ap.add_argument("--opts", default="default",
                help="semicolon list of option sets run with every build: default, or "
                     "comma-separated mvm_options fields, e.g. 'default;pairwise_row_groups=2'")
ap.add_argument("--workload", choices=["cube", "c3", "c2"], default="cube")
ap.add_argument("--buffers", type=int, default=6)
ap.add_argument("--rounds", type=int, default=3)
ap.add_argument("--no-check", action="store_true",
                help="skip the bit-equality check across builds (diagnostic builds, e.g. "
                     "tools/diag cheap_lines / no_assoc patches, compute other values)")
ap.add_argument("--scenes", type=int, default=None, help="scenes per launch (cube 250, c3 1000)")
ap.add_argument("--dets", default="256",
                help="detections per view (cube): one count, or N,M,P per view")
ap.add_argument("--alloc", default=None,
                help="comma list of buffer kinds instead of --buffers torch buffers: "
                     "torch | vmm:MB (HIP VMM API: physical chunks of MB MiB mapped contiguously)")
args = ap.parse_args()


class MemLocation(ctypes.Structure):
    _fields_ = [("type", ctypes.c_int), ("id", ctypes.c_int)]


class AllocFlags(ctypes.Structure):
    _fields_ = [("compressionType", ctypes.c_ubyte), ("gpuDirectRDMACapable", ctypes.c_ubyte),
                ("usage", ctypes.c_ushort)]


class AllocProp(ctypes.Structure):
    _fields_ = [("type", ctypes.c_int), ("requestedHandleType", ctypes.c_int),
                ("location", MemLocation), ("win32HandleMetaData", ctypes.c_void_p),
                ("allocFlags", AllocFlags)]


class AccessDesc(ctypes.Structure):
    _fields_ = [("location", MemLocation), ("flags", ctypes.c_int)]


class DevPtr:
    def __init__(self, ptr, n):
        self.__cuda_array_interface__ = {"shape": (n,), "typestr": "<f4", "data": (ptr, False),
                                         "version": 2}


def vmm_buffer(n, chunk_mb):
    """n float32 as physical chunks of chunk_mb MiB (hipMemCreate) mapped back to back."""
    hip = ctypes.CDLL("libamdhip64.so")
    prop = AllocProp()
    prop.type = 1                       # hipMemAllocationTypePinned
    prop.location = MemLocation(1, 0)   # hipMemLocationTypeDevice, device 0
    gran = ctypes.c_size_t()
    assert hip.hipMemGetAllocationGranularity(ctypes.byref(gran), ctypes.byref(prop), 1) == 0
    chunk = max(gran.value, chunk_mb << 20) // gran.value * gran.value
    size = (4 * n + chunk - 1) // chunk * chunk
    base = ctypes.c_void_p()
    assert hip.hipMemAddressReserve(ctypes.byref(base), ctypes.c_size_t(size),
                                    ctypes.c_size_t(max(chunk, 1 << 21)), None,
                                    ctypes.c_ulonglong(0)) == 0
    for off in range(0, size, chunk):
        h = ctypes.c_void_p()
        st = hip.hipMemCreate(ctypes.byref(h), ctypes.c_size_t(chunk), ctypes.byref(prop),
                              ctypes.c_ulonglong(0))
        assert st == 0, f"hipMemCreate {st}"
        assert hip.hipMemMap(ctypes.c_void_p(base.value + off), ctypes.c_size_t(chunk),
                             ctypes.c_size_t(0), h, ctypes.c_ulonglong(0)) == 0
    acc = AccessDesc(MemLocation(1, 0), 3)   # hipMemAccessFlagsProtReadWrite
    assert hip.hipMemSetAccess(base, ctypes.c_size_t(size), ctypes.byref(acc),
                               ctypes.c_size_t(1)) == 0
    print(f"vmm buffer: granularity {gran.value} B, chunk {chunk >> 20} MiB, "
          f"{size // chunk} chunks at 0x{base.value:x}")
    return torch.as_tensor(DevPtr(base.value, n), device=torch.device("cuda", 0))

def parse_opts(spec):
    if spec == "default":
        return None
    kw = dict(kv.split("=") for kv in spec.split(","))
    return _native.make_options(**{k: (int(v) if v.lstrip("-").isdigit() else v)
                                   for k, v in kw.items()})


opt_sets = {o: parse_opts(o) for o in args.opts.split(";")}
libs = {}
for path in args.libs.split(","):
    lib = ctypes.CDLL(os.path.abspath(path), mode=ctypes.RTLD_LOCAL)
    for name, (res, argt) in _native.SIGNATURES.items():
        fn = getattr(lib, name, None)   # older builds lack newer entry points
        if fn is not None:
            fn.restype, fn.argtypes = res, argt
    for o in opt_sets:   # one column per (build, option set)
        libs[os.path.basename(path) + ("" if o == "default" else f"[{o}]")] = (lib, opt_sets[o])

dev = torch.device("cuda", 0)
P = lambda t: ctypes.c_void_p(t.data_ptr())   # noqa: E731
if args.workload == "cube":
    dets = [int(x) for x in args.dets.split(",")]
    b = make_scenes(args.scenes or 250, 3, dets[0] if len(dets) == 1 else dets, seed=0)
    plan = ops.TripletPlan(b.cam_offs, b.n_scenes, device=dev)
    n_out = plan.n_cube
else:
    b = (make_scenes(args.scenes or 1000, 3, 256, seed=0) if args.workload == "c2"
         else make_scenes(args.scenes or 1000, 4, 1024, seed=0))
    plan = ops.PairwisePlan(b.cam_offs, b.n_scenes, b.n_cams, b.pairs, device=dev, row_align="auto")
    n_out = plan.dist_size
    pa = (ctypes.c_int32 * len(plan.pair_a))(*plan.pair_a)
    pb = (ctypes.c_int32 * len(plan.pair_b))(*plan.pair_b)
pts, co, F = (torch.from_numpy(x).to(dev) for x in (b.pts, b.cam_offs, b.F))
am = torch.empty(plan.n_rows, dtype=torch.int32, device=dev)
mv = torch.empty(plan.n_rows, dtype=torch.float32, device=dev)
stream = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)


def launch(entry, out):
    lib, opt = entry
    po = ctypes.byref(opt) if opt is not None else None
    if args.workload == "cube":
        st = lib.mvm_triplet_cost_argmin_ex(P(pts), P(co), P(F), plan.n_scenes, plan.max_n,
                                            P(plan.cube_offs), P(plan.row_offs), P(out), P(am),
                                            P(mv), P(plan.workspace), plan.workspace.numel(),
                                            po, stream)
    else:
        st = lib.mvm_pairwise_residual_argmin_ex(P(pts), P(co), P(F), pa, pb, plan.n_scenes,
                                                 plan.n_cams, len(plan.pair_a), plan.max_n,
                                                 P(plan.dist_offs), P(plan.row_offs), P(out),
                                                 P(am), P(mv), po, stream)
    assert st == 0, st


kinds = args.alloc.split(",") if args.alloc else ["torch"] * args.buffers
reps = 20 if args.workload == "c2" else 3
bufs = [torch.empty(n_out, dtype=torch.float32, device=dev) if k == "torch"
        else vmm_buffer(n_out, int(k.split(":")[1])) for k in kinds]
times = {(n, i): [] for n in libs for i in range(len(bufs))}
ptimes = {i: [] for i in range(len(bufs))}
ev = lambda: torch.cuda.Event(enable_timing=True)   # noqa: E731
for rnd in range(args.rounds + 1):
    names = list(libs)
    k = rnd % len(names)
    order = names[k:] + names[:k]   # rotate: every build takes every position (order bias)
    for i, out in enumerate(bufs):
        ref = None
        for name in order:
            lib = libs[name]
            launch(lib, out)
            e0, e1 = ev(), ev()
            e0.record()
            for _ in range(reps):
                launch(lib, out)
            e1.record()
            torch.cuda.synchronize()
            if rnd:
                times[(name, i)].append(e0.elapsed_time(e1) / reps)
            if rnd == 0 and not args.no_check:   # every build's results equal the first's
                chk = (am.cpu().numpy().tobytes(), out[:1 << 22].cpu().numpy().tobytes(),
                       out[-(1 << 22):].cpu().numpy().tobytes())
                if ref is None:
                    ref = chk
                assert chk == ref, f"{name} differs from the first build"
        q0, q1 = ev(), ev()
        q0.record()
        for _ in range(3):
            ops.hbm_write_probe(out)
        q1.record()
        torch.cuda.synchronize()
        if rnd:
            ptimes[i].append(q0.elapsed_time(q1) / 3)
print(f"{args.workload}: median ms per launch, per output buffer (probe = write probe on that buffer)")
print("buffer       probe   " + "  ".join(f"{n:>22}" for n in libs))
for i in range(len(bufs)):
    print(f"{i:>2} {kinds[i]:>8}  {np.median(ptimes[i]):.3f}  " +
          "  ".join(f"{np.median(times[(n, i)]):>22.3f}" for n in libs))
print("mean         " + f"{np.mean([np.median(ptimes[i]) for i in ptimes]):.3f}  " +
      "  ".join(f"{np.mean([np.median(times[(n, i)]) for i in range(len(bufs))]):>22.3f}"
                for n in libs))
