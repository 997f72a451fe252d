"""HBM write-probe variants (MVM_PROBE_MODE / MVM_PROBE_GRID), 4 GiB buffer, HIP events."""
import os, sys, subprocess, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

def one():
    import torch
    from bpc_baseline_amd import ops
    # MVM_PROBE_ELEMS: buffer size in float32s (default 1 GiElem = 4 GiB)
    buf = torch.empty(int(os.environ.get("MVM_PROBE_ELEMS", 1 << 30)), dtype=torch.float32, device="cuda")
    for _ in range(3):
        ops.hbm_write_probe(buf)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        ops.hbm_write_probe(buf)
    e1.record()
    torch.cuda.synchronize()
    t = e0.elapsed_time(e1) / 10 * 1e-3
    print(json.dumps({"mode": os.environ.get("MVM_PROBE_MODE", "17"), "grid": os.environ.get("MVM_PROBE_GRID", ""),
                      "lds": os.environ.get("MVM_PROBE_LDS", ""),
                      "rpw": os.environ.get("MVM_PROBE_RPW", ""), "rg": os.environ.get("MVM_PROBE_RG", ""),
                      "pace": os.environ.get("MVM_PROBE_PACE", ""),
                      "bytes": buf.numel() * 4, "ms": t * 1e3,
                      "TB/s": buf.numel() * 4 / t / 1e12}))

if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "one":
        one()
    else:
        modes = [(0, ""), (1, ""), (2, ""), (3, ""), (4, "1024"), (4, "2048"), (4, "4096"),
                 (5, "2048"), (5, "4096"), (6, ""), (7, ""), (8, ""), (9, ""), (10, ""), (11, ""), (12, ""), (13, ""), (14, ""), (15, ""), (16, ""), (17, ""), (18, "512"), (18, "768"), (18, "1024"), (18, "1536"), (18, "65472")]
        if len(sys.argv) > 1 and sys.argv[1] == "occupancy":
            # resident workgroups per CU capped by unused LDS: 8 (none), 4, 3, 2
            modes = [(m, "", l) for m in (17, 12) for l in (0, 40000, 50000, 60000)]
        elif len(sys.argv) > 1 and sys.argv[1] == "shape":
            # store shapes of candidate decompositions (write_probe_shape_kernel)
            modes = [(17, "", 0)] + [(m, "", 50000, rpw, rg) for m, rpw, rg in
                                      ((20, 16, 4), (20, 16, 1), (20, 8, 8), (20, 4, 16), (20, 4, 1),
                                       (21, 16, 16), (21, 16, 4), (21, 16, 1), (21, 32, 8), (21, 8, 32),
                                       (21, 64, 4))]
        elif len(sys.argv) > 1 and sys.argv[1] == "paced":
            # the same shapes with stores paced by s_sleep (stand-in for the arithmetic)
            modes = [(17, "", 0)] + [(20, "", 50000, rpw, rg, pace) for rpw, rg in
                                      ((16, 4), (16, 1), (4, 1), (4, 4)) for pace in (0, 1, 2, 4)]
        elif len(sys.argv) > 1:
            keep = set(int(x) for x in sys.argv[1].split(","))
            modes = [m for m in modes if m[0] in keep]
        for rep in range(2):
            for mode, grid, *lds in modes:
                env = dict(os.environ, MVM_PROBE_MODE=str(mode))
                if lds:
                    env["MVM_PROBE_LDS"] = str(lds[0])
                if len(lds) > 1:
                    env["MVM_PROBE_RPW"], env["MVM_PROBE_RG"] = str(lds[1]), str(lds[2])
                if len(lds) > 3:
                    env["MVM_PROBE_PACE"] = str(lds[3])
                if grid:
                    env["MVM_PROBE_GRID"] = grid
                subprocess.run([sys.executable, __file__, "one"], env=env, check=True, timeout=120)
