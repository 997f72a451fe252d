"""Multi-rank path on CPU (gloo, world_size 2): scene sharding + the single
association gather reproduce the single-process result exactly.  The GPU
kernel is replaced by the oracle here (CPU-only test of the sharding logic;
the HIP kernel's parity is covered by the -m gpu tests)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, n_scenes, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from bpc_baseline_amd.distributed import init_from_env, shard_range, gather_rows, max_over_ranks
    from bpc_baseline_amd.synth import make_scenes
    from oracle import oracle as O
    env = init_from_env(backend="gloo", use_gpu=False)
    a, b = shard_range(n_scenes, env.rank, env.world)
    batch = make_scenes(b - a, 4, 23, seed=5, first_scene=a, ragged=True)
    _, am, mv, _, _ = O.pairwise(batch.pts, batch.cam_offs, batch.F, batch.pairs, batch.n_scenes,
                                 batch.n_cams, want_dist=False)
    got = gather_rows(env, torch.from_numpy(am), torch.from_numpy(mv))
    t = max_over_ranks(env, float(env.rank + 1))
    if env.is_root:
        np.save(os.path.join(out_dir, "argmin.npy"), got[0].numpy())
        np.save(os.path.join(out_dir, "minval.npy"), got[1].numpy())
        np.save(os.path.join(out_dir, "tmax.npy"), np.array([t]))
    env.barrier()
    torch.distributed.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 4, 8])
def test_sharded_gather_equals_single_process(tmp_path, world):
    from bpc_baseline_amd.synth import make_scenes
    from oracle import oracle as O
    n_scenes = 7
    mp.spawn(_worker, args=(world, _free_port(), n_scenes, str(tmp_path)), nprocs=world, join=True)
    full = make_scenes(n_scenes, 4, 23, seed=5, ragged=True)
    _, am, mv, _, _ = O.pairwise(full.pts, full.cam_offs, full.F, full.pairs, n_scenes, 4,
                                 want_dist=False)
    assert np.array_equal(np.load(tmp_path / "argmin.npy"), am)
    assert np.array_equal(np.load(tmp_path / "minval.npy").view(np.int32), mv.view(np.int32))
    assert float(np.load(tmp_path / "tmax.npy")[0]) == world


def _chunked_worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from bpc_baseline_amd.distributed import init_from_env, ChunkedRowGather
    env = init_from_env(backend="gloo", use_gpu=False)
    n = 103
    a = torch.arange(n, dtype=torch.int32) + 1000 * rank
    m = torch.arange(n, dtype=torch.float32) * 0.5 + rank
    pieces = [(0, 40), (40, 41), (41, 103)]
    g = ChunkedRowGather(env, (a, m), pieces)
    for k in range(len(pieces)):
        g.issue(k)
    recv = g.finish()
    if env.is_root:
        np.save(os.path.join(out_dir, "a.npy"), recv[0].numpy())
        np.save(os.path.join(out_dir, "m.npy"), recv[1].numpy())
    env.barrier()
    torch.distributed.destroy_process_group()


def test_chunked_gather_pieces(tmp_path):
    world = 2
    mp.spawn(_chunked_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    a = np.load(tmp_path / "a.npy")
    m = np.load(tmp_path / "m.npy")
    for r in range(world):
        assert np.array_equal(a[r], np.arange(103) + 1000 * r)
        assert np.array_equal(m[r], np.arange(103, dtype=np.float32) * 0.5 + r)


@pytest.mark.gpu
def test_bench_rccl_process_group_single_rank(tmp_path):
    """bench.py with the RCCL ("nccl") process group forced at world 1: the
    device-bound group, the per-launch async gathers into rank 0's receive
    buffers and the barriers all run on the real backend; the gathered rows
    equal the local association and the last launch is bit-exact vs the oracle."""
    import json
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, MVM_DIST_FORCE="1", MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(_free_port()))
    env.pop("MVM_DIST_BACKEND", None)
    r = subprocess.run([sys.executable, os.path.join(repo, "bench.py"), "--scenes", "40",
                        "--chunk", "20", "--steps", "1", "--warmup", "1", "--cpu-seconds", "0"],
                       env=env, capture_output=True, text=True, timeout=300, cwd=repo)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    rows = line["parity_rows_detail"]["rows_checked"]
    assert rows == 40 * 6 * 1024
    assert line["parity_rows"] == f"{rows}/{rows} bit-exact vs oracle"
    assert line["parity"].startswith("bit-exact")
    assert "nccl" in line["config"]["parallelism"]


def _run_bench(repo, argv, env, tmp_path, name):
    import subprocess
    import sys
    r = subprocess.run(argv, env=env, capture_output=True, text=True, timeout=400, cwd=repo)
    (tmp_path / f"{name}.err").write_text(r.stderr)
    assert r.returncode == 0, f"{name}: rc {r.returncode}\n{r.stderr[-3000:]}"
    import json
    return json.loads(r.stdout.strip().splitlines()[-1])


@pytest.mark.gpu
@pytest.mark.parametrize("world,n_scenes", [(2, 24), (2, 25), (4, 21), (8, 40)])
def test_ranks_real_kernel_equal_single_process(tmp_path, world, n_scenes):
    """bench.py under torchrun with 2 (4, 8) ranks sharing the one GPU (gloo group):
    each rank runs libmvmatch.so's pairwise kernel on its own scene shard, the
    association rows are gathered to rank 0 (chunked async gathers for equal
    shards, the one-shot padded gather for 13 + 12 scenes), and rank 0's
    gathered rows equal a single-process run of the same scenes bit for bit,
    and the oracle's np.argmin rows (process_pose.py:154-159: scenes are
    independent, so sharding must not change any row)."""
    import sys
    from bpc_baseline_amd.synth import make_scenes
    from oracle import oracle as O
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    common = ["--workload", "c3", "--scenes", str(n_scenes), "--chunk", "8", "--steps", "1",
              "--warmup", "1", "--cpu-seconds", "0"]
    env1 = dict(os.environ)
    for k in ("MVM_DIST_FORCE", "MVM_DIST_BACKEND", "WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env1.pop(k, None)
    single = _run_bench(repo, [sys.executable, "bench.py", *common,
                               "--dump-association", str(tmp_path / "single")],
                        env1, tmp_path, "single")
    env2 = dict(env1, MVM_DIST_BACKEND="gloo")
    multi = _run_bench(repo, [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                              "--nproc-per-node", str(world), "--master-addr", "127.0.0.1",
                              "--master-port", str(_free_port()), "bench.py", "--gpus", str(world),
                              *common, "--cpu-seconds", "1",
                              "--dump-association", str(tmp_path / "multi")],
                       env2, tmp_path, "multi")
    assert multi["n_gpus"] == world
    assert multi["process_group"]["world_size"] == world
    assert multi["process_group"]["backend"] == "gloo"
    assert multi["config"]["n_scenes_total"] == n_scenes
    rows = n_scenes * 6 * 1024
    for line in (single, multi):     # every rank's rows, as gathered to rank 0
        assert line["parity_rows"] == f"{rows}/{rows} bit-exact vs oracle"
    assert multi["parity_rows_detail"]["ranks"] == world
    assert multi["parity"].startswith("bit-exact") and single["parity"].startswith("bit-exact")
    assert multi["step_split"]["gather_ms"] > 0
    # the N > 1 line carries what the N = 1 line does, measured the same way:
    # the same launch path (one hipGraph per launch), a CPU baseline, and a
    # roofline over the slowest rank next to rank 0's
    assert single["config"]["launch_mode"] == multi["config"]["launch_mode"] == "launch"
    assert single["config"]["launch"] == multi["config"]["launch"]
    assert multi["cpu_baseline"] and multi["cpu_baseline"]["value"] > 0
    assert multi["cpu_baseline"]["cores"] >= 1
    rf = multi["roofline"]
    assert rf["ranks"].startswith("slowest rank")
    assert rf["avg_launch_ms"] >= rf["rank0"]["avg_launch_ms"] > 0
    assert rf["achieved"] <= rf["rank0"]["achieved"]
    assert 0 <= multi["step_split"]["exposed_tail_ms"]
    assert multi["step_split"]["exposed_tail_frac"] >= 0
    assert multi["config"]["launches_per_step"] >= min(5, n_scenes // world)
    a1 = np.load(tmp_path / "single" / "argmin.npy")
    m1 = np.load(tmp_path / "single" / "minval.npy")
    a2 = np.load(tmp_path / "multi" / "argmin.npy")
    m2 = np.load(tmp_path / "multi" / "minval.npy")
    assert np.array_equal(a1, a2)
    assert np.array_equal(m1.view(np.int32), m2.view(np.int32))
    b = make_scenes(n_scenes, 4, 1024, seed=0)
    _, ra, rm, _, _ = O.pairwise(b.pts, b.cam_offs, b.F, b.pairs, n_scenes, 4, want_dist=False)
    assert np.array_equal(a2, ra)
    assert np.array_equal(m2.view(np.int32), rm.view(np.int32))


@pytest.mark.gpu
@pytest.mark.parametrize("workload,mode", [("c3", "steps"), ("c2cube", "steps"),
                                           ("c3", "launch"), ("c2cube", "launch"),
                                           ("c3", "steps2"), ("c3", "steps2-3")])
def test_bench_graph_replay_single_gpu(tmp_path, workload, mode):
    """bench.py's single-GPU timed steps as hipGraph replays (one graph for the
    K steps, or one per launch): the captured launches of every step run (the
    last launch's outputs are bit-exact vs the oracle), the per-launch event
    average covers every launch of every step, and the dispatch window says
    which of the kernel's launches a profile of the run must average."""
    import json
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ)
    env.pop("MVM_DIST_FORCE", None)
    # steps2-3: three steps on two streams (the last one odd-numbered: even),
    # steps2 with two (the last one on the second stream's association rows)
    mode, steps = (mode.split("-")[0], int(mode.split("-")[1])) if "-" in mode else (mode, 2)
    r = subprocess.run([sys.executable, os.path.join(repo, "bench.py"), "--workload", workload,
                        "--scenes", "24", "--chunk", "8", "--steps", str(steps), "--warmup", "1",
                        "--cpu-seconds", "0", "--graph", mode],
                       env=env, capture_output=True, text=True, timeout=300, cwd=repo)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["parity"].startswith("bit-exact")
    pr = line["parity_rows"]          # "ok/total bit-exact vs oracle" (a mismatch exits 3)
    assert pr is None or pr.split("/")[0] == pr.split("/")[1].split()[0]
    assert line["config"]["launch_mode"] == mode
    assert line["config"]["launch"].startswith("one hipGraph holding the K steps" if mode.startswith("steps")
                                               else "one hipGraph per launch")
    assert line["config"]["launches_per_step"] == 3
    assert line["roofline"]["avg_launch_ms"] > 0
    w = line["roofline"]["dispatch_window"]
    # warmup step (3) + the untimed first replay (K steps x 3) | K x 3 timed | PCIe leg (3)
    # + the kernel timed alone (five launches, kernel_isolated)
    assert (w["before"], w["timed"], w["after"]) == (3 + 3 * steps, 3 * steps, 3 + 5)


def _bench_env():
    env = dict(os.environ)
    for k in ("MVM_DIST_FORCE", "MVM_DIST_BACKEND", "WORLD_SIZE", "RANK", "LOCAL_RANK",
              "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    return env


@pytest.mark.parametrize("world", [2, 4])
def test_bench_launches_its_own_ranks(tmp_path, world):
    """`python bench.py --gpus N` with no launcher starts N ranks itself (torchrun
    as a child process) and every rank joins one process group of N."""
    import json
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "bench.py", "--gpus", str(world), "--dry-run"],
                       env=_bench_env(), capture_output=True, text=True, timeout=300, cwd=repo)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == world
    assert line["process_group"] == {"world_size": world, "backend": "gloo"}
    assert line["ranks_seen"] == list(range(world))
    assert f"launching {world} ranks" in r.stderr


@pytest.mark.parametrize("env_world,gpus", [("3", 2), ("1", 2), ("2", 1)])
def test_bench_world_mismatch_fails(env_world, gpus):
    """A process group whose size is not --gpus ends the run non-zero (never
    a line with another n_gpus than asked for)."""
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(_bench_env(), WORLD_SIZE=env_world, RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, "bench.py", "--gpus", str(gpus), "--dry-run"],
                       env=env, capture_output=True, text=True, timeout=120, cwd=repo)
    assert r.returncode != 0
    assert f"--gpus {gpus} but WORLD_SIZE={env_world}" in r.stderr
    assert not r.stdout.strip()


def test_init_timeout_reaches_process_group(tmp_path):
    """init_from_env gives the process group a finite collective timeout."""
    mp.spawn(_timeout_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    assert float((tmp_path / "timeout").read_text()) == 7.0


def _timeout_worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from bpc_baseline_amd.distributed import init_from_env
    env = init_from_env(backend="gloo", use_gpu=False, timeout_s=7)
    if env.is_root:
        with open(os.path.join(out_dir, "timeout"), "w") as fh:
            fh.write(str(env.timeout.total_seconds()))
    env.barrier()
    torch.distributed.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2])
def test_bench_gpus_n_without_launcher(tmp_path, world):
    """`MVM_DIST_BACKEND=gloo python bench.py --gpus 2` with no launcher prefix:
    bench.py starts the ranks itself, the line says n_gpus 2 with a process
    group of 2, and every gathered association row is bit-exact vs the oracle."""
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(_bench_env(), MVM_DIST_BACKEND="gloo")
    n_scenes = 24
    line = _run_bench(repo, [sys.executable, "bench.py", "--gpus", str(world), "--scenes",
                             str(n_scenes), "--chunk", "8", "--steps", "1", "--warmup", "1",
                             "--cpu-seconds", "0"], env, tmp_path, "nolauncher")
    assert line["n_gpus"] == world
    assert line["process_group"]["world_size"] == world
    rows = n_scenes * 6 * 1024
    assert line["parity_rows"] == f"{rows}/{rows} bit-exact vs oracle"
    assert line["roofline"]["per_slot"]["slots"]


@pytest.mark.gpu
@pytest.mark.parametrize("cube,extra", [("free", []), ("free", ["--match-pipeline", "on"]),
                                        ("free", ["--lsap-input", "bmin8"]), ("keep", [])])
def test_bench_c2match_line_small(cube, extra):
    """bench.py --workload c2match on a small batch: the line's own parity
    against the CPU chain (block keys or cube, residuals, assignment, matches,
    costs, X) holds in every mode, serial or with consecutive steps
    overlapped, with and without the 8-row minima, with and without the cube."""
    import json
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ)
    env.pop("MVM_DIST_FORCE", None)
    r = subprocess.run([sys.executable, os.path.join(repo, "bench.py"), "--workload", "c2match",
                        "--scenes", "24", "--steps", "3", "--warmup", "1", "--cpu-seconds", "0",
                        "--cube", cube, *extra],
                       env=env, capture_output=True, text=True, timeout=300, cwd=repo)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["parity"].startswith("equal vs the CPU chain"), line["parity"]
    assert all(all(v for k, v in d.items() if k != "scene" and k != "matches")
               for d in line["parity_detail"]), line["parity_detail"]
    assert line["value"] > 0 and line["config"]["n_scenes_total"] == 24
