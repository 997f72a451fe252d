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
    assert line["gather_check"] == "rank-0 rows equal after gather"
    assert line["parity"].startswith("bit-exact")
    assert "nccl" in line["config"]["parallelism"]


@pytest.mark.gpu
@pytest.mark.parametrize("workload", ["c3", "c2cube"])
def test_bench_graph_replay_single_gpu(tmp_path, workload):
    """bench.py's single-GPU step as one hipGraph replay: the captured launches
    run on every replay (the last launch's outputs are bit-exact vs the oracle)
    and the per-launch event average covers every launch of the step."""
    import json
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ)
    env.pop("MVM_DIST_FORCE", None)
    r = subprocess.run([sys.executable, os.path.join(repo, "bench.py"), "--workload", workload,
                        "--scenes", "24", "--chunk", "8", "--steps", "2", "--warmup", "1",
                        "--cpu-seconds", "0", "--graph", "on"],
                       env=env, capture_output=True, text=True, timeout=300, cwd=repo)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["parity"].startswith("bit-exact")
    assert line["config"]["launch"].startswith("one hipGraph replay")
    assert line["config"]["launches_per_step"] == 3
    assert line["roofline"]["avg_launch_ms"] > 0
