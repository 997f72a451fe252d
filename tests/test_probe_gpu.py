"""The HBM write probe (bench.py's roofline reference) over a buffer larger
than one dispatch can cover: a 1-D grid counts work-items in 32 bits, so the
probe splits buffers beyond 2^32 / 256 workgroups x 8 KiB (~137 GB) into
several launches (csrc/mvm_common.hip).  Every float must be written."""
import pytest
import torch

from bpc_baseline_amd import ops

pytestmark = pytest.mark.gpu


def test_write_probe_covers_buffers_beyond_one_dispatch(cuda):
    n = 150 * (1 << 30) // 4                       # 150 GiB of float32
    torch.cuda.empty_cache()
    if torch.cuda.mem_get_info(cuda)[0] < 4 * n + (8 << 30):
        pytest.skip("needs ~160 GiB of free HBM")
    buf = torch.empty(n, dtype=torch.float32, device=cuda)
    try:
        buf.zero_()
        ops.hbm_write_probe(buf)
        torch.cuda.synchronize(cuda)
        step = 1 << 28                              # 1 GiB views
        for s in range(0, n, step):
            assert bool((buf[s:s + step] == 1.0).all()), f"probe left floats unwritten at {s}"
    finally:
        del buf
        torch.cuda.empty_cache()
