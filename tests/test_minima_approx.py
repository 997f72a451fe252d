"""The float32 block minima of mvm_triplet_minima, modelled on
the CPU: min_j f32(f32(e12 + e23) + e13) * f32(1/3) lands within a few units
in the last place of the float32 cube value of the exact fp64 minimum, and
wherever its lower 16 bits are at least 8 units from a carry (and the value
is >= 2^-100) its upper 16 bits are the exact key's.  The kernel rechecks the
rest in fp64; this pins the margin it relies on with the oracle's residuals.
"""
import numpy as np
import pytest

MARGIN = 8                     # kApproxMargin (csrc/mvm_cube.hip)
TINY = 0x0D800000              # kApproxTiny: the bits of 2^-100


def _scene(seed, n):
    from bpc_baseline_amd.synth import make_scenes
    from oracle import oracle as O
    b = make_scenes(1, 3, n, seed=seed)
    r = O.residuals(b.pts, b.cam_offs, b.F, 1, n)[0]
    return r[0, :n, :n], r[1, :n, :n].T, r[2, :n, :n].T        # e12 [i,j], e13 [i,k], e23 [j,k]


@pytest.mark.parametrize("seed", [1, 5, 9])
def test_float32_block_minima_within_margin(seed):
    n = 128
    e12, e13, e23 = _scene(seed, n)
    # exact: the fp64 sums in the reference's order, the cube's float32 value
    s64 = (e12[:, :, None] + e13[:, None, :]) + e23[None, :, :]          # [i, j, k]
    m64 = s64.reshape(n, n // 32, 32, n).min(axis=2)                      # block minima [i, jb, k]
    exact = (m64 / 3.0).astype(np.float32).view(np.uint32).astype(np.int64)
    # the kernel's float32 form
    f12, f13, f23 = (a.astype(np.float32) for a in (e12, e13, e23))
    v = f12[:, :, None] + f23[None, :, :]
    m32 = v.reshape(n, n // 32, 32, n).min(axis=2)
    approx = ((m32 + f13[:, None, :]) * np.float32(1.0 / 3.0)).astype(np.float32)
    bits = approx.view(np.uint32).astype(np.int64)
    dist = np.abs(bits - exact)
    assert dist.max() <= 6, dist.max()                    # the bound DESIGN 3.11 derives
    lo = bits & 0xFFFF
    ok = (lo >= MARGIN) & (lo <= 0xFFFF - MARGIN) & (bits >= TINY)
    assert ok.mean() > 0.999
    assert np.array_equal((bits[ok] | 0x80000000) >> 16, (exact[ok] | 0x80000000) >> 16)
