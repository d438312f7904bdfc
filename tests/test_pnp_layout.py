"""PnPsolver batch work-area layout (host only): the allocation covers every byte the carve
touches, for any mix of correspondence counts N <= 8192 and hypothesis counts.  An earlier
version summed unaligned Refine-scratch sizes while the carve aligned each sub-buffer, so the
last solvers' Refine buffers ran past the work area (the 9f527cb fault)."""
import ctypes as C

import numpy as np
import pytest


def _check(N, K, minSet):
    from c_orb_slam_amd._lib import lib
    n = len(N)
    N, K, mS = (np.ascontiguousarray(a, np.int32) for a in (N, K, minSet))
    out = np.zeros(4, np.int64)
    rc = lib().orbgpu_unit_pnp_layout(n, N.ctypes.data, K.ctypes.data, mS.ctypes.data, out.ctypes.data)
    return rc, out


@pytest.mark.parametrize("seed", range(20))
def test_layout_covers_carve(seed):
    rng = np.random.default_rng(seed)
    n = int(rng.integers(1, 120))
    N = rng.integers(4, 8193, n)
    N[rng.random(n) < 0.3] = rng.integers(4, 40, int((rng.random(n) < 0.3).sum()) or 1)[0]
    K = rng.integers(1, 301, n)
    minSet = rng.choice([3, 4], n)
    rc, out = _check(N, K, minSet)
    assert rc == 0, out
    assert out[1] <= out[0] and out[3] <= out[2]


@pytest.mark.parametrize("N", [4, 5, 31, 32, 33, 63, 64, 65, 255, 256, 257, 1023, 4096, 8191, 8192])
def test_layout_edges(N):
    for K in (1, 2, 63, 64, 65, 300):
        rc, out = _check([N] * 7, [K] * 7, [4] * 7)
        assert rc == 0 and out[1] <= out[0] and out[3] <= out[2], (N, K, out)
