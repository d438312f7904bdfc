"""GPU BA building blocks vs the oracle: canonical FP64 sum (ora_csum) and the dense
LDL^T pose-system solve (ora_ldlt_solve), bit-identical by construction."""
import ctypes as C

import numpy as np
import pytest

import oracle_lib
from oracle_lib import ptr

pytestmark = pytest.mark.gpu


def _ora_csum(v):
    L = oracle_lib.lib()
    L.ora_csum.restype = C.c_double
    L.ora_csum.argtypes = [C.c_void_p, C.c_int]
    w = np.array(v, np.float64)
    return L.ora_csum(ptr(w), len(w))


def _ora_ldlt(S, b):
    L = oracle_lib.lib()
    L.ora_ldlt_solve.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p]
    A = np.array(S, np.float64)
    x = np.zeros(len(b))
    ok = L.ora_ldlt_solve(ptr(A), len(b), ptr(np.array(b, np.float64)), ptr(x))
    return ok, x


@pytest.mark.parametrize("n", [0, 1, 2, 63, 64, 65, 127, 128, 129, 4095, 4096, 4097, 15000, 300000])
def test_csum_matches_oracle(gpu, n):
    from c_orb_slam_amd._lib import lib
    rng = np.random.default_rng(n)
    v = rng.normal(0, 1, n) * 10.0 ** rng.integers(-8, 8, n)
    if n:
        v[0] = -0.0 if n == 1 else v[0]
    out = C.c_double()
    assert lib().orbgpu_unit_csum(ptr(np.ascontiguousarray(v)), n, C.byref(out)) == 0
    ref = _ora_csum(v)
    assert out.value == ref or (np.isnan(out.value) and np.isnan(ref))
    assert np.signbit(out.value) == np.signbit(ref)


def _spd(rng, n):
    A = rng.normal(size=(n, n))
    S = A @ A.T + n * np.eye(n)
    return S


@pytest.mark.parametrize("variant", [0, 1, 4, 5, 6, 7])
@pytest.mark.parametrize("n", [1, 2, 5, 6, 12, 60, 63, 64, 65, 66, 84, 90, 95, 96, 97, 126, 127, 128])
def test_ldlt_matches_oracle(gpu, n, variant):
    from c_orb_slam_amd._lib import lib
    rng = np.random.default_rng(100 + n)
    S = _spd(rng, n)
    # only the upper triangle is read: poison the lower one
    S_in = S.copy()
    S_in[np.tril_indices(n, -1)] = np.nan
    b = rng.normal(size=n)
    x = np.zeros(n)
    ok = C.c_int()
    rc = lib().orbgpu_unit_ldlt_solve(n, ptr(np.ascontiguousarray(S_in)), ptr(b), ptr(x), variant, C.byref(ok))
    if variant == 0 and n >= 128:   # the register solver keeps b in column n: n <= 127 (the product's n <= 126)
        assert rc != 0
        return
    if variant in (4, 5, 6, 7) and n > 96:   # the row- / column-owner / row-lane / 2-D solvers: n <= 96
        assert rc != 0
        return
    assert rc == 0
    oko, xo = _ora_ldlt(S_in, b)
    assert ok.value == oko == 1
    assert np.array_equal(x, xo), np.abs(x - xo).max()
    np.testing.assert_allclose(S @ x, b, rtol=1e-8, atol=1e-8)


def _banded_spd(rng, nblk, bw, loops=()):
    """Schur-complement-shaped SPD matrix: 6x6 blocks, block bandwidth bw, plus loop-closure blocks."""
    n = 6 * nblk
    S = np.zeros((n, n))
    for i in range(nblk):
        for j in range(i, min(nblk, i + bw + 1)):
            S[6 * i:6 * i + 6, 6 * j:6 * j + 6] = rng.normal(size=(6, 6))
    for i, j in loops:
        S[6 * i:6 * i + 6, 6 * j:6 * j + 6] = rng.normal(size=(6, 6))
    S = np.triu(S) + np.triu(S, 1).T
    S += np.diag(np.abs(S).sum(1) + 1.0)
    return S


@pytest.mark.parametrize("n,kind", [(1, "dense"), (63, "dense"), (64, "dense"), (65, "dense"), (130, "dense"),
                                    (200, "dense"), (511, "dense"), (600, "banded"), (1200, "banded"),
                                    (1200, "loops"), (1998, "banded")])
def test_ldlt_tiled_matches_oracle(gpu, n, kind):
    from c_orb_slam_amd._lib import lib
    rng = np.random.default_rng(7 + n)
    if kind == "dense":
        S = _spd(rng, n)
    else:
        nb = n // 6
        S = _banded_spd(rng, nb, 8, loops=[(1, nb - 2), (3, nb // 2)] if kind == "loops" else ())
        n = 6 * nb
    S_in = S.copy()
    S_in[np.tril_indices(n, -1)] = np.nan   # only the upper triangle is read
    b = rng.normal(size=n)
    x = np.zeros(n)
    ok = C.c_int()
    assert lib().orbgpu_unit_ldlt_solve(n, ptr(np.ascontiguousarray(S_in)), ptr(b), ptr(x), 2, C.byref(ok)) == 0
    oko, xo = _ora_ldlt(S_in, b)
    assert ok.value == oko == 1
    assert np.array_equal(x, xo), np.abs(x - xo).max()
    np.testing.assert_allclose(S @ x, b, rtol=1e-8, atol=1e-8)


def _ora_ldlt_nd(S, b):
    L = oracle_lib.lib()
    L.ora_ldlt_solve_nd.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p]
    x = np.zeros(len(b))
    ok = L.ora_ldlt_solve_nd(ptr(np.ascontiguousarray(S, np.float64)), len(b), ptr(np.array(b, np.float64)), ptr(x))
    return ok, x


@pytest.mark.parametrize("nb,kind", [(30, "banded"), (200, "banded"), (333, "banded"), (200, "loops"),
                                     (400, "laps"), (150, "random")])
def test_ldlt_nested_dissection_matches_oracle(gpu, nb, kind):
    """The level-scheduled tiled LDL^T in nested-dissection order (variant 3: the order the BA
    uses for >= 24 poses) against the oracle's block-sparse restatement in the same order:
    bit-identical x, and S x = b."""
    from c_orb_slam_amd._lib import lib
    rng = np.random.default_rng(100 + nb)
    if kind == "laps":   # a 4-lap circuit: the same place on every lap covisible
        n_lap = nb // 4
        loops = [(i, i + n_lap * m) for i in range(0, n_lap, 2) for m in (1, 2, 3) if i + n_lap * m < nb]
        S = _banded_spd(rng, nb, 6, loops=loops)
    elif kind == "random":
        pairs = rng.integers(0, nb, (3 * nb, 2))
        S = _banded_spd(rng, nb, 1, loops=[(min(a, b), max(a, b)) for a, b in pairs if a != b])
    else:
        S = _banded_spd(rng, nb, 8, loops=[(1, nb - 2), (3, nb // 2), (nb // 4, 3 * nb // 4)] if kind == "loops" else ())
    n = 6 * nb
    S_in = S.copy()
    S_in[np.tril_indices(n, -1)] = np.nan   # only the upper triangle is read
    b = rng.normal(size=n)
    x = np.zeros(n)
    ok = C.c_int()
    assert lib().orbgpu_unit_ldlt_solve(n, ptr(np.ascontiguousarray(S_in)), ptr(b), ptr(x), 3, C.byref(ok)) == 0
    oko, xo = _ora_ldlt_nd(np.triu(S), b)
    assert ok.value == oko == 1
    assert np.array_equal(x, xo), np.abs(x - xo).max()
    np.testing.assert_allclose(S @ x, b, rtol=1e-8, atol=1e-8)


def test_ldlt_nested_dissection_zero_pivot_fails(gpu):
    from c_orb_slam_amd._lib import lib
    rng = np.random.default_rng(5)
    S = _banded_spd(rng, 120, 4, loops=[(2, 110)])
    S[6 * 70 + 2, :] = 0.0
    S[:, 6 * 70 + 2] = 0.0   # an exactly zero pivot in the middle of the order
    x = np.full(720, 7.0)
    ok = C.c_int(5)
    assert lib().orbgpu_unit_ldlt_solve(720, ptr(np.ascontiguousarray(S)), ptr(np.ones(720)), ptr(x), 3, C.byref(ok)) == 0
    assert ok.value == 0
    assert (x == 7.0).all()


def test_ldlt_tiled_zero_pivot_fails(gpu):
    from c_orb_slam_amd._lib import lib
    n = 300
    S = np.eye(n) * 2.0
    S[150, 150] = 0.0
    x = np.full(n, 7.0)
    ok = C.c_int(5)
    assert lib().orbgpu_unit_ldlt_solve(n, ptr(S), ptr(np.ones(n)), ptr(x), 2, C.byref(ok)) == 0
    assert ok.value == 0


def test_ldlt_zero_pivot_fails(gpu):
    from c_orb_slam_amd._lib import lib
    S = np.eye(12)
    S[7, 7] = 0.0
    x = np.zeros(12)
    ok = C.c_int(5)
    for variant in (0, 1, 4, 5, 6, 7):
        assert lib().orbgpu_unit_ldlt_solve(12, ptr(S), ptr(np.ones(12)), ptr(x), variant, C.byref(ok)) == 0
        assert ok.value == 0


def test_wave_tree_matches_canonical_tree(gpu):
    from c_orb_slam_amd._lib import lib
    rng = np.random.default_rng(7)
    for trial in range(20):
        v = rng.normal(0, 1, 64) * 10.0 ** rng.integers(-10, 10, 64)
        out = C.c_double()
        assert lib().orbgpu_unit_wave_tree(ptr(np.ascontiguousarray(v)), C.byref(out)) == 0
        assert out.value == _ora_csum(v), trial



def test_shared_div_matches_division(gpu):
    """SharedDiv (one reciprocal per denominator, ba_math.hpp) is bit-identical to the FP64
    division on operands across the fast range, its edges, zeros, signed zeros, subnormals,
    huge values, infinities and NaN (outside the range it divides plainly)."""
    from c_orb_slam_amd._lib import lib
    rng = np.random.default_rng(11)
    n = 1 << 20
    a = rng.uniform(1, 2, n) * np.exp2(rng.integers(-330, 330, n)) * rng.choice([-1.0, 1.0], n)
    b = rng.uniform(1, 2, n) * np.exp2(rng.integers(-330, 330, n)) * rng.choice([-1.0, 1.0], n)
    # BA-shaped operands: depths 0.1-1000 m, pixel-scale numerators, rotation entries
    k = n // 4
    b[:k] = rng.uniform(0.1, 1000, k) ** rng.choice([1, 2], k)
    a[:k] = rng.normal(0, 1, k) * 10.0 ** rng.integers(-3, 7, k)
    special = np.array([0.0, -0.0, np.inf, -np.inf, np.nan, 5e-324, -5e-324, 2.2250738585072014e-308,
                        1.7976931348623157e308, 2.0 ** -300, 2.0 ** 300, float.fromhex("0x1.0000000000001p-300"),
                        float.fromhex("0x1.fffffffffffffp299"), 1.0])
    ns = len(special)
    a[k:k + ns * ns] = np.repeat(special, ns)
    b[k:k + ns * ns] = np.tile(special, ns)
    out = np.zeros(2 * n)
    assert lib().orbgpu_unit_shared_div(ptr(a), ptr(b), n, ptr(out)) == 0
    got, ref = out[0::2].view(np.uint64), out[1::2].view(np.uint64)
    nan = np.isnan(out[1::2])
    assert np.array_equal(np.isnan(out[0::2]), nan)
    assert np.array_equal(got[~nan], ref[~nan]), int(np.sum(got[~nan] != ref[~nan]))
