"""CPU: the elimination order and the block-sparse LDL^T of the large pose systems.

* The product's nested-dissection order (orbgpu_unit_nd_order, csrc/ordering.cpp; host only)
  equals the oracle's independent restatement (oracle/ordering.c) on band, loop-closed,
  random and disconnected graphs and on BA-shaped pose graphs with and without loop closures
  (the reference orders with AMD inside Eigen's SimplicialLDLT, linear_solver_eigen.h:60-124;
  the canonical order both sides share is the one stated in ordering.hpp).
* The oracle's block-sparse factorisation in that order (ora_ldlt_solve_nd) solves the system
  (numpy, 1e-9) and is bit-identical to the dense right-looking LDL^T (ora_ldlt_solve, the
  per-element operation sequence every LDL^T of this repo follows) run on the permuted matrix.
* A loop-closed map keeps its factor small in this order where natural order fills the whole
  band between the loop's ends.
"""
import ctypes as C

import numpy as np
import pytest

import oracle_lib
from ba_cases import global_ba_problem
from c_orb_slam_amd._lib import lib, ptr


def _csr(n, edges):
    nb = [set() for _ in range(n)]
    for a, b in edges:
        if a != b:
            nb[a].add(b)
            nb[b].add(a)
    as_ = np.zeros(n + 1, np.int32)
    adj = []
    for i in range(n):
        as_[i + 1] = as_[i] + len(nb[i])
        adj += sorted(nb[i])
    return as_, np.array(adj + [0], np.int32)


def _gpu_order(n, as_, adj, leaf=32):
    perm = np.zeros(max(n, 1), np.int32)
    nn, h = C.c_int32(), C.c_int32()
    assert lib().orbgpu_unit_nd_order(n, ptr(as_), ptr(adj), leaf, ptr(perm), C.byref(nn), C.byref(h)) == 0
    return perm[:n], nn.value, h.value


def _ora_order(n, as_, adj, leaf=32):
    L = oracle_lib.lib()
    L.ora_nd_order.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p]
    perm = np.zeros(max(n, 1), np.int32)
    L.ora_nd_order(n, ptr(as_), ptr(adj), leaf, ptr(perm))
    return perm[:n]


def _band(n, bw, chords=()):
    e = [(i, j) for i in range(n) for j in range(i + 1, min(n, i + bw + 1))]
    return e + list(chords)


def _pose_graph(pr):
    """Poses (every keyframe but mnId 0) adjacent when they share a point: the Schur pattern."""
    free = pr["kf_id"] != 0
    pidx = -np.ones(len(free), np.int64)
    pidx[free] = np.arange(int(free.sum()))
    pe, ke = pr["edge_pt"], pidx[pr["edge_kf"]]
    o = np.argsort(pe, kind="stable")
    pe, ke = pe[o], ke[o]
    cut = np.flatnonzero(np.r_[True, pe[1:] != pe[:-1], True])
    edges = set()
    for s, t in zip(cut[:-1], cut[1:]):
        ks = [k for k in ke[s:t] if k >= 0]
        for a in ks:
            for b in ks:
                if a < b:
                    edges.add((int(a), int(b)))
    return int(free.sum()), sorted(edges)


GRAPHS = {
    "band": (400, _band(400, 9)),
    "ring": (300, _band(300, 6, [(i, 299 - j) for i in range(4) for j in range(4)])),
    "laps": (500, _band(500, 8, [(i, i + 125 * m) for i in range(0, 125, 3) for m in (1, 2, 3) if i + 125 * m < 500])),
    "random": (350, [tuple(x) for x in np.random.default_rng(3).integers(0, 350, (1400, 2))]),
    "components": (260, _band(100, 5) + [(100 + a, 100 + b) for a, b in _band(90, 3)] +
                   [(190 + a, 190 + b) for a, b in _band(70, 12)]),
    "small": (20, _band(20, 2)),
    "clique": (60, [(i, j) for i in range(60) for j in range(i + 1, 60)]),
}


@pytest.mark.parametrize("name", sorted(GRAPHS))
def test_nd_order_product_equals_oracle(name):
    n, edges = GRAPHS[name]
    as_, adj = _csr(n, edges)
    for leaf in (8, 32):
        g, nn, h = _gpu_order(n, as_, adj, leaf)
        o = _ora_order(n, as_, adj, leaf)
        assert np.array_equal(np.sort(g), np.arange(n))
        assert np.array_equal(g, o), name
        assert nn >= 1 and h >= 0
        if name in ("band", "laps", "ring") and leaf == 8:
            assert h >= 3   # a tree, not one node


@pytest.mark.parametrize("laps", [0, 3])
def test_nd_order_ba_pose_graph(laps):
    pr = global_ba_problem(2, n_kf=300, pts_per_kf=40, laps=laps)
    n, edges = _pose_graph(pr)
    as_, adj = _csr(n, edges)
    g, nn, h = _gpu_order(n, as_, adj)
    assert np.array_equal(g, _ora_order(n, as_, adj))
    assert h >= 2


def _spd_blocks(rng, nb, edges):
    n = 6 * nb
    S = np.zeros((n, n))
    for i in range(nb):
        S[6 * i:6 * i + 6, 6 * i:6 * i + 6] = rng.normal(size=(6, 6))
    for a, b in edges:
        i, j = min(a, b), max(a, b)
        S[6 * i:6 * i + 6, 6 * j:6 * j + 6] = rng.normal(size=(6, 6))
    S = np.triu(S) + np.triu(S, 1).T
    S += np.diag(np.abs(S).sum(1) + 1.0)
    return S


@pytest.mark.parametrize("name", ["band", "ring", "laps", "components"])
def test_sparse_oracle_solves_and_matches_dense_sequence(name):
    nb, edges = GRAPHS[name]
    nb = min(nb, 160)
    edges = [(a, b) for a, b in edges if a < nb and b < nb]
    rng = np.random.default_rng(11)
    S = _spd_blocks(rng, nb, edges)
    n = 6 * nb
    b = rng.normal(size=n)
    L = oracle_lib.lib()
    L.ora_ldlt_solve_nd.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p]
    L.ora_ldlt_solve.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p]
    Su = np.triu(S).copy()
    x = np.zeros(n)
    assert L.ora_ldlt_solve_nd(ptr(Su), n, ptr(b), ptr(x)) == 1
    np.testing.assert_allclose(S @ x, b, rtol=1e-9, atol=1e-9)
    # the same order through the product's ordering entry, then the dense oracle on P S P^T
    as_, adj = _csr(nb, [(a, b) for a, b in edges if a != b])
    perm, _, _ = _gpu_order(nb, as_, adj)
    rows = (6 * perm[:, None] + np.arange(6)[None, :]).reshape(-1)
    Sp = np.triu(S[np.ix_(rows, rows)]).copy()
    xp = np.zeros(n)
    assert L.ora_ldlt_solve(ptr(Sp), n, ptr(b[rows].copy()), ptr(xp)) == 1
    xd = np.zeros(n)
    xd[rows] = xp
    assert np.array_equal(x, xd), np.abs(x - xd).max()


def test_loop_closed_map_fill_is_bounded():
    """Natural order on a 3-lap map fills the band between each loop's ends; the nested
    dissection keeps the factor within a few times the pattern."""
    pr = global_ba_problem(4, n_kf=600, pts_per_kf=30, laps=3)
    n, edges = _pose_graph(pr)
    far = sum(1 for a, b in edges if b - a > 100)
    assert far > 50                               # long-range covisibility exists
    as_, adj = _csr(n, edges)
    perm, _, h = _gpu_order(n, as_, adj)
    pos = np.empty(n, np.int64)
    pos[perm] = np.arange(n)

    def fill(order_pos):
        rows = [set() for _ in range(n)]
        for a, b in edges:
            i, j = sorted((int(order_pos[a]), int(order_pos[b])))
            rows[i].add(j)
        tot = 0
        for p in range(n):
            r = sorted(rows[p])
            tot += len(r)
            if r:
                rows[r[0]].update(r[1:])
        return tot
    nat, nd = fill(np.arange(n)), fill(pos)
    assert nd < nat / 3, (nd, nat)
    assert h >= 3


def test_nd_order_rejects_malformed_graphs():
    """orbgpu_unit_nd_order validates its CSR input: offsets from 0 and
    non-decreasing, neighbours in [0, n), no self loops -> ORB_E_INVALID, nothing read out of
    range."""
    ORB_E_INVALID = -1
    n = 6
    as_, adj = _csr(n, [(i, i + 1) for i in range(n - 1)])
    perm = np.zeros(n, np.int32)
    nn, h = C.c_int32(), C.c_int32()

    def call(a, d):
        return lib().orbgpu_unit_nd_order(n, ptr(a), ptr(d), 4, ptr(perm), C.byref(nn), C.byref(h))

    assert call(as_, adj) == 0
    bad = as_.copy()
    bad[0] = 1
    assert call(bad, adj) == ORB_E_INVALID                 # offsets not from 0
    bad = as_.copy()
    bad[3] = bad[2] - 1
    assert call(bad, adj) == ORB_E_INVALID                 # decreasing offsets
    for v in (-1, n, 10**6):
        d = adj.copy()
        d[2] = v
        assert call(as_, d) == ORB_E_INVALID               # neighbour out of range
    d = adj.copy()
    d[as_[2]] = 2
    assert call(as_, d) == ORB_E_INVALID                   # self loop
