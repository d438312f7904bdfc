"""GPU Sim3 RANSAC vs the CPU oracle (reference src/Sim3Solver.cc).

Loop-closure-shaped problems (LoopClosing.cc:333-389): N in {20..400}, 40%
outliers, SetRansacParameters(0.99, 20, 300), iterate(5) per call, bFixScale
true (stereo) and false (monocular scale drift).  Every call must agree with
the oracle: T12 present (tolerance 1e-5 relative, in practice bit-equal),
vbInliers, nInliers, bNoMore, the iteration counter, the best estimate
(R, t, s) and the rand() stream position.
"""
import numpy as np
import pytest

import oracle_lib
from sim3_cases import sim3_problem

pytestmark = pytest.mark.gpu


def _pair(pr, minInliers=20):
    from c_orb_slam_amd.ransac import Sim3Solver
    args = (pr["X1"], pr["X2"], pr["s1"], pr["s2"], pr["idx1"], pr["N1"], pr["K1"], pr["K2"], pr["fix"])
    g, o = Sim3Solver(*args), oracle_lib.OracleSim3(*args)
    g.SetRansacParameters(0.99, minInliers, 300)
    o.set_ransac(0.99, minInliers, 300)
    return g, o


def _same_rng(rg, ro):
    return tuple(rg.s.tbl) + (rg.s.f, rg.s.r) == tuple(ro[0:33])


@pytest.mark.parametrize("N,seed,fix,outl", [(20, 1, True, 0.2), (60, 2, True, 0.4), (150, 3, False, 0.4),
                                             (400, 4, False, 0.5), (90, 5, True, 0.7), (35, 6, False, 0.3),
                                             (250, 7, True, 0.9)])
def test_sim3_iterate_sequence(gpu, N, seed, fix, outl):
    from c_orb_slam_amd.ransac import Rng
    pr = sim3_problem(seed, N, outlier_frac=outl, fix_scale=fix)
    g, o = _pair(pr)
    rg, ro = Rng(1), oracle_lib.new_rng(1)
    for call in range(80):
        Tg, nmg, ing, ning = g.iterate(5, rg)
        oko, To, ino, nino, nmo = o.iterate(5, ro)
        assert (Tg is not None) == oko, f"call {call}"
        assert nmg == nmo and ning == nino, f"call {call}"
        assert np.array_equal(ing, ino)
        if oko:
            np.testing.assert_allclose(Tg, To, rtol=1e-5, atol=1e-6)
        assert g.state()[0] == o.iterations
        Ro, to, so = o.estimate()
        np.testing.assert_allclose(g.GetEstimatedRotation(), Ro, rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(g.GetEstimatedTranslation().ravel(), to, rtol=1e-5, atol=1e-6)
        assert abs(g.GetEstimatedScale() - so) <= 1e-5 * abs(so)
        assert _same_rng(rg, ro), "RNG stream position diverged"
        if oko or nmo:
            break


def test_sim3_recovers_similarity(gpu):
    from c_orb_slam_amd.ransac import Rng
    pr = sim3_problem(3, 300, outlier_frac=0.4, fix_scale=False)
    g, _ = _pair(pr)
    r = Rng(1)
    for _ in range(60):
        T, nm, inl, n = g.iterate(5, r)
        if T is not None or nm:
            break
    assert T is not None and n > 20
    assert abs(g.GetEstimatedScale() - pr["s"]) < 0.05 * pr["s"]
    np.testing.assert_allclose(g.GetEstimatedRotation(), pr["T12"][:3, :3] / pr["s"], atol=0.05)


def test_sim3_batch_matches_sequential(gpu):
    """64 loop candidates in one launch (independent rand streams) == oracle one by one."""
    from c_orb_slam_amd.ransac import Rng, sim3_iterate_batch
    probs = [sim3_problem(200 + k, [30, 120, 300][k % 3], outlier_frac=0.5, fix_scale=bool(k & 1)) for k in range(64)]
    pairs = [_pair(pr) for pr in probs]
    rgs = [Rng(3000 + k) for k in range(64)]
    ros = [oracle_lib.new_rng(3000 + k) for k in range(64)]
    for rnd in range(4):
        res = sim3_iterate_batch([p[0] for p in pairs], 5, rgs)
        for k, ((g, o), (Tg, nmg, ing, ning)) in enumerate(zip(pairs, res)):
            oko, To, ino, nino, nmo = o.iterate(5, ros[k])
            assert (Tg is not None) == oko and nmg == nmo and ning == nino, (rnd, k)
            assert np.array_equal(ing, ino), (rnd, k)
            if oko:
                np.testing.assert_allclose(Tg, To, rtol=1e-5, atol=1e-6)
            assert _same_rng(rgs[k], ros[k]), (rnd, k)


def test_sim3_too_few_and_shared_stream(gpu):
    from c_orb_slam_amd.ransac import Rng, sim3_iterate_batch
    pr = sim3_problem(9, 10)
    g, o = _pair(pr)   # minInliers 20 > N -> bNoMore, no draws consumed
    r = Rng(1)
    before = tuple(r.s.tbl)
    T, nm, inl, n = g.iterate(5, r)
    assert T is None and nm and n == 0 and tuple(r.s.tbl) == before
    # one stream shared by three solvers: consumed in solver order, like sequential calls
    probs = [sim3_problem(40 + k, 80, outlier_frac=0.6) for k in range(3)]
    pairs = [_pair(p) for p in probs]
    shared, ro = Rng(7), oracle_lib.new_rng(7)
    res = sim3_iterate_batch([p[0] for p in pairs], 5, [shared] * 3)
    for (g, o), (Tg, nmg, ing, ning) in zip(pairs, res):
        oko, To, ino, nino, nmo = o.iterate(5, ro)
        assert (Tg is not None) == oko and ning == nino and np.array_equal(ing, ino)
    assert _same_rng(shared, ro)
