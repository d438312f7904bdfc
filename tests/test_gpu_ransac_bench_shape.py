"""The benched RANSAC call shape and the device replay's cross-chunk paths vs the CPU oracle.

`bench.py` times `iterate(300)` over 100 problems per call (PnPsolver.cc:165-258,
Sim3Solver.cc:140-207).  At that shape the hypothesis kernels run several 64-hypothesis
workgroups per solver, each regenerating the rand() stream up to its own words
(ransac_dev.hpp `draw_range`), `k_pnp_check` / `k_sim3_check` span many 16-hypothesis blocks,
and `k_pnp_replay` / `k_sim3_replay` carry their state (PnP: best count, cached Refine;
Sim3: the running maximum of `>=` updates) across 64-hypothesis chunks.  Every test asserts,
per solver and per call: pose presence and value, vbInliers, nInliers, bNoMore, the solver's
iteration counter and the rand() stream position (and for Sim3 the best estimate).

The late-event problems were found by scanning seeds with the oracle's event log
(`OraclePnP.events()`, `OracleSim3.events()`); each test re-asserts the event positions it
relies on, so a change to the case generators cannot silently turn them into early events.
"""
import numpy as np
import pytest

import oracle_lib
from pnp_cases import pnp_problem
from sim3_cases import sim3_problem

pytestmark = pytest.mark.gpu

HYP = 300


def _rng_eq(rg, ro):
    return tuple(rg.s.tbl) + (rg.s.f, rg.s.r) == tuple(ro[0:33])


def _pnp_pair(pr, minInliers, epsilon):
    from c_orb_slam_amd.ransac import PnPsolver
    g = PnPsolver(pr["p3d"], pr["p2d"], pr["sigma2"], pr["kp_idx"], pr["n_matches"], *pr["K"])
    o = oracle_lib.OraclePnP(pr["p3d"], pr["p2d"], pr["sigma2"], pr["kp_idx"], pr["n_matches"], *pr["K"])
    g.SetRansacParameters(0.99, minInliers, 300, 4, epsilon, 5.991)
    o.set_ransac(0.99, minInliers, 300, 4, epsilon, 5.991)
    return g, o


def _sim3_pair(pr, minInliers):
    from c_orb_slam_amd.ransac import Sim3Solver
    args = (pr["X1"], pr["X2"], pr["s1"], pr["s2"], pr["idx1"], pr["N1"], pr["K1"], pr["K2"], pr["fix"])
    g, o = Sim3Solver(*args), oracle_lib.OracleSim3(*args)
    g.SetRansacParameters(0.99, minInliers, 300)
    o.set_ransac(0.99, minInliers, 300)
    return g, o


def _check_pnp(tag, g, o, rg, ro, res):
    Tg, nmg, ing, ning = res
    oko, To, ino, nino, nmo = o.iterate(HYP, ro)
    assert (Tg is not None) == oko, tag
    assert nmg == nmo and ning == nino, tag
    assert np.array_equal(ing, ino), tag
    if oko:
        np.testing.assert_allclose(Tg, To, rtol=1e-5, atol=1e-6, err_msg=str(tag))
    assert g.state()[0] == o.iterations, tag
    assert _rng_eq(rg, ro), f"{tag}: RNG stream position diverged"
    return o.events()


def _check_sim3(tag, g, o, rg, ro, res):
    Tg, nmg, ing, ning = res
    oko, To, ino, nino, nmo = o.iterate(HYP, ro)
    assert (Tg is not None) == oko, tag
    assert nmg == nmo and ning == nino, tag
    assert np.array_equal(ing, ino), tag
    if oko:
        np.testing.assert_allclose(Tg, To, rtol=1e-5, atol=1e-6, err_msg=str(tag))
    assert g.state()[0] == o.iterations, tag
    Ro, to, so = o.estimate()
    np.testing.assert_allclose(g.GetEstimatedRotation(), Ro, rtol=1e-5, atol=1e-6, err_msg=str(tag))
    np.testing.assert_allclose(g.GetEstimatedTranslation().ravel(), to, rtol=1e-5, atol=1e-6, err_msg=str(tag))
    assert abs(g.GetEstimatedScale() - so) <= 1e-5 * abs(so), tag
    assert _rng_eq(rg, ro), f"{tag}: RNG stream position diverged"
    return o.events()


@pytest.mark.parametrize("N", [50, 150, 500])
def test_pnp_bench_shape(gpu, N):
    """bench.py's exact call: 100 problems, SetRansacParameters(0.99, N, 300, 4, 0.4, 5.991),
    iterate(300), two calls in a row (minInliers = N: every draw is solved and scored, the `||`
    loop runs the call's full 300 iterations, bNoMore after each)."""
    from c_orb_slam_amd.ransac import Rng, iterate_batch
    probs = [pnp_problem(1000 + s, N) for s in range(100)]
    pairs = [_pnp_pair(pr, N, 0.4) for pr in probs]
    rgs = [Rng(1 + k) for k in range(100)]
    ros = [oracle_lib.new_rng(1 + k) for k in range(100)]
    for call in range(2):
        res = iterate_batch([p[0] for p in pairs], HYP, rgs)
        for k, ((g, o), r) in enumerate(zip(pairs, res)):
            _check_pnp((N, call, k), g, o, rgs[k], ros[k], r)
            assert g.state()[0] == HYP * (call + 1)


def test_sim3_bench_shape(gpu):
    """bench.py's Sim3 call: 100 loop candidates of N = 150 pairs at 90 % outliers,
    SetRansacParameters(0.99, 36, 300) (mRansacMaxIts = 300), iterate(300).  No hypothesis exceeds
    minInliers, so the `>=` best updates run through all five 64-hypothesis chunks; the second
    call finds the budget spent (bNoMore, no draws); SetRansacParameters restarts it."""
    from c_orb_slam_amd.ransac import Rng, sim3_iterate_batch
    N3, min3 = 150, 36
    probs = [sim3_problem(2000 + s, N3, outlier_frac=0.9) for s in range(100)]
    pairs = [_sim3_pair(pr, min3) for pr in probs]
    rgs = [Rng(1 + k) for k in range(100)]
    ros = [oracle_lib.new_rng(1 + k) for k in range(100)]
    late_updates = 0
    for call in range(3):
        if call == 2:
            for g, o in pairs:
                g.SetRansacParameters(0.99, min3, 300)
                o.set_ransac(0.99, min3, 300)
        res = sim3_iterate_batch([p[0] for p in pairs], HYP, rgs)
        for k, ((g, o), r) in enumerate(zip(pairs, res)):
            ev = _check_sim3((call, k), g, o, rgs[k], ros[k], r)
            late_updates += any(h >= 64 for h, kind in ev)
            if call == 1:
                assert r[1] and not ev   # budget spent: bNoMore, nothing drawn
    assert late_updates >= 50, late_updates   # the shape does exercise the cross-chunk maximum


# (problem seed, N, outlier fraction, epsilon, rand seed) -> the oracle's events of iterate(300).
# kinds: 1 best update, 2 Refine failed, 3 Refine succeeded (pose returned)
PNP_LATE = [
    # first event and success in the second chunk (64 < h <= 128)
    ((4, 150, 0.55, 0.35, 11), [(77, 1), (77, 3)]),
    ((6, 150, 0.6, 0.3, 13), [(91, 1), (91, 3)]),
    # success after hypothesis 128
    ((0, 150, 0.6, 0.3, 7), [(133, 1), (133, 3)]),
    ((3, 500, 0.6, 0.3, 10), [(178, 1), (178, 3)]),
    ((7, 500, 0.6, 0.3, 14), [(282, 1), (282, 3)]),
    # best in chunk 0 with a failed Refine, a better hypothesis in a later chunk that succeeds
    ((28, 500, 0.6, 0.3, 35), [(31, 1), (31, 2), (76, 1), (76, 3)]),
    ((78, 150, 0.5, 0.45, 85), [(2, 1), (2, 2), (118, 1), (118, 3)]),
    ((232, 150, 0.5, 0.45, 239), [(53, 1), (53, 2), (179, 1), (179, 3)]),
    # late best updates whose Refine fails: the loop runs out and returns the best (bNoMore);
    # (241, 2) is a hypothesis at minInliers that does not beat the best (cached Refine)
    ((52, 150, 0.6, 0.3, 59), [(27, 1), (27, 2), (241, 2), (283, 1), (283, 2)]),
    ((84, 500, 0.5, 0.45, 91), [(32, 1), (32, 2), (85, 1), (85, 2)]),
    ((237, 150, 0.45, 0.5, 244), [(63, 1), (63, 2), (167, 1), (167, 2)]),
    ((3, 500, 0.55, 0.4, 10), [(161, 1), (161, 2)]),
]


def _pnp_late_problem(case):
    seed, N, outl, eps, _ = case
    return pnp_problem(seed, N, outlier_frac=outl), eps


def test_pnp_late_events_batch(gpu):
    """All late-event problems in one batched launch (independent streams), then a second call
    on each (state carried: best set, cached Refine, the iteration counter)."""
    from c_orb_slam_amd.ransac import Rng, iterate_batch
    pairs, rgs, ros = [], [], []
    for case, _ in PNP_LATE:
        pr, eps = _pnp_late_problem(case)
        pairs.append(_pnp_pair(pr, 10, eps))
        rgs.append(Rng(case[4]))
        ros.append(oracle_lib.new_rng(case[4]))
    for call in range(2):
        res = iterate_batch([p[0] for p in pairs], HYP, rgs)
        for k, ((g, o), r) in enumerate(zip(pairs, res)):
            ev = _check_pnp((call, PNP_LATE[k][0]), g, o, rgs[k], ros[k], r)
            if call == 0:
                assert ev == PNP_LATE[k][1], (PNP_LATE[k][0], ev)


@pytest.mark.parametrize("case,events", PNP_LATE[:6])
def test_pnp_late_events_single(gpu, case, events):
    """The same problems one solver per call (the non-batched entry point)."""
    from c_orb_slam_amd.ransac import Rng
    pr, eps = _pnp_late_problem(case)
    g, o = _pnp_pair(pr, 10, eps)
    rg, ro = Rng(case[4]), oracle_lib.new_rng(case[4])
    ev = _check_pnp(case, g, o, rg, ro, g.iterate(HYP, rg))
    assert ev == events


# (problem seed, N, outlier fraction, bFixScale, minInliers, rand seed): success after 64 / 128
SIM3_LATE = [
    ((247, 150, 0.8, False, 24, 258), 67),
    ((275, 150, 0.75, True, 30, 286), 90),
    ((292, 150, 0.75, True, 30, 303), 223),
]


def test_sim3_late_events(gpu):
    """Sim3 problems whose returning update (`>=` best with more than minInliers) comes in a later
    chunk after updates in earlier ones, plus loop candidates whose last update is after 128 with
    no return; all in one batch, then the next call on each."""
    from c_orb_slam_amd.ransac import Rng, sim3_iterate_batch
    cases = list(SIM3_LATE)
    # no-return cases: updates in chunk 0 and after hypothesis 128
    cases += [((0, 150, 0.75, True, 30, 11), None), ((0, 300, 0.75, False, 60, 11), None),
              ((1, 150, 0.75, True, 30, 12), None)]
    pairs, rgs, ros = [], [], []
    for (seed, N, outl, fix, mi, rs), _ in cases:
        pairs.append(_sim3_pair(sim3_problem(seed, N, outlier_frac=outl, fix_scale=fix), mi))
        rgs.append(Rng(rs))
        ros.append(oracle_lib.new_rng(rs))
    for call in range(2):
        res = sim3_iterate_batch([p[0] for p in pairs], HYP, rgs)
        for k, ((g, o), r) in enumerate(zip(pairs, res)):
            ev = _check_sim3((call, cases[k][0]), g, o, rgs[k], ros[k], r)
            if call == 0:
                want = cases[k][1]
                if want is None:
                    assert ev and ev[0][0] < 64 and ev[-1][0] >= 128 and all(kind == 1 for _, kind in ev), ev
                else:
                    assert ev[-1] == (want, 3) and ev[0][0] < 64, ev
