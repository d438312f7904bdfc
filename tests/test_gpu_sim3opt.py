"""Optimizer::OptimizeSim3 (Optimizer.cc:1046-1241) on the GPU vs the CPU oracle.

One persistent workgroup per loop candidate runs the whole call: optimize(5) with the
numeric Jacobians of EdgeSim3ProjectXYZ / EdgeInverseSim3ProjectXYZ, chi2 gating against
th2, optimize(10 | 5) on the inliers.  The 7x7 system is summed in the oracle's canonical
order and the pivoted LDL^T, Sim3 exp/product/inverse and LM control are the same operation
sequence -> the refined g2o::Sim3 (8 doubles), the erased matches and nIn are bit-identical
to oracle/ba.c ora_optimize_sim3.
"""
import numpy as np
import pytest

import oracle_lib
from sim3opt_cases import sim3opt_problem

pytestmark = pytest.mark.gpu

EUROC4 = (435.2047, 435.2047, 367.4517, 252.2009)


def _run_check(pr):
    from c_orb_slam_amd import OptimizeSim3
    S0 = oracle_lib.oracle_sim3_from_Rts(pr["R0"], pr["t0"], pr["s0"])
    n, S, er = OptimizeSim3(pr, S0)
    on, oS, oer, _ = oracle_lib.oracle_optimize_sim3(pr, S0)
    assert n == on
    assert np.array_equal(S.view(np.uint64), oS.view(np.uint64)), (S, oS)
    assert np.array_equal(er, oer)
    return n, S, er, S0


@pytest.mark.parametrize("fix", [True, False])
@pytest.mark.parametrize("seed", range(4))
def test_sim3opt_matches_oracle(gpu, seed, fix):
    pr = sim3opt_problem(seed=seed, fix_scale=fix)
    n, S, er, S0 = _run_check(pr)
    assert n >= 10 and er[pr["gross"]].mean() > 0.8


@pytest.mark.parametrize("kw", [dict(outlier_frac=0.0), dict(outlier_frac=0.5), dict(N=2000, match_frac=0.9),
                                dict(N=60, match_frac=0.3), dict(rot_deg=4.0, trans=0.3),
                                dict(cam1=EUROC4, cam2=EUROC4), dict(cam2=EUROC4), dict(th2=5.991),
                                dict(fix_scale=False, scale_noise=0.2), dict(outlier_frac=0.97)])
def test_sim3opt_edge_cases(gpu, kw):
    _run_check(sim3opt_problem(seed=11, **kw))


def test_sim3opt_early_return_leaves_estimate(gpu):
    from c_orb_slam_amd import OptimizeSim3
    pr = sim3opt_problem(seed=4, N=40, match_frac=0.25)
    assert pr["valid"].sum() < 10
    n, S, er, S0 = _run_check(pr)
    assert n == 0 and np.array_equal(S, S0)
    pr0 = dict(pr, valid=np.zeros(pr["N"], np.uint8))   # no correspondence at all
    n, S, er = OptimizeSim3(pr0, S0)
    assert n == 0 and np.array_equal(S, S0) and not er.any()


def test_sim3opt_batch_equals_single(gpu):
    from c_orb_slam_amd import OptimizeSim3Batch
    prs = [sim3opt_problem(seed=20 + i, fix_scale=bool(i % 2), N=300 + 150 * i) for i in range(6)]
    S0 = [oracle_lib.oracle_sim3_from_Rts(p["R0"], p["t0"], p["s0"]) for p in prs]
    n, S, er = OptimizeSim3Batch(prs, S0)
    for i, p in enumerate(prs):
        on, oS, oer, _ = oracle_lib.oracle_optimize_sim3(p, S0[i])
        assert n[i] == on and np.array_equal(S[i], oS) and np.array_equal(er[i], oer)


def test_sim3opt_capacity(gpu):
    from c_orb_slam_amd import OptimizeSim3, OrbGpuError
    pr = sim3opt_problem(seed=1, N=2100, match_frac=1.0)
    pr["valid"][:] = 1
    S0 = oracle_lib.oracle_sim3_from_Rts(pr["R0"], pr["t0"], pr["s0"])
    with pytest.raises(OrbGpuError):
        OptimizeSim3(pr, S0)
