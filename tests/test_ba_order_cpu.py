"""How far the canonical-tree accumulation order (oracle/ba.c ora_csum, shared with the GPU
kernels) moves the BA results away from the reference's own order (g2o's sequential "+="
over edges in internalId order, block_solver.hpp:353-560; sequential chi2 and computeScale,
sparse_optimizer.cpp:61-114).  CPU only: both are oracle modes."""
import numpy as np

import oracle_lib
from ba_cases import ba_problem, global_ba_problem
from pose_cases import pose_problem


def _run_both(fn):
    with oracle_lib.ba_order("g2o"):
        g = fn()
    with oracle_lib.ba_order("canonical"):
        c = fn()
    return g, c


def test_order_modes_differ_and_agree_local_ba():
    pr = ba_problem(0)
    g, c = _run_both(lambda: oracle_lib.oracle_local_ba(pr))
    assert g["iterations"] == c["iterations"]
    assert np.array_equal(g["edge_erase"], c["edge_erase"])
    # the orders really differ in the last bits ...
    assert not np.array_equal(np.asarray(g["trial_chi2"]), np.asarray(c["trial_chi2"]))
    # ... and agree far inside the north star's 1e-5
    np.testing.assert_allclose(g["trial_chi2"], c["trial_chi2"], rtol=1e-9)
    np.testing.assert_allclose(g["kf_Tcw"], c["kf_Tcw"], rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(g["pt_pos"], c["pt_pos"], rtol=1e-6, atol=1e-6)


def test_order_modes_agree_global_ba():
    pr = global_ba_problem(0, n_kf=48, pts_per_kf=60)
    g, c = _run_both(lambda: oracle_lib.oracle_global_ba(pr, 10, False))
    assert g["iterations"] == c["iterations"]
    np.testing.assert_allclose(g["solve_chi2"], c["solve_chi2"], rtol=1e-9)
    np.testing.assert_allclose(g["kf_Tcw"], c["kf_Tcw"], rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(g["pt_pos"], c["pt_pos"], rtol=1e-6, atol=1e-6)


def test_order_modes_agree_pose_optimization():
    for seed in range(4):
        pr = pose_problem(seed, N=400)
        g, c = _run_both(lambda: oracle_lib.oracle_pose_optimization(pr))
        assert g["inliers"] == c["inliers"]
        assert np.array_equal(g["outlier"], c["outlier"])
        np.testing.assert_allclose(g["Tcw"], c["Tcw"], rtol=1e-6, atol=1e-6)
