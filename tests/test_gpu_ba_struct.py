"""GPU: the BA structure built on the device (ba_struct_gpu.hip) equals the host restatement
(ba_struct.cpp) list for list -- initializeOptimization(level) + buildIndexMapping +
BlockSolver::buildStructure (g2o sparse_optimizer.cpp:198-287, block_solver.hpp:139-216): the
active edges, vertices by mnId, per-vertex edge lists, each landmark's pose terms in pose order,
the Schur blocks (diagonal first, then first use) and their terms in landmark order."""
import ctypes as C

import numpy as np
import pytest

from ba_cases import ba_problem, global_ba_problem

pytestmark = pytest.mark.gpu


def _both(pr, fixed, level_mask=None, level=0):
    from c_orb_slam_amd._lib import lib, ptr
    nkf, npt, ne = len(pr["kf_id"]), len(pr["pt_id"]), len(pr["edge_pt"])
    ek = np.ascontiguousarray(pr["edge_kf"], np.int32)
    ep = np.ascontiguousarray(pr["edge_pt"], np.int32)
    lv = np.zeros(ne, np.uint8) if level_mask is None else np.ascontiguousarray(level_mask, np.uint8)
    fx = np.ascontiguousarray(fixed, np.uint8)
    kid = np.ascontiguousarray(pr["kf_id"], np.int32)
    pid = np.ascontiguousarray(pr["pt_id"], np.int32)
    outs = []
    for gpu in (0, 1, 2):   # host, multi-launch device builder, one-workgroup device builder
        cap = 64 * ne + 8 * (nkf + npt) + 1024
        while True:
            out = np.zeros(cap, np.int32)
            n = C.c_longlong()
            rc = lib().orbgpu_unit_ba_struct_all(nkf, npt, ne, ptr(ek), ptr(ep), ptr(lv), ptr(fx), ptr(kid), ptr(pid),
                                                 level, gpu, ptr(out), cap, C.byref(n))
            if rc == -3 and n.value > cap:   # ORB_E_CAPACITY
                cap = n.value
                continue
            assert rc == 0, (gpu, rc)
            outs.append(out[:n.value].copy())
            break
    assert np.array_equal(outs[1], outs[2])
    return outs[:2]


def _local_fixed(pr):
    return ((~pr["kf_local"].astype(bool)) | (pr["kf_id"] == 0)).astype(np.uint8)


@pytest.mark.parametrize("kw", [dict(seed=0), dict(seed=5, n_local=12, n_fixed=6, n_pt=800, outlier_frac=0.3),
                                dict(seed=6, n_local=20, n_fixed=10, n_pt=1500, obs_range=(2, 20)),
                                dict(seed=4, n_local=2, n_fixed=5, n_pt=150)])
def test_device_structure_equals_host_local(gpu, kw):
    pr = ba_problem(**kw)
    h, g = _both(pr, _local_fixed(pr))
    assert h[:8].tolist() == g[:8].tolist()
    assert np.array_equal(h, g)
    # the second optimisation level: outliers moved to level 1 (Optimizer.cc:672-702)
    rng = np.random.default_rng(kw["seed"])
    lvl = (rng.random(len(pr["edge_pt"])) < 0.1).astype(np.uint8)
    h, g = _both(pr, _local_fixed(pr), lvl, 0)
    assert np.array_equal(h, g)
    h, g = _both(pr, _local_fixed(pr), lvl, 1)
    assert np.array_equal(h, g)


@pytest.mark.parametrize("n_kf,laps", [(128, 0), (400, 0), (2000, 4)])
def test_device_structure_equals_host_global(gpu, n_kf, laps):
    pr = global_ba_problem(3, n_kf=n_kf, pts_per_kf=150, laps=laps)
    fixed = (pr["kf_id"] == 0).astype(np.uint8)
    h, g = _both(pr, fixed)
    assert h[:8].tolist() == g[:8].tolist()
    assert np.array_equal(h, g)


def test_device_structure_shuffled_ids(gpu):
    """mnIds not in index order (vertices sort by id, g2o's _ivMap), every level-0 edge active."""
    pr = ba_problem(9, n_local=10, n_fixed=5, n_pt=600)
    rng = np.random.default_rng(1)
    pr = dict(pr)
    pr["kf_id"] = rng.permutation(len(pr["kf_id"])).astype(np.int32) * 3 + 1
    pr["pt_id"] = rng.permutation(len(pr["pt_id"])).astype(np.int32) * 7 - 100000
    h, g = _both(pr, _local_fixed(pr))
    assert np.array_equal(h, g)


def test_device_structure_rejects_duplicate_edges(gpu):
    """Two edges between one (pose, landmark) pair: both builders refuse (g2o would build a
    duplicate Hpl block)."""
    from c_orb_slam_amd._lib import lib, ptr
    pr = ba_problem(2, n_local=4, n_fixed=2, n_pt=100)
    ek = np.ascontiguousarray(np.concatenate([pr["edge_kf"], pr["edge_kf"][:1]]), np.int32)
    ep = np.ascontiguousarray(np.concatenate([pr["edge_pt"], pr["edge_pt"][:1]]), np.int32)
    ne = len(ek)
    lv = np.zeros(ne, np.uint8)
    fx = _local_fixed(pr)
    kid = np.ascontiguousarray(pr["kf_id"], np.int32)
    pid = np.ascontiguousarray(pr["pt_id"], np.int32)
    out = np.zeros(64 * ne + 4096, np.int32)
    n = C.c_longlong()
    for gpu_ in (0, 1, 2):
        if fx[ek[0]]:
            pytest.skip("the duplicated edge hangs off a fixed keyframe")
        rc = lib().orbgpu_unit_ba_struct_all(len(kid), len(pid), ne, ptr(ek), ptr(ep), ptr(lv), ptr(fx), ptr(kid),
                                             ptr(pid), 0, gpu_, ptr(out), len(out), C.byref(n))
        assert rc == -1, (gpu_, rc)


@pytest.mark.parametrize("case", ["no_active_edges", "max_free_poses", "over_free_poses", "long_landmark",
                                  "descending_ids"])
def test_small_structure_edge_cases(gpu, case):
    """The one-workgroup builder (build_small, gpu = 2) at its limits: no active edge at the level,
    23 free poses (its maximum) and 24 (the multi-launch builder takes over), a landmark seen by
    every keyframe, point ids in descending order (the LDS bitonic sort) -- every list equal to
    the host's (_both compares all three builders)."""
    if case == "no_active_edges":
        pr = ba_problem(3, n_local=6, n_fixed=3, n_pt=200)
        h, g = _both(pr, _local_fixed(pr), np.zeros(len(pr["edge_pt"]), np.uint8), 1)
        assert h[:8].tolist()[:4] == [0, 0, 0, 0]
        return
    if case in ("max_free_poses", "over_free_poses"):
        nl = 24 if case == "max_free_poses" else 25   # kf_id 0 is fixed too: 23 / 24 free poses
        pr = ba_problem(11, n_local=nl, n_fixed=4, n_pt=900, obs_range=(2, 12))
    elif case == "long_landmark":
        pr = dict(ba_problem(12, n_local=14, n_fixed=8, n_pt=400))
        nkf = len(pr["kf_id"])
        seen = set(zip(pr["edge_kf"].tolist(), pr["edge_pt"].tolist()))
        add = [k for k in range(nkf) if (k, 0) not in seen]
        pr["edge_kf"] = np.concatenate([pr["edge_kf"], np.array(add, np.int32)])
        pr["edge_pt"] = np.concatenate([pr["edge_pt"], np.zeros(len(add), np.int32)])
    else:
        pr = dict(ba_problem(13, n_local=10, n_fixed=5, n_pt=700))
        pr["pt_id"] = (np.arange(len(pr["pt_id"]))[::-1] * 5 + 17).astype(np.int32)
    h, g = _both(pr, _local_fixed(pr))
    assert np.array_equal(h, g)
