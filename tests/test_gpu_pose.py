"""Optimizer::PoseOptimization (Optimizer.cc:239-451) on the GPU vs the CPU oracle.

One persistent workgroup per frame runs the whole call (4 rounds x optimize(10), chi2
classification, robust kernel dropped after round 3).  The per-iteration 6x6 system is
summed in the oracle's canonical order and the pivoted LDL^T / SE3 update / LM control
are the same operation sequence -> the pose (float Tcw), outlier flags and inlier count
are bit-identical to oracle/ba.c ora_pose_optimization.
"""
import numpy as np
import pytest

import oracle_lib
from pose_cases import pose_problem

pytestmark = pytest.mark.gpu


def _check(pr, n, T, outl):
    o = oracle_lib.oracle_pose_optimization(pr)
    assert n == o["inliers"]
    assert np.array_equal(T, o["Tcw"])
    mp = pr["has_mp"].astype(bool)
    assert np.array_equal(outl[mp], o["outlier"][mp])
    return o


@pytest.mark.parametrize("seed", range(6))
def test_pose_matches_oracle(gpu, seed):
    from c_orb_slam_amd import PoseOptimization
    pr = pose_problem(seed)
    n, T, outl = PoseOptimization(pr)
    o = _check(pr, n, T, outl)
    # the synthetic gross outliers end up flagged, the pose moves toward the truth
    gross = pr["gross"] & pr["has_mp"].astype(bool)
    assert outl[gross].mean() > 0.9
    assert np.linalg.norm(T[:3, 3] - pr["T_true"][:3, 3]) < np.linalg.norm(pr["Tcw"][:3, 3] - pr["T_true"][:3, 3])
    assert o["inliers"] > 0


@pytest.mark.parametrize("kw", [dict(stereo_frac=0.0), dict(stereo_frac=1.0), dict(outlier_frac=0.45),
                                dict(N=12, mp_frac=1.0), dict(N=40, mp_frac=0.3), dict(N=5800, mp_frac=0.7),
                                dict(rot_deg=3.0, trans=0.5), dict(outlier_frac=0.95, N=300)])
def test_pose_edge_cases(gpu, kw):
    from c_orb_slam_amd import PoseOptimization
    pr = pose_problem(7, **kw)
    n, T, outl = PoseOptimization(pr)
    _check(pr, n, T, outl)


def test_pose_too_few_correspondences(gpu):
    from c_orb_slam_amd import PoseOptimization
    pr = pose_problem(3, N=30)
    pr["has_mp"][:] = 0
    pr["has_mp"][[4, 9]] = 1
    prev = np.full(30, 7, np.uint8)
    n, T, outl = PoseOptimization(pr, prev)
    assert n == 0
    assert np.array_equal(T, pr["Tcw"])
    assert outl[4] == 0 and outl[9] == 0 and (np.delete(outl, [4, 9]) == 7).all()


def test_pose_outlier_rows_without_map_point_untouched(gpu):
    from c_orb_slam_amd import PoseOptimization
    pr = pose_problem(11, N=400)
    prev = np.full(400, 5, np.uint8)
    _, _, outl = PoseOptimization(pr, prev)
    mp = pr["has_mp"].astype(bool)
    assert (outl[~mp] == 5).all() and set(np.unique(outl[mp])) <= {0, 1}


def test_pose_batch_equals_single(gpu):
    from c_orb_slam_amd import PoseOptimization, PoseOptimizationBatch
    frames = [pose_problem(s, N=600 + 300 * s) for s in range(5)]
    n, T, outs = PoseOptimizationBatch(frames)
    for f, pr in enumerate(frames):
        n1, T1, o1 = PoseOptimization(pr)
        assert n[f] == n1 and np.array_equal(T[f], T1) and np.array_equal(outs[f], o1)


def test_pose_capacity(gpu):
    from c_orb_slam_amd import PoseOptimization
    from c_orb_slam_amd._lib import OrbGpuError
    pr = pose_problem(1, N=8300, mp_frac=1.0)
    with pytest.raises(OrbGpuError):
        PoseOptimization(pr)


def test_pose_device_mode_equals_host(gpu):
    import torch
    from c_orb_slam_amd import PoseOptimizationBatch
    from c_orb_slam_amd.optimizer import PoseOptimizationBatchDevice
    frames = [pose_problem(20 + s, N=500 + 700 * s) for s in range(4)]
    frames.append(pose_problem(30, N=20, mp_frac=0.1))           # < 3 correspondences
    frames[-1]["has_mp"][:] = 0
    frames[-1]["has_mp"][:2] = 1
    n_h, T_h, o_h = PoseOptimizationBatch(frames)
    dev = torch.device("cuda", 0)
    df = [dict(Tcw=torch.from_numpy(np.ascontiguousarray(f["Tcw"], np.float32).reshape(16)).to(dev),
               has_mp=torch.from_numpy(f["has_mp"]).to(dev), Xw=torch.from_numpy(f["Xw"]).to(dev),
               obs=torch.from_numpy(f["obs"]).to(dev), inv_sigma2=torch.from_numpy(f["inv_sigma2"]).to(dev),
               cam=f["cam"]) for f in frames]
    T_d = [torch.zeros(16, dtype=torch.float32, device=dev) for _ in frames]
    o_d = [torch.full((len(f["has_mp"]),), 9, dtype=torch.uint8, device=dev) for f in frames]
    n_d = PoseOptimizationBatchDevice(df, T_d, o_d)
    assert np.array_equal(n_d, n_h)
    for f, fr in enumerate(frames):
        assert np.array_equal(T_d[f].cpu().numpy().reshape(4, 4), T_h[f])
        mp = fr["has_mp"].astype(bool)
        od = o_d[f].cpu().numpy()
        assert np.array_equal(od[mp], o_h[f][mp]) and (od[~mp] == 9).all()
