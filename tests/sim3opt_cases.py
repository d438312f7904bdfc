"""Optimizer::OptimizeSim3-shaped problems (LoopClosing::ComputeSim3, LoopClosing.cc:320-326):
keyframe 1 (current) and keyframe 2 (loop candidate) share a set of map-point matches; the
initial g2o::Sim3 is the Sim3Solver estimate (truth perturbed); pixel noise sigma = 1.2^octave;
gross outliers; th2 = 10; bFixScale true for stereo, false for monocular."""
import numpy as np

KITTI4 = (718.856, 718.856, 607.1928, 185.2157)


def _rot(rng, deg):
    a = np.deg2rad(rng.normal(0, deg, 3))
    th = np.linalg.norm(a)
    k = a / th
    K = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
    return np.eye(3) + np.sin(th) * K + (1 - np.cos(th)) * K @ K


def sim3opt_problem(seed=0, N=600, match_frac=0.3, outlier_frac=0.15, fix_scale=True, rot_deg=1.0, trans=0.05,
                    scale_noise=0.02, cam1=KITTI4, cam2=KITTI4, th2=10.0):
    """Returns the problem dict (oracle/C-ABI field names) plus the true and initial Sim3 (R, t, s)."""
    rng = np.random.default_rng(seed)
    W, H = 1241, 376
    fx1, fy1, cx1, cy1 = cam1
    fx2, fy2, cx2, cy2 = cam2
    # true S12: X1 = s R X2 + t
    R = _rot(rng, 8.0)
    t = rng.normal(0, 1.5, 3)
    s = 1.0 if fix_scale else float(np.exp(rng.normal(0, 0.3)))
    u1 = rng.uniform(10, W - 10, N)
    v1 = rng.uniform(10, H - 10, N)
    z1 = rng.uniform(5, 50, N)
    X1 = np.stack([(u1 - cx1) / fx1 * z1, (v1 - cy1) / fy1 * z1, z1], 1)
    X2 = ((X1 - t) @ R) / s            # X2 = R^T (X1 - t) / s
    p2 = X2[:, :2] / X2[:, 2:3]
    u2 = p2[:, 0] * fx2 + cx2
    v2 = p2[:, 1] * fy2 + cy2
    oct1 = rng.integers(0, 8, N)
    oct2 = np.clip(oct1 + rng.integers(-1, 2, N), 0, 7)
    valid = (rng.random(N) < match_frac) & (X2[:, 2] > 0.5)
    out = rng.random(N) < outlier_frac
    ang = rng.uniform(0, 2 * np.pi, N)
    o1 = np.stack([u1, v1], 1) + rng.normal(0, 1, (N, 2)) * (1.2 ** oct1)[:, None]
    o2 = np.stack([u2, v2], 1) + rng.normal(0, 1, (N, 2)) * (1.2 ** oct2)[:, None]
    o2 = np.where(out[:, None], o2 + 30 * np.stack([np.cos(ang), np.sin(ang)], 1), o2)
    # 3-D points carry depth noise (they are map points, not ground truth)
    X1n = X1 * (1 + rng.normal(0, 0.005, (N, 1)))
    X2n = X2 * (1 + rng.normal(0, 0.005, (N, 1)))
    R0 = _rot(rng, rot_deg) @ R
    t0 = t + rng.normal(0, trans, 3)
    s0 = s if fix_scale else s * float(np.exp(rng.normal(0, scale_noise)))
    isig1 = (np.float32(1.0) / np.float32(1.2) ** (2 * oct1)).astype(np.float32)
    isig2 = (np.float32(1.0) / np.float32(1.2) ** (2 * oct2)).astype(np.float32)
    return dict(N=N, valid=valid.astype(np.uint8), X1c=X1n.astype(np.float32), X2c=X2n.astype(np.float32),
                obs1=o1.astype(np.float32), obs2=o2.astype(np.float32), inv_sigma2_1=isig1, inv_sigma2_2=isig2,
                K1=np.array(cam1, np.float32), K2=np.array(cam2, np.float32), th2=np.float32(th2),
                bFixScale=int(fix_scale), R0=R0.astype(np.float32), t0=t0.astype(np.float32), s0=np.float32(s0),
                R_true=R, t_true=t, s_true=s, gross=out & valid)
