"""Relocalization-shaped EPnP RANSAC problems.

N correspondences, 30% gross outliers; inliers are projections of random 3D
points (depth 5-50 m) under a random camera pose with sigma = 1 px x scale(level);
KITTI intrinsics; sigma^2 per level as ORBextractor (1.2^(2l)).
"""
import numpy as np

KITTI = (718.856, 718.856, 607.1928, 185.2157)


def rot(rng, max_deg=30.0):
    a = np.deg2rad(rng.uniform(-max_deg, max_deg, 3))
    cx, cy, cz = np.cos(a)
    sx, sy, sz = np.sin(a)
    Rx = np.array([[1, 0, 0], [0, cx, -sx], [0, sx, cx]])
    Ry = np.array([[cy, 0, sy], [0, 1, 0], [-sy, 0, cy]])
    Rz = np.array([[cz, -sz, 0], [sz, cz, 0], [0, 0, 1]])
    return Rz @ Ry @ Rx


def pnp_problem(seed, N, outlier_frac=0.3, K=KITTI, w=1241, h=376):
    rng = np.random.default_rng(seed)
    fx, fy, cx, cy = K
    R = rot(rng)
    t = rng.uniform(-2, 2, 3)
    u = rng.uniform(20, w - 20, N)
    v = rng.uniform(20, h - 20, N)
    d = rng.uniform(5, 50, N)
    Xc = np.stack([(u - cx) / fx * d, (v - cy) / fy * d, d], 1)
    Xw = (Xc - t) @ R            # R^T (Xc - t)
    octave = rng.integers(0, 8, N)
    scale = 1.2 ** octave
    uv = np.stack([u, v], 1) + rng.normal(0, 1.0, (N, 2)) * scale[:, None]
    nout = int(round(outlier_frac * N))
    out = rng.choice(N, nout, replace=False)
    uv[out] = np.stack([rng.uniform(0, w, nout), rng.uniform(0, h, nout)], 1)
    sigma2 = (np.float32(1.2) ** (2 * octave)).astype(np.float32)
    Tcw = np.eye(4, dtype=np.float32)
    Tcw[:3, :3] = R
    Tcw[:3, 3] = t
    # the reference packs only matched, non-bad map points; kp_idx maps them back
    n_matches = N + N // 5
    kp_idx = np.sort(rng.choice(n_matches, N, replace=False)).astype(np.int32)
    return dict(p3d=Xw.astype(np.float32), p2d=uv.astype(np.float32), sigma2=sigma2, kp_idx=kp_idx,
                n_matches=n_matches, K=K, Tcw=Tcw, outliers=out)
