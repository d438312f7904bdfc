"""Loop-closure-shaped Sim3 RANSAC problems (LoopClosing.cc:333-389).

N matched map-point pairs between two keyframes: X1c (KF1 camera frame,
depth 5-50 m); X2c = S21 X1c for a random similarity (scale 1 for stereo /
bFixScale, 0.5-2 for monocular drift) with 1 px x scale(level) image noise
re-lifted at the same depth; `outlier_frac` gross outliers.  KITTI intrinsics
for both keyframes; sigma^2 per level as ORBextractor (1.2^(2l)).
"""
import numpy as np

from pnp_cases import KITTI, rot


def _project(X, K):
    fx, fy, cx, cy = K
    return np.stack([fx * X[:, 0] / X[:, 2] + cx, fy * X[:, 1] / X[:, 2] + cy], 1)


def _lift(uv, d, K):
    fx, fy, cx, cy = K
    return np.stack([(uv[:, 0] - cx) / fx * d, (uv[:, 1] - cy) / fy * d, d], 1)


def sim3_problem(seed, N, outlier_frac=0.4, fix_scale=True, K=KITTI, w=1241, h=376):
    rng = np.random.default_rng(seed)
    uv1 = np.stack([rng.uniform(20, w - 20, N), rng.uniform(20, h - 20, N)], 1)
    d1 = rng.uniform(5, 50, N)
    X1 = _lift(uv1, d1, K)
    R12 = rot(rng, 10.0)
    t12 = rng.uniform(-1, 1, 3)
    s12 = 1.0 if fix_scale else float(rng.uniform(0.5, 2.0))
    # X1 = s12 R12 X2 + t12  =>  X2 = R12^T (X1 - t12) / s12
    X2 = ((X1 - t12) @ R12) / s12
    oct1 = rng.integers(0, 8, N)
    oct2 = rng.integers(0, 8, N)
    uv2 = _project(X2, K) + rng.normal(0, 1.0, (N, 2)) * (1.2 ** oct2)[:, None]
    X2 = _lift(uv2, X2[:, 2], K)
    uv1n = uv1 + rng.normal(0, 1.0, (N, 2)) * (1.2 ** oct1)[:, None]
    X1 = _lift(uv1n, d1, K)
    nout = int(round(outlier_frac * N))
    out = rng.choice(N, nout, replace=False)
    X2[out] = _lift(np.stack([rng.uniform(0, w, nout), rng.uniform(0, h, nout)], 1), rng.uniform(5, 50, nout), K)
    s2_1 = (np.float32(1.2) ** (2 * oct1)).astype(np.float32)
    s2_2 = (np.float32(1.2) ** (2 * oct2)).astype(np.float32)
    N1 = N + N // 3
    idx1 = np.sort(rng.choice(N1, N, replace=False)).astype(np.int32)
    T12 = np.eye(4)
    T12[:3, :3] = s12 * R12
    T12[:3, 3] = t12
    Kv = np.array(K, np.float32)
    return dict(X1=X1.astype(np.float32), X2=X2.astype(np.float32), s1=s2_1, s2=s2_2, idx1=idx1, N1=N1, K1=Kv,
                K2=Kv, fix=fix_scale, T12=T12, s=s12, outliers=out)
