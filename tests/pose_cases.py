"""Optimizer::PoseOptimization-shaped problems (Tracking: TrackWithMotionModel /
TrackLocalMap, Tracking.cc:885-1010): one frame, N keypoints of which a fraction carry a
map point; KITTI intrinsics; stereo observations with mvuRight; the initial pose is the
true one perturbed (motion-model prediction); pixel noise sigma = 1.2^octave; gross outliers."""
import numpy as np

KITTI = (718.856, 718.856, 607.1928, 185.2157, 386.1448)


def _rot(rng, deg):
    a = np.deg2rad(rng.normal(0, deg, 3))
    th = np.linalg.norm(a)
    k = a / th
    K = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
    return np.eye(3) + np.sin(th) * K + (1 - np.cos(th)) * K @ K


def pose_problem(seed=0, N=1500, mp_frac=0.7, stereo_frac=0.6, outlier_frac=0.1, rot_deg=0.5, trans=0.05, cam=KITTI):
    rng = np.random.default_rng(seed)
    fx, fy, cx, cy, bf = cam
    W, H = 1241, 376
    R = _rot(rng, 2.0)
    t = rng.normal(0, 1.0, 3)
    u = rng.uniform(20, W - 20, N)
    v = rng.uniform(20, H - 20, N)
    z = rng.uniform(4, 60, N)
    Xc = np.stack([(u - cx) / fx * z, (v - cy) / fy * z, z], 1)
    Xw = (Xc - t) @ R            # Xc = R Xw + t
    octv = rng.integers(0, 8, N)
    s = 1.2 ** octv
    obs_u = u + rng.normal(0, 1, N) * s
    obs_v = v + rng.normal(0, 1, N) * s
    ur = np.where(rng.random(N) < stereo_frac, obs_u - bf / z + rng.normal(0, 1, N) * s, -1.0)
    out = rng.random(N) < outlier_frac
    ang = rng.uniform(0, 2 * np.pi, N)
    obs_u = np.where(out, obs_u + 25 * np.cos(ang), obs_u)
    obs_v = np.where(out, obs_v + 25 * np.sin(ang), obs_v)
    ur = np.where(out & (ur >= 0), ur + 25 * np.cos(ang), ur)
    ur = np.where((ur < 0) & (ur != -1.0), 0.0, ur)
    T_true = np.eye(4)
    T_true[:3, :3] = R
    T_true[:3, 3] = t
    T0 = T_true.copy()
    T0[:3, :3] = _rot(rng, rot_deg) @ R
    T0[:3, 3] = t + rng.normal(0, trans, 3)
    isig = (np.float32(1.0) / np.float32(1.2) ** (2 * octv)).astype(np.float32)
    return dict(Tcw=T0.astype(np.float32), has_mp=(rng.random(N) < mp_frac).astype(np.uint8),
                Xw=Xw.astype(np.float32), obs=np.stack([obs_u, obs_v, ur], 1).astype(np.float32),
                inv_sigma2=isig, cam=np.array(cam, np.float32), T_true=T_true, gross=out)
