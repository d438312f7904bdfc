"""Local-BA-shaped problems (EuRoC MH_05 stereo).

n_local local keyframes (the one with mnId 0 is fixed) + n_fixed fixed
keyframes; n_pt map points, each observed by U{2..8} keyframes (at least one
local); `stereo_frac` of the observations carry uRight; EuRoC intrinsics
(fx=fy=435.2047, cx=367.4517, cy=252.2009, bf=47.9064).  Noise: poses 1 cm /
0.5 deg, points 5 cm, pixels sigma = 1 x 1.2^octave, `outlier_frac` gross
outliers (20 px).  Edge order mimics the reference: map points in list order,
each point's observations in a per-point shuffled (pointer-map) order.
"""
import numpy as np

EUROC = (435.2047, 435.2047, 367.4517, 252.2009, 47.9064)


def _rot(rng, deg):
    a = np.deg2rad(rng.normal(0, deg, 3))
    th = np.linalg.norm(a)
    if th < 1e-12:
        return np.eye(3)
    k = a / th
    K = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
    return np.eye(3) + np.sin(th) * K + (1 - np.cos(th)) * K @ K


def ba_problem(seed=0, n_local=15, n_fixed=15, n_pt=3000, stereo_frac=0.7, outlier_frac=0.05, obs_range=(2, 8),
               cam=EUROC):
    rng = np.random.default_rng(seed)
    fx, fy, cx, cy, bf = cam
    nkf = n_local + n_fixed
    # keyframes along a gently curving path, all looking roughly +z
    Rwc, twc = [], []
    for k in range(nkf):
        Rwc.append(_rot(rng, 2.0))
        twc.append(np.array([0.15 * k, 0.02 * np.sin(k), 0.05 * k]) + rng.normal(0, 0.02, 3))
    Tcw_true = []
    for R, t in zip(Rwc, twc):
        T = np.eye(4)
        T[:3, :3] = R.T
        T[:3, 3] = -R.T @ t
        Tcw_true.append(T)
    # points in front of the middle of the path
    Xw = np.stack([rng.uniform(-4, 9, n_pt), rng.uniform(-2.5, 2.5, n_pt), rng.uniform(3, 12, n_pt)], 1)
    ids = rng.permutation(np.arange(1, nkf + 200))[:nkf]
    local = np.zeros(nkf, np.uint8)
    local[:n_local] = 1
    ids[0] = 0                                   # the first local keyframe is the map origin (fixed)
    edges_pt, edges_kf, obs, isig = [], [], [], []
    lo, hi = obs_range
    W, H = 2 * cx, 2 * cy

    def visible(p, kf):
        T = Tcw_true[kf]
        Xc = T[:3, :3] @ Xw[p] + T[:3, 3]
        if Xc[2] < 1.0:
            return False
        u, v = fx * Xc[0] / Xc[2] + cx, fy * Xc[1] / Xc[2] + cy
        return 10 <= u < W - 10 and 10 <= v < H - 10

    for p in range(n_pt):
        while True:
            vis = [kf for kf in range(nkf) if visible(p, kf)]
            if len(vis) >= lo and any(local[kf] for kf in vis):
                break
            Xw[p] = [rng.uniform(-4, 9), rng.uniform(-2.5, 2.5), rng.uniform(3, 12)]
        k = min(int(rng.integers(lo, hi + 1)), len(vis))
        kfs = rng.choice(vis, k, replace=False)
        if not local[kfs].any():
            kfs[0] = rng.choice([kf for kf in vis if local[kf]])
            kfs = np.unique(kfs)
        rng.shuffle(kfs)
        for kf in kfs:
            T = Tcw_true[kf]
            Xc = T[:3, :3] @ Xw[p] + T[:3, 3]
            octv = int(rng.integers(0, 8))
            s = 1.2 ** octv
            u = fx * Xc[0] / Xc[2] + cx + rng.normal(0, s)
            v = fy * Xc[1] / Xc[2] + cy + rng.normal(0, s)
            ur = -1.0
            if rng.random() < stereo_frac:
                ur = u - bf / Xc[2] + rng.normal(0, s)
            if rng.random() < outlier_frac:
                a = rng.uniform(0, 2 * np.pi)
                u += 20 * np.cos(a)
                v += 20 * np.sin(a)
                if ur >= 0:
                    ur += 20 * np.cos(a)
            if ur < 0 and ur != -1.0:
                ur = 0.0
            edges_pt.append(p)
            edges_kf.append(kf)
            obs.append((u, v, ur))
            isig.append(np.float32(1.0) / np.float32(1.2) ** (2 * octv))
    # noisy initial estimates (the fixed keyframes and the origin keep their true pose)
    Tcw0 = np.zeros((nkf, 16), np.float32)
    for k in range(nkf):
        T = Tcw_true[k].copy()
        if local[k] and ids[k] != 0:
            T[:3, :3] = _rot(rng, 0.5) @ T[:3, :3]
            T[:3, 3] += rng.normal(0, 0.01, 3)
        Tcw0[k] = T.astype(np.float32).ravel()
    X0 = (Xw + rng.normal(0, 0.05, Xw.shape)).astype(np.float32)
    kcam = np.tile(np.array(cam, np.float32), (nkf, 1))
    pt_ids = rng.permutation(np.arange(10, 10 + 4 * n_pt))[:n_pt].astype(np.int32)
    return dict(kf_id=ids.astype(np.int32), kf_Tcw=Tcw0, kf_local=local, kf_cam=kcam, pt_id=pt_ids, pt_pos=X0,
                edge_pt=np.array(edges_pt, np.int32), edge_kf=np.array(edges_kf, np.int32),
                edge_obs=np.array(obs, np.float32), edge_inv_sigma2=np.array(isig, np.float32),
                Tcw_true=np.array(Tcw_true), Xw_true=Xw)


KITTI = (718.856, 718.856, 607.1928, 185.2157, 386.1448)   # Stereo/KITTI00-02.yaml:8-25
KITTI_WH = (1241, 376)


def _rot_y(a):
    c, s = np.cos(a), np.sin(a)
    return np.array([[c, 0, s], [0, 1, 0], [-s, 0, c]])


def global_ba_problem(seed=0, n_kf=64, pts_per_kf=150, obs_range=(3, 10), stereo_frac=0.5, cam=KITTI,
                      pose_noise=(0.02, 0.2), point_noise=0.1, laps=0, loop_frac=0.05, loop_obs=(1, 3)):
    """Merged-map global-BA-shaped problem (KITTI intrinsics).

    Keyframes ~1 m apart along a gently turning drive; each keyframe creates `pts_per_kf`
    points 5-40 m ahead, each observed by U{obs_range} consecutive keyframes starting at
    its creator (visibility-checked, >= 2 observations).  No gross outliers: LoopClosing
    runs BundleAdjustment with bRobust=false (LoopClosing.cc:650).  Keyframe mnId = index
    (id 0 fixed); edges in map-point order, each point's observations in shuffled order.
    Vectorised numpy (10^5-10^6 edges in seconds).

    laps >= 2: the drive is a circuit driven `laps` times (n_kf / laps keyframes per lap, each
    lap 0.5 m further out), the shape of a map whose loops LoopClosing has closed before
    GlobalBundleAdjustemnt runs (LoopClosing.cc:231-360, 650): a `loop_frac` share of the
    points is also observed by U{loop_obs} keyframes at the same place on every other lap (the
    observations SearchAndFuse adds), so keyframes far apart in mnId share points and the
    pose system gains long-range covisibility, not just a band."""
    rng = np.random.default_rng(seed)
    fx, fy, cx, cy, bf = cam
    W, H = KITTI_WH
    if laps >= 2:
        n_lap = n_kf // laps
        idx = np.arange(n_kf)
        yaw = 2 * np.pi * (idx % n_lap) / n_lap + rng.normal(0, 0.002, n_kf)
        R = n_lap / (2 * np.pi) + 0.5 * (idx // n_lap)
        twc = np.stack([R - R * np.cos(yaw), rng.normal(0, 0.05, n_kf), R * np.sin(yaw)], 1)
    else:
        yaw = np.cumsum(rng.normal(0, 0.02, n_kf))
        step = np.stack([np.sin(yaw), np.zeros(n_kf), np.cos(yaw)], 1)
        twc = np.cumsum(step, 0) - step[0]
    Rwc = np.stack([_rot_y(a) for a in yaw])
    Rcw = np.transpose(Rwc, (0, 2, 1))
    tcw = -np.einsum("kij,kj->ki", Rcw, twc)
    # candidate points in each creator keyframe's frame
    n = n_kf * pts_per_kf
    creator = np.repeat(np.arange(n_kf), pts_per_kf)
    z = rng.uniform(5, 40, n)
    u = rng.uniform(20, W - 20, n)
    v = rng.uniform(20, H - 20, n)
    Xc = np.stack([(u - cx) / fx * z, (v - cy) / fy * z, z], 1)
    Xw = np.einsum("nij,nj->ni", Rwc[creator], Xc) + twc[creator]
    lo, hi = obs_range
    k = rng.integers(lo, hi + 1, n)
    pe, ke = [], []
    for j in range(hi):                               # j-th observer = creator + j
        kf = creator + j
        ok = (j < k) & (kf < n_kf)
        kfc = np.minimum(kf, n_kf - 1)
        Xcj = np.einsum("nij,nj->ni", Rcw[kfc], Xw) + tcw[kfc]
        zz = Xcj[:, 2]
        with np.errstate(divide="ignore", invalid="ignore"):
            uu, vv = fx * Xcj[:, 0] / zz + cx, fy * Xcj[:, 1] / zz + cy
        ok &= (zz > 1.0) & (uu >= 10) & (uu < W - 10) & (vv >= 10) & (vv < H - 10)
        pe.append(np.flatnonzero(ok))
        ke.append(kf[ok])
    if laps >= 2:   # loop closures: the same place on the other laps
        lp = np.flatnonzero(rng.random(n) < loop_frac)
        kl = rng.integers(loop_obs[0], loop_obs[1] + 1, len(lp))
        base = creator[lp] % n_lap
        for m in range(laps):
            for j in range(loop_obs[1]):
                kf = base + m * n_lap + j
                ok = (j < kl) & (kf < n_kf) & (kf // n_lap != creator[lp] // n_lap) & (kf != creator[lp])
                kfc = np.minimum(kf, n_kf - 1)
                Xcj = np.einsum("nij,nj->ni", Rcw[kfc], Xw[lp]) + tcw[kfc]
                zz = Xcj[:, 2]
                with np.errstate(divide="ignore", invalid="ignore"):
                    uu, vv = fx * Xcj[:, 0] / zz + cx, fy * Xcj[:, 1] / zz + cy
                ok &= (zz > 1.0) & (uu >= 10) & (uu < W - 10) & (vv >= 10) & (vv < H - 10)
                pe.append(lp[ok])
                ke.append(kf[ok])
    pe, ke = np.concatenate(pe), np.concatenate(ke)
    # one observation per (point, keyframe) (a KeyFrame holds a MapPoint once)
    _, first = np.unique(pe.astype(np.int64) * n_kf + ke, return_index=True)
    pe, ke = pe[np.sort(first)], ke[np.sort(first)]
    cnt = np.bincount(pe, minlength=n)
    keep = cnt >= 2
    newid = np.cumsum(keep) - 1
    m = keep[pe]
    pe, ke = newid[pe[m]], ke[m]
    Xw = Xw[keep]
    npt = len(Xw)
    # edge order: by point, then a per-point shuffle (observation map order)
    order = np.lexsort((rng.random(len(pe)), pe))
    pe, ke = pe[order], ke[order]
    Xc = np.einsum("nij,nj->ni", Rcw[ke], Xw[pe]) + tcw[ke]
    octv = rng.integers(0, 8, len(pe))
    s = 1.2 ** octv
    uu = fx * Xc[:, 0] / Xc[:, 2] + cx + rng.normal(0, 1, len(pe)) * s
    vv = fy * Xc[:, 1] / Xc[:, 2] + cy + rng.normal(0, 1, len(pe)) * s
    ur = np.where(rng.random(len(pe)) < stereo_frac, uu - bf / Xc[:, 2] + rng.normal(0, 1, len(pe)) * s, -1.0)
    ur = np.where((ur < 0) & (ur != -1.0), 0.0, ur)
    isig = (np.float32(1.0) / np.float32(1.2) ** (2 * octv)).astype(np.float32)
    Tcw0 = np.zeros((n_kf, 16), np.float32)
    Tcw_true = np.zeros((n_kf, 4, 4))
    for kk in range(n_kf):
        T = np.eye(4)
        T[:3, :3] = Rcw[kk]
        T[:3, 3] = tcw[kk]
        Tcw_true[kk] = T
        if kk:
            T = T.copy()
            T[:3, :3] = _rot(rng, pose_noise[1]) @ T[:3, :3]
            T[:3, 3] += rng.normal(0, pose_noise[0], 3)
        Tcw0[kk] = T.astype(np.float32).ravel()
    X0 = (Xw + rng.normal(0, point_noise, Xw.shape)).astype(np.float32)
    return dict(kf_id=np.arange(n_kf, dtype=np.int32), kf_Tcw=Tcw0, kf_local=np.ones(n_kf, np.uint8),
                kf_cam=np.tile(np.array(cam, np.float32), (n_kf, 1)),
                pt_id=np.arange(npt, dtype=np.int32) + 1, pt_pos=X0,
                edge_pt=pe.astype(np.int32), edge_kf=ke.astype(np.int32),
                edge_obs=np.stack([uu, vv, ur], 1).astype(np.float32), edge_inv_sigma2=isig,
                Tcw_true=Tcw_true, Xw_true=Xw)
