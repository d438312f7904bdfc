"""Seeded synthetic inputs shaped like the reference's benchmark sequences.

The datasets the reference is run on (KITTI, EuRoC, TUM) are not available
(SURVEY.md F5), so every measurement and parity case uses these generators.
SURVEY.md §8(d) config 2: piecewise-constant random rectangles (values
U[0,255]) over a smooth gradient, additive Gaussian noise sigma=3, clamped to
u8; frame t+1 is frame t warped by a small homography (<=3 px shift, <=1 deg
rotation).
"""
import numpy as np

KITTI_W, KITTI_H = 1241, 376


def textured_image(rng, w=KITTI_W, h=KITTI_H, n_rects=None):
    if n_rects is None:
        n_rects = max(40, (w * h) // 400)
    yy, xx = np.mgrid[0:h, 0:w].astype(np.float32)
    gx, gy = rng.uniform(-0.1, 0.1, size=2)
    img = 110.0 + gx * (xx - w / 2) + gy * (yy - h / 2)
    for _ in range(n_rects):
        big = rng.random() < 0.1
        rw = rng.integers(6, max(8, w // (6 if big else 40)))
        rh = rng.integers(6, max(8, h // (4 if big else 20)))
        x0, y0 = rng.integers(-rw // 2, w), rng.integers(-rh // 2, h)
        img[max(0, y0):max(0, y0 + rh), max(0, x0):max(0, x0 + rw)] = rng.uniform(0, 255)
    img += rng.normal(0.0, 3.0, size=img.shape)
    return np.clip(np.rint(img), 0, 255).astype(np.uint8)


# KITTI-00 intrinsics (Examples/Stereo/KITTI00-02.yaml:8-25); other sizes scale them.
KITTI_K = (718.856, 718.856, 607.1928, 185.2157)
KITTI_BF = 386.1448


def intrinsics(w, h):
    if (w, h) == (KITTI_W, KITTI_H):
        return KITTI_K
    s = w / KITTI_W
    return (KITTI_K[0] * s, KITTI_K[1] * s, w / 2.0, h / 2.0)


def small_rotation(rng, fx, max_shift=3.0, max_rot_deg=1.0):
    """Camera rotation: roll <= 1 deg, pan/tilt shifting the image <= 3 px."""
    roll = np.deg2rad(rng.uniform(-max_rot_deg, max_rot_deg))
    yaw, pitch = rng.uniform(-max_shift, max_shift, size=2) / fx
    cz, sz = np.cos(roll), np.sin(roll)
    cy_, sy_ = np.cos(yaw), np.sin(yaw)
    cp, sp = np.cos(pitch), np.sin(pitch)
    Rz = np.array([[cz, -sz, 0], [sz, cz, 0], [0, 0, 1.0]])
    Ry = np.array([[cy_, 0, sy_], [0, 1.0, 0], [-sy_, 0, cy_]])
    Rx = np.array([[1.0, 0, 0], [0, cp, -sp], [0, sp, cp]])
    return Rz @ Ry @ Rx


def rotation_homography(K4, R):
    fx, fy, cx, cy = K4
    K = np.array([[fx, 0, cx], [0, fy, cy], [0, 0, 1.0]])
    return K @ R @ np.linalg.inv(K)


def warp(img, H):
    """Bilinear warp: out(x) = img(H^-1 x), border replicate; returns u8."""
    h, w = img.shape
    Hi = np.linalg.inv(H)
    yy, xx = np.mgrid[0:h, 0:w].astype(np.float64)
    den = Hi[2, 0] * xx + Hi[2, 1] * yy + Hi[2, 2]
    sx = (Hi[0, 0] * xx + Hi[0, 1] * yy + Hi[0, 2]) / den
    sy = (Hi[1, 0] * xx + Hi[1, 1] * yy + Hi[1, 2]) / den
    sx = np.clip(sx, 0, w - 1.001)
    sy = np.clip(sy, 0, h - 1.001)
    x0, y0 = np.floor(sx).astype(np.int64), np.floor(sy).astype(np.int64)
    fx, fy = sx - x0, sy - y0
    f = img.astype(np.float64)
    v = (f[y0, x0] * (1 - fx) * (1 - fy) + f[y0, x0 + 1] * fx * (1 - fy)
         + f[y0 + 1, x0] * (1 - fx) * fy + f[y0 + 1, x0 + 1] * fx * fy)
    return np.clip(np.rint(v), 0, 255).astype(np.uint8)


def sequence(seed, n_frames, w=KITTI_W, h=KITTI_H, return_rotations=False):
    """n_frames u8 images (n, h, w); frame t+1 is frame t seen by the camera
    rotated by R_t (homography K R K^-1) plus +-2 grey levels of noise.
    Returns (frames, Hs) or (frames, Hs, Rs)."""
    rng = np.random.default_rng(seed)
    K4 = intrinsics(w, h)
    frames = [textured_image(rng, w, h)]
    Hs, Rs = [], []
    for _ in range(n_frames - 1):
        R = small_rotation(rng, K4[0])
        H = rotation_homography(K4, R)
        nxt = warp(frames[-1], H)
        nxt = np.clip(nxt.astype(np.int16) + rng.integers(-2, 3, size=nxt.shape), 0, 255).astype(np.uint8)
        frames.append(nxt)
        Hs.append(H)
        Rs.append(R)
    if return_rotations:
        return np.stack(frames), Hs, Rs
    return np.stack(frames), Hs


def lift_map_points(rng, kps, K4, depth_range=(5.0, 50.0)):
    """World points (camera frame of the last frame = world) for keypoints: X = d K^-1 [u v 1]."""
    fx, fy, cx, cy = K4
    d = rng.uniform(*depth_range, size=len(kps))
    X = np.stack([(kps["x"] - cx) / fx * d, (kps["y"] - cy) / fy * d, d], axis=1)
    return X.astype(np.float32)


def pose_from_rotation(R, t=(0.0, 0.0, 0.0)):
    T = np.eye(4, dtype=np.float32)
    T[:3, :3] = R
    T[:3, 3] = t
    return T


def stereo_pair(rng, w=KITTI_W, h=KITTI_H, n_rects=None, max_disp=64):
    """Rectified stereo pair: the right image is the left one with every
    rectangle shifted left by its own integer disparity in [0, max_disp]; independent sensor noise."""
    if n_rects is None:
        n_rects = max(40, (w * h) // 400)
    yy, xx = np.mgrid[0:h, 0:w].astype(np.float32)
    gx, gy = rng.uniform(-0.1, 0.1, size=2)
    base = 110.0 + gx * (xx - w / 2) + gy * (yy - h / 2)
    left, right = base.copy(), base.copy()
    for _ in range(n_rects):
        big = rng.random() < 0.1
        rw = rng.integers(6, max(8, w // (6 if big else 40)))
        rh = rng.integers(6, max(8, h // (4 if big else 20)))
        x0, y0 = rng.integers(-rw // 2, w), rng.integers(-rh // 2, h)
        v = rng.uniform(0, 255)
        d = int(rng.integers(0, max_disp + 1))
        left[max(0, y0):max(0, y0 + rh), max(0, x0):max(0, x0 + rw)] = v
        right[max(0, y0):max(0, y0 + rh), max(0, x0 - d):max(0, x0 - d + rw)] = v
    out = []
    for img in (left, right):
        img = img + rng.normal(0.0, 3.0, size=img.shape)
        out.append(np.clip(np.rint(img), 0, 255).astype(np.uint8))
    return out[0], out[1]


def stereo_batch(seed, n, w=KITTI_W, h=KITTI_H):
    """n independent stereo pairs: (lefts, rights), each (n, h, w) u8."""
    rng = np.random.default_rng(seed)
    pairs = [stereo_pair(rng, w, h) for _ in range(n)]
    return np.stack([p[0] for p in pairs]), np.stack([p[1] for p in pairs])


def stereo_sequence(seed, n_frames, w=KITTI_W, h=KITTI_H, return_rotations=False):
    """Left frames as in sequence(); right frame = left resampled with a smooth ground-plane-like
    disparity field d(x, y) = 4 + 36 * y / h (+-2 px ripple), plus independent noise."""
    out = sequence(seed, n_frames, w, h, return_rotations=True)
    lefts = out[0]
    rng = np.random.default_rng(seed + 7919)
    yy, xx = np.mgrid[0:h, 0:w].astype(np.float64)
    d = 4.0 + 36.0 * yy / h + 2.0 * np.sin(xx / 37.0)
    sx = np.clip(xx + d, 0, w - 1.001)
    x0 = np.floor(sx).astype(np.int64)
    fx = sx - x0
    rights = []
    for L in lefts:
        f = L.astype(np.float64)
        yi = yy.astype(np.int64)
        v = f[yi, x0] * (1 - fx) + f[yi, x0 + 1] * fx
        v += rng.normal(0.0, 1.0, size=v.shape)
        rights.append(np.clip(np.rint(v), 0, 255).astype(np.uint8))
    rights = np.stack(rights)
    if return_rotations:
        return lefts, rights, out[1], out[2]
    return lefts, rights
