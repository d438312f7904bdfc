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


def small_homography(rng, w=KITTI_W, h=KITTI_H, max_shift=3.0, max_rot_deg=1.0):
    th = np.deg2rad(rng.uniform(-max_rot_deg, max_rot_deg))
    tx, ty = rng.uniform(-max_shift, max_shift, size=2)
    c, s = np.cos(th), np.sin(th)
    cx, cy = w / 2.0, h / 2.0
    # rotate about the image centre, then translate
    H = np.array([[c, -s, cx - c * cx + s * cy + tx],
                  [s, c, cy - s * cx - c * cy + ty],
                  [0, 0, 1.0]])
    return H


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


def sequence(seed, n_frames, w=KITTI_W, h=KITTI_H):
    """n_frames u8 images (n, h, w) and the n-1 homographies frame t -> t+1."""
    rng = np.random.default_rng(seed)
    frames = [textured_image(rng, w, h)]
    Hs = []
    for _ in range(n_frames - 1):
        H = small_homography(rng, w, h)
        nxt = warp(frames[-1], H)
        nxt = np.clip(nxt.astype(np.int16) + rng.integers(-2, 3, size=nxt.shape), 0, 255).astype(np.uint8)
        frames.append(nxt)
        Hs.append(H)
    return np.stack(frames), Hs
