"""Oracle checks for Frame::UndistortKeyPoints / ComputeImageBounds (Frame.cc:404-464) on CPU.

cv::undistortPoints is OpenCV (absent here): its restatement (oracle ocv_semantics.c) is pinned
by (a) an independent float64 restatement of OpenCV 3.2 cvUndistortPoints' loop, bit for bit,
(b) the forward distortion model: distort(undistort(p)) returns p to within the 5-iteration
fixed point's residual on the reference's own camera settings, (c) the k1 == 0 copy rule."""
import numpy as np
import pytest

import oracle_lib
from undistort_cases import CAMERAS, K_of, distort, random_keys


def _py_undistort(x, y, K, d):
    """OpenCV 3.2 imgproc/undistort.cpp cvUndistortPoints, R = I, P = K, iters = 5, in Python
    floats (IEEE double, one rounding per operation)."""
    k = [0.0] * 8
    for i, v in enumerate(d):
        k[i] = float(np.float32(v))
    A = [[float(v) for v in row] for row in K.astype(np.float32)]
    fx, fy, cx, cy = A[0][0], A[1][1], A[0][2], A[1][2]
    ifx, ify = 1.0 / fx, 1.0 / fy
    x = float(x)
    y = float(y)
    x0 = x = (x - cx) * ifx
    y0 = y = (y - cy) * ify
    for _ in range(5):
        r2 = x * x + y * y
        icdist = (1 + ((k[7] * r2 + k[6]) * r2 + k[5]) * r2) / (1 + ((k[4] * r2 + k[1]) * r2 + k[0]) * r2)
        dX = 2 * k[2] * x * y + k[3] * (r2 + 2 * x * x)
        dY = k[2] * (r2 + 2 * y * y) + 2 * k[3] * x * y
        x = (x0 - dX) * icdist
        y = (y0 - dY) * icdist
    xx = A[0][0] * x + A[0][1] * y + A[0][2]
    yy = A[1][0] * x + A[1][1] * y + A[1][2]
    ww = 1.0 / (A[2][0] * x + A[2][1] * y + A[2][2])
    return np.float32(xx * ww), np.float32(yy * ww)


@pytest.mark.parametrize("name", sorted(CAMERAS))
def test_oracle_matches_python_restatement(name):
    cam, d, w, h = CAMERAS[name]
    K = K_of(cam)
    keys = random_keys(np.random.default_rng(1), 300, w, h)
    out = oracle_lib.oracle_undistort_keypoints(keys, K, np.float32(d))
    for i in range(len(keys)):
        ex, ey = _py_undistort(keys["x"][i], keys["y"][i], K, d)
        assert out["x"][i] == ex and out["y"][i] == ey, (i, out[i], ex, ey)
    # every other KeyPoint field is copied
    for f in ("size", "angle", "response", "octave", "class_id"):
        assert np.array_equal(out[f], keys[f])


@pytest.mark.parametrize("name", sorted(CAMERAS))
def test_undistort_inverts_forward_model(name):
    cam, d, w, h = CAMERAS[name]
    K = K_of(cam)
    keys = random_keys(np.random.default_rng(2), 500, w, h)
    # undistorted points of a central region, distorted forward, then undistorted again
    x = 0.25 * w + 0.5 * w * np.random.default_rng(3).random(500)
    y = 0.25 * h + 0.5 * h * np.random.default_rng(4).random(500)
    xd, yd = distort(x, y, K, d)
    keys["x"], keys["y"] = xd.astype(np.float32), yd.astype(np.float32)
    out = oracle_lib.oracle_undistort_keypoints(keys, K, np.float32(d))
    err = np.hypot(out["x"] - x, out["y"] - y)
    assert err.max() < 0.05, err.max()   # 5 fixed-point iterations on mild lens distortion


def test_k1_zero_copies_keys():
    cam, d, w, h = CAMERAS["tum1"]
    keys = random_keys(np.random.default_rng(5), 64, w, h)
    d0 = np.float32([0.0, -0.9, 0.01, 0.02, 1.1])   # Frame.cc:406 looks at k1 only
    out = oracle_lib.oracle_undistort_keypoints(keys, K_of(cam), d0)
    assert np.array_equal(out.view(np.uint8), keys.view(np.uint8))


def test_image_bounds():
    cam, d, w, h = CAMERAS["tum1"]
    K = K_of(cam)
    b = oracle_lib.oracle_compute_image_bounds(w, h, K, np.zeros(5, np.float32))
    assert b[:4] == (0.0, 640.0, 0.0, 480.0)
    assert b[4] == np.float32(np.float32(64) / np.float32(640)) and b[5] == np.float32(np.float32(48) / np.float32(480))
    b = oracle_lib.oracle_compute_image_bounds(w, h, K, np.float32(d))
    c = oracle_lib.oracle_undistort_points(np.float32([[0, 0], [w, 0], [0, h], [w, h]]), K, np.float32(d))
    assert b[0] == min(c[0, 0], c[2, 0]) and b[1] == max(c[1, 0], c[3, 0])
    assert b[2] == min(c[0, 1], c[1, 1]) and b[3] == max(c[2, 1], c[3, 1])
    assert b[4] == np.float32(np.float32(64) / np.float32(b[1] - b[0]))
    # TUM1's k1 > 0: the undistorted corners move inwards (the bounds shrink); EuRoC's k1 < 0
    # (barrel): outwards (the bounds grow)
    assert 0 < b[0] and b[1] < w and 0 < b[2] and b[3] < h
    cam, d, w, h = CAMERAS["euroc"]
    b = oracle_lib.oracle_compute_image_bounds(w, h, K_of(cam), np.float32(d))
    assert b[0] < 0 and b[1] > w and b[2] < 0 and b[3] > h
