"""Camera cases for Frame::UndistortKeyPoints / ComputeImageBounds (Frame.cc:404-464).

Intrinsics and distortion coefficients as the reference's example settings give them
(Examples/Monocular/TUM1.yaml:8-17, TUM2.yaml:8-17, EuRoC.yaml:8-16; image sizes from the
datasets: TUM 640x480, EuRoC 752x480).  Tracking's constructor makes mDistCoef 4x1 and appends
k3 only when it is non-zero (Tracking.cc:66-77), so TUM gets 5 coefficients and EuRoC 4."""
import numpy as np

import oracle_lib

CAMERAS = {
    "tum1": ((517.306408, 516.469215, 318.643040, 255.313989), (0.262383, -0.953104, -0.005358, 0.002628, 1.163314),
             640, 480),
    "tum2": ((520.908620, 521.007327, 325.141442, 249.701764), (0.231222, -0.784899, -0.003257, -0.000105, 0.917205),
             640, 480),
    "euroc": ((458.654, 457.296, 367.215, 248.375), (-0.28340811, 0.07395907, 0.00019359, 1.76187114e-05), 752, 480),
}


def K_of(cam):
    fx, fy, cx, cy = cam
    return np.array([[fx, 0, cx], [0, fy, cy], [0, 0, 1]], np.float32)


def random_keys(rng, n, w, h):
    k = np.zeros(n, oracle_lib.KP_DTYPE)
    k["x"] = rng.uniform(0, w, n).astype(np.float32)
    k["y"] = rng.uniform(0, h, n).astype(np.float32)
    k["size"] = np.float32(31)
    k["angle"] = rng.uniform(0, 360, n).astype(np.float32)
    k["response"] = rng.uniform(0, 100, n).astype(np.float32)
    k["octave"] = rng.integers(0, 8, n)
    k["class_id"] = -1
    return k


def distort(x, y, K, d):
    """The forward Brown-Conrady model cv::projectPoints applies (k1 k2 p1 p2 [k3]), float64."""
    fx, fy, cx, cy = float(K[0, 0]), float(K[1, 1]), float(K[0, 2]), float(K[1, 2])
    k = np.zeros(5)
    k[:len(d)] = np.asarray(d, np.float64)
    xn, yn = (x - cx) / fx, (y - cy) / fy
    r2 = xn * xn + yn * yn
    rad = 1 + k[0] * r2 + k[1] * r2 * r2 + k[4] * r2 ** 3
    xd = xn * rad + 2 * k[2] * xn * yn + k[3] * (r2 + 2 * xn * xn)
    yd = yn * rad + k[2] * (r2 + 2 * yn * yn) + 2 * k[3] * xn * yn
    return xd * fx + cx, yd * fy + cy
