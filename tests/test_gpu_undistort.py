"""Frame::UndistortKeyPoints / ComputeImageBounds on the GPU vs the oracle (Frame.cc:404-464).

Bit-exact KeyPoint bytes (the undistorted pt and every copied field) on the reference's own
camera settings (TUM1, TUM2, EuRoC), through the host form, the device batch form and a
config-1 pipeline (TUM-sized extraction on the GPU, then the device undistortion of its
keypoints).  cv::undistortPoints itself is "parity unpinned" (OpenCV absent); its restatement
is pinned on CPU by tests/test_undistort_cpu.py."""
import numpy as np
import pytest

import oracle_lib
from c_orb_slam_amd import synthetic
from undistort_cases import CAMERAS, K_of, random_keys

pytestmark = pytest.mark.gpu


def _same(a, b):
    return len(a) == len(b) and np.array_equal(a.view(np.uint8), b.view(np.uint8))


@pytest.mark.parametrize("name", sorted(CAMERAS))
@pytest.mark.parametrize("n", [0, 1, 1000, 4096])
def test_undistort_keypoints_host(gpu, name, n):
    cam, d, w, h = CAMERAS[name]
    K, dist = K_of(cam), np.float32(d)
    keys = random_keys(np.random.default_rng(n + 17), n, w, h)
    m = gpu.ORBmatcher(0.9, True)
    got = m.UndistortKeyPoints(keys, K, dist)
    exp = oracle_lib.oracle_undistort_keypoints(keys, K, dist)
    assert _same(got, exp)


def test_undistort_k1_zero_is_copy(gpu):
    cam, _, w, h = CAMERAS["tum1"]
    keys = random_keys(np.random.default_rng(3), 500, w, h)
    m = gpu.ORBmatcher(0.9, True)
    got = m.UndistortKeyPoints(keys, K_of(cam), np.float32([0.0, -0.9, 0.01, 0.02, 1.1]))
    assert _same(got, keys)


def test_undistort_device_batch(gpu):
    import torch
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(11)
    frames, expect = [], []
    for f, name in enumerate(["tum1", "euroc", "tum2", "tum1", "euroc"] * 6):   # 30 frames: 2 launches
        cam, d, w, h = CAMERAS[name]
        n = [0, 7, 1200, 333, 2048][f % 5]
        keys = random_keys(rng, n, w, h)
        dist = np.float32(d) if f % 7 else np.zeros(len(d), np.float32)   # some frames undistorted
        kd = torch.from_numpy(keys.view(np.int32).reshape(n, 7)).to(dev)
        frames.append(dict(keys=kd, keysUn=torch.full((n, 7), -1, dtype=torch.int32, device=dev), K=K_of(cam),
                           dist=dist))
        expect.append(oracle_lib.oracle_undistort_keypoints(keys, K_of(cam), dist))
    m = gpu.ORBmatcher(0.9, True)
    m.UndistortKeyPoints_device(frames)
    torch.cuda.synchronize()
    for f, e in zip(frames, expect):
        got = f["keysUn"].cpu().numpy().reshape(-1).view(oracle_lib.KP_DTYPE)
        assert _same(got, e)


@pytest.mark.parametrize("name", sorted(CAMERAS))
def test_compute_image_bounds(gpu, name):
    cam, d, w, h = CAMERAS[name]
    m = gpu.ORBmatcher(0.9, True)
    for dist in (np.float32(d), np.zeros(len(d), np.float32)):
        got = m.ComputeImageBounds(w, h, K_of(cam), dist)
        exp = oracle_lib.oracle_compute_image_bounds(w, h, K_of(cam), dist)
        assert np.array_equal(np.float32(got), np.float32(exp)), (got, exp)


def test_config1_extract_then_undistort(gpu):
    """SURVEY config 1 (TUM fr1, monocular 640x480, nFeatures 1000): Frame(imGray) = ExtractORB +
    UndistortKeyPoints (Frame.cc:135-143) with the extraction's keypoints left on the device."""
    import torch
    cam, d, w, h = CAMERAS["tum1"]
    frames, _ = synthetic.sequence(3, 4, w, h)
    B, cap = len(frames), 2 * 1000 + 64
    ex = gpu.ORBextractor(1000, 1.2, 8, 20, 7, max_width=w, max_height=h, max_batch=B)
    dev = torch.device("cuda", 0)
    d_img = torch.from_numpy(np.ascontiguousarray(np.stack(frames))).to(dev)
    d_k = torch.zeros((B, cap, 7), dtype=torch.int32, device=dev)
    d_d = torch.zeros((B, cap, 32), dtype=torch.uint8, device=dev)
    n = ex.extract_device(d_img.data_ptr(), B, w, h, w, w * h, d_k.data_ptr(), d_d.data_ptr(), cap)
    d_u = torch.zeros_like(d_k)
    fr = [dict(keys=d_k[b, :n[b]], keysUn=d_u[b, :n[b]], K=K_of(cam), dist=np.float32(d)) for b in range(B)]
    m = gpu.ORBmatcher(0.9, True)
    m.UndistortKeyPoints_device(fr)
    torch.cuda.synchronize()
    orc = oracle_lib.OracleExtractor(1000, 1.2, 8, 20, 7)
    for b in range(B):
        keys = d_k[b, :n[b]].cpu().numpy().reshape(-1).view(oracle_lib.KP_DTYPE)
        ok, _ = orc(frames[b])
        assert _same(keys, ok)   # the extraction itself (test_gpu_extract.py holds it bit-exact)
        got = d_u[b, :n[b]].cpu().numpy().reshape(-1).view(oracle_lib.KP_DTYPE)
        assert _same(got, oracle_lib.oracle_undistort_keypoints(ok, K_of(cam), np.float32(d)))
        assert n[b] > 500
