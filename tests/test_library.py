"""CPU: the C-ABI library loads, exports every symbol include/orbslam_gpu.h declares,
validates arguments before touching the device, and reports ORB_E_NODEVICE
(never a silent CPU fallback) when no GPU is visible."""
import ctypes as C
import re
from pathlib import Path

import numpy as np
import pytest

import c_orb_slam_amd as orb
from c_orb_slam_amd._lib import (ORB_E_INVALID, ORB_E_NODEVICE, header_functions, lib, ptr)


def test_all_header_symbols_exported():
    L = lib()
    names = header_functions()
    assert len(names) >= 20
    for n in names:
        assert hasattr(L, n), n


def test_version_and_device_probe():
    assert b"gfx950" in lib().orbgpu_version()
    # the header's ABI revision (ORBmatcher_SearchLocalPoints_batch's signature changed: 2)
    hdr = (Path(__file__).resolve().parents[1] / "include" / "orbslam_gpu.h").read_text()
    rev = int(re.search(r"#define ORBGPU_ABI_VERSION (\d+)", hdr).group(1))
    assert lib().orbgpu_abi_version() == rev == 2
    assert orb.device_available() in (True, False)


def test_invalid_arguments_rejected_without_device():
    L = lib()
    h = C.c_void_p()
    assert L.ORBextractor_create(1200, 1.2, 0, 20, 7, 640, 480, 1, C.byref(h)) == ORB_E_INVALID
    assert L.ORBextractor_create(1200, 1.0, 8, 20, 7, 640, 480, 1, C.byref(h)) == ORB_E_INVALID
    assert L.ORBextractor_create(1200, 1.2, 8, 20, 7, 0, 480, 1, C.byref(h)) == ORB_E_INVALID
    assert L.ORBextractor_destroy(None) == ORB_E_INVALID
    assert L.ORBmatcher_destroy(None) == ORB_E_INVALID
    assert L.ORBmatcher_create(0.6, 1, None) == ORB_E_INVALID


def test_descriptor_distance_host_entry():
    a = np.arange(32, dtype=np.uint8)
    b = a[::-1].copy()
    assert orb.ORBmatcher.DescriptorDistance(a, b) == int(np.unpackbits(a ^ b).sum())


@pytest.mark.skipif(orb.device_available(), reason="a GPU is visible here")
def test_no_silent_cpu_fallback():
    with pytest.raises(orb.OrbGpuError) as ei:
        orb.ORBextractor(1200, 1.2, 8, 20, 7)
    assert ei.value.code == ORB_E_NODEVICE
    with pytest.raises(orb.OrbGpuError):
        orb.ORBmatcher(0.9, True)


def test_ransac_solvers_validate_and_refuse_without_device():
    L = lib()
    h = C.c_void_p()
    X = np.zeros((4, 3), np.float32)
    s = np.ones(4, np.float32)
    K = np.array([700, 700, 600, 180], np.float32)
    idx = np.arange(4, dtype=np.int32)
    # N < 3 and out-of-range idx1 are argument errors, checked before the device
    assert L.Sim3Solver_create(2, ptr(X), ptr(X), ptr(s), ptr(s), ptr(idx), 4, ptr(K), ptr(K), 1,
                               C.byref(h)) == ORB_E_INVALID
    bad = np.array([0, 1, 2, 9], np.int32)
    assert L.Sim3Solver_create(4, ptr(X), ptr(X), ptr(s), ptr(s), ptr(bad), 4, ptr(K), ptr(K), 1,
                               C.byref(h)) == ORB_E_INVALID
    assert L.Sim3Solver_destroy(None) == ORB_E_INVALID
    assert L.PnPsolver_destroy(None) == ORB_E_INVALID
    if not orb.device_available():
        assert L.Sim3Solver_create(4, ptr(X), ptr(X), ptr(s), ptr(s), ptr(idx), 4, ptr(K), ptr(K), 1,
                                   C.byref(h)) == ORB_E_NODEVICE


def test_ba_validates_without_device():
    from c_orb_slam_amd._lib import ba_problem, ba_result
    L = lib()
    kid = np.array([0, 1], np.int32)
    T = np.tile(np.eye(4, dtype=np.float32).ravel(), (2, 1))
    loc = np.array([1, 1], np.uint8)
    cam = np.tile(np.array([435, 435, 367, 252, 47.9], np.float32), (2, 1))
    pid = np.array([5], np.int32)
    X = np.array([[0, 0, 5]], np.float32)
    ept = np.array([0, 0], np.int32)
    ekf = np.array([1, 1], np.int32)          # duplicate (keyframe, point) edge
    obs = np.zeros((2, 3), np.float32)
    isg = np.ones(2, np.float32)
    P = ba_problem(2, ptr(kid), ptr(T), ptr(loc), ptr(cam), 1, ptr(pid), ptr(X), 2, ptr(ept), ptr(ekf), ptr(obs),
                   ptr(isg))
    To, Xo, er = np.zeros_like(T), np.zeros_like(X), np.zeros(2, np.uint8)
    R = ba_result(ptr(To), ptr(Xo), ptr(er))
    assert L.Optimizer_LocalBundleAdjustment(C.byref(P), None, C.byref(R)) == ORB_E_INVALID
    ekf[1] = 0
    kid[1] = 0                                 # duplicate keyframe id
    assert L.Optimizer_LocalBundleAdjustment(C.byref(P), None, C.byref(R)) == ORB_E_INVALID
    kid[1] = 1
    if not orb.device_available():
        assert L.Optimizer_LocalBundleAdjustment(C.byref(P), None, C.byref(R)) == ORB_E_NODEVICE


def test_optimize_sim3_validates_without_device():
    from c_orb_slam_amd._lib import sim3opt_problem
    L = lib()
    N = 4
    v = np.ones(N, np.uint8)
    X = np.ones((N, 3), np.float32)
    o = np.zeros((N, 2), np.float32)
    s = np.ones(N, np.float32)
    P = sim3opt_problem(N, ptr(v), ptr(X), ptr(X), ptr(o), ptr(o), ptr(s), ptr(s))
    P.th2 = 10.0
    S = np.array([0, 0, 0, 1, 0, 0, 0, 1], np.float64)
    er = np.zeros(N, np.uint8)
    n = C.c_int()
    assert L.Optimizer_OptimizeSim3(None, ptr(S), ptr(er), C.byref(n)) == ORB_E_INVALID
    P2 = sim3opt_problem(N, ptr(v), None, ptr(X), ptr(o), ptr(o), ptr(s), ptr(s))
    assert L.Optimizer_OptimizeSim3(C.byref(P2), ptr(S), ptr(er), C.byref(n)) == ORB_E_INVALID
    P.th2 = float("nan")
    assert L.Optimizer_OptimizeSim3(C.byref(P), ptr(S), ptr(er), C.byref(n)) == ORB_E_INVALID
    P.th2 = 10.0
    if not orb.device_available():
        assert L.Optimizer_OptimizeSim3(C.byref(P), ptr(S), ptr(er), C.byref(n)) == ORB_E_NODEVICE


def _abi_image():
    """tests/c_abi/abi_caller.c's seeded 640x480 image, restated (uint32 LCG, 8-bit blocks + noise)."""
    W, H = 640, 480
    img = np.zeros((H, W), np.uint8)
    s = 12345
    for y in range(H):
        for x in range(W):
            s = (s * 1664525 + 1013904223) & 0xFFFFFFFF
            img[y, x] = ((x // 40) * 37 + (y // 30) * 91) % 200 + ((s >> 24) & 31)
    return img


def test_c11_caller_compiles_links_and_runs(tmp_path):
    """A plain C11 translation unit includes include/orbslam_gpu.h with -std=c11 -pedantic -Werror,
    links against liborbslam_gpu.so and calls it: the host-only entry points answer, and without
    a device the create() calls report ORB_E_NODEVICE."""
    import shutil
    import subprocess
    from pathlib import Path
    root = Path(__file__).resolve().parents[1]
    cc = shutil.which("gcc") or shutil.which("cc")
    if cc is None:
        pytest.skip("no C compiler")
    exe = tmp_path / "abi_caller"
    r = subprocess.run([cc, "-std=c11", "-pedantic", "-Wall", "-Wextra", "-Werror", "-O1", f"-I{root / 'include'}",
                        str(root / "tests" / "c_abi" / "abi_caller.c"), f"-L{root / 'c_orb_slam_amd'}", "-lorbslam_gpu",
                        f"-Wl,-rpath,{root / 'c_orb_slam_amd'}", "-o", str(exe)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert "abi_caller ok" in r.stdout


@pytest.mark.gpu
def test_c11_caller_extracts_like_the_python_binding(tmp_path):
    """The prebuilt C11 caller (make abi -> build/abi_caller) runs ORBextractor_extract from host
    buffers to host buffers on the GPU; its keypoints and descriptors equal the ctypes binding's
    and the oracle's, byte for byte."""
    import subprocess
    from pathlib import Path
    import oracle_lib
    root = Path(__file__).resolve().parents[1]
    exe = root / "build" / "abi_caller"
    assert exe.exists(), "build/abi_caller missing: run `make abi` before the GPU tests"
    out = tmp_path / "kps.bin"
    r = subprocess.run([str(exe), str(out)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr + r.stdout
    raw = out.read_bytes()
    n = int(np.frombuffer(raw[:4], np.int32)[0])
    ck = np.frombuffer(raw[4:4 + 28 * n], dtype=np.uint8)
    cd = np.frombuffer(raw[4 + 28 * n:4 + 60 * n], dtype=np.uint8).reshape(n, 32)
    img = _abi_image()
    kps, desc = orb.ORBextractor(1000, 1.2, 8, 20, 7, max_width=640, max_height=480)(img)
    assert len(kps) == n
    assert np.array_equal(kps.view(np.uint8).reshape(-1), ck)
    assert np.array_equal(desc, cd)
    okps, odesc = oracle_lib.OracleExtractor(1000, 1.2, 8, 20, 7)(img)
    assert np.array_equal(okps.view(np.uint8).reshape(-1), ck) and np.array_equal(odesc, cd)
