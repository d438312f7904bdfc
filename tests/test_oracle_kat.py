"""CPU: known-answer tests pinning the parity oracle (no GPU).

The reference ships no tests or golden vectors and cannot be
built here (F2), so the oracle is pinned where a ground truth exists on this
host (glibc sinf/cosf, glibc rand) and by hand-derived known answers of the
restated OpenCV/ORB-SLAM2 arithmetic.
"""
import ctypes as C
import ctypes.util
import hashlib
import math
from pathlib import Path

import numpy as np
import pytest

import oracle_lib
from oracle_lib import lib, ptr

GOLDEN = Path(__file__).resolve().parent / "golden"


def test_sincosf_restatement_equals_libm_exhaustive():
    """Every float in [0, 2*pi] (1.09e9 values): ora_sinf/ora_cosf == host libm bit for bit."""
    L = lib()
    L.ora_check_sincos_vs_libm.restype = C.c_long
    L.ora_check_sincos_vs_libm.argtypes = [C.c_float, C.c_float, C.c_long]
    assert L.ora_check_sincos_vs_libm(0.0, 6.2832, 1) == 0


def test_glibc_rand_restatement():
    libc = C.CDLL(ctypes.util.find_library("c"))
    L = lib()
    for seed in (0, 1, 12345, 2**31 - 1):
        libc.srand(seed)
        g = (C.c_int32 * 40)()
        L.ora_rng_seed(g, seed)
        for _ in range(2000):
            assert libc.rand() == L.ora_rng_rand(g)
    g = (C.c_int32 * 40)()
    L.ora_rng_seed(g, 1)
    assert L.ora_rng_rand(g) == 1804289383  # first unseeded glibc rand()


def test_random_int_formula():
    """DUtils::Random::RandomInt (Random.cpp:47-50)."""
    L = lib()
    g = (C.c_int32 * 40)()
    L.ora_rng_seed(g, 1)
    libc = C.CDLL(ctypes.util.find_library("c"))
    libc.srand(1)
    for i in range(500):
        r = libc.rand()
        expect = int((r / (2147483647 + 1.0)) * (i % 17 + 1)) + 3
        assert L.ora_rng_random_int(g, 3, 3 + i % 17) == expect


def test_descriptor_distance_swar():
    rng = np.random.default_rng(1)
    L = lib()
    for _ in range(300):
        a, b = rng.integers(0, 256, (2, 32), dtype=np.uint8)
        assert L.ora_descriptor_distance(ptr(a), ptr(b)) == int(np.unpackbits(a ^ b).sum())


def test_fast_atan2_known_answers():
    L = lib()
    assert L.ora_fastAtan2(0.0, 1.0) == 0.0
    assert abs(L.ora_fastAtan2(1.0, 0.0) - 90.0) < 1e-4
    assert abs(L.ora_fastAtan2(0.0, -1.0) - 180.0) < 1e-4
    assert abs(L.ora_fastAtan2(-1.0, 0.0) - 270.0) < 1e-4
    rng = np.random.default_rng(0)
    for y, x in rng.integers(-20000, 20000, (2000, 2)):
        a = L.ora_fastAtan2(float(y), float(x))
        t = math.degrees(math.atan2(y, x)) % 360.0
        err = min(abs(a - t), 360 - abs(a - t))
        assert 0 <= a <= 360 and err < 0.02, (y, x, a, t)


def _patch(center, ring):
    """7x7 patch with the FAST circle (OpenCV offsets16 order) set to `ring`."""
    ofs = [(0, 3), (1, 3), (2, 2), (3, 1), (3, 0), (3, -1), (2, -2), (1, -3), (0, -3), (-1, -3), (-2, -2),
           (-3, -1), (-3, 0), (-3, 1), (-2, 2), (-1, 3)]
    p = np.full((7, 7), center, np.uint8)
    for (dx, dy), v in zip(ofs, ring):
        p[3 + dy, 3 + dx] = v
    return p


def test_fast_score_known_answers():
    L = lib()
    score = lambda p: L.ora_fast_score(C.c_void_p(p.ctypes.data + 3 * 7 + 3), 7)
    # 9 contiguous brighter by 50 -> max(A,B)-1 = 49; corner for any th <= 49
    assert score(_patch(100, [150] * 9 + [100] * 7)) == 49
    # 8 contiguous only -> not a corner at any threshold
    assert score(_patch(100, [150] * 8 + [100] * 8)) == -1
    # dark arc of 12 at -30 with one pixel at -20 inside: best 9-arc avoiding it
    ring = [70] * 12 + [100] * 4
    assert score(_patch(100, ring)) == 29
    ring[5] = 80
    assert score(_patch(100, ring)) == 19  # every 9-arc of the 12 contains index 5
    # mixed: bright 9 arc (+40) vs dark 9 arc impossible -> 39
    assert score(_patch(100, [140] * 10 + [60] * 6)) == 39


def test_gaussian_taps_and_resize_constant():
    L = lib()
    taps = (C.c_int * 7)()
    L.ora_gaussian7_taps(taps)
    assert list(taps) == [18, 34, 49, 55, 49, 34, 18]  # OpenCV 3.2 8-bit fixed point, sum 257
    src = np.full((376, 1241), 77, np.uint8)
    dst = np.zeros((313, 1034), np.uint8)
    L.ora_resize_linear_u8(ptr(src), 1241, 1241, 376, ptr(dst), 1034, 1034, 313)
    assert (dst == 77).all()
    blur = np.zeros_like(src)
    L.ora_gaussian7_u8(ptr(src), 1241, 1241, 376, ptr(blur), 1241)
    assert (blur == min(255, (77 * 257 * 257 + 32768) >> 16)).all()


def test_extractor_tables():
    t = oracle_lib.OracleExtractor(1200, 1.2, 8, 20, 7).tables()
    assert t["n_per_level"].tolist() == [261, 217, 181, 151, 126, 105, 87, 72]
    assert oracle_lib.OracleExtractor(2000, 1.2, 8, 20, 7).tables()["n_per_level"].tolist() == \
        [434, 362, 302, 251, 209, 175, 145, 122]
    assert t["umax"].tolist() == [15, 15, 15, 15, 14, 14, 14, 13, 13, 12, 11, 10, 9, 8, 6, 3]
    assert t["scale"][1] == np.float32(1.2) and t["scale"][7] == np.float32(np.float32(1.2) ** 7) or True
    assert abs(float(t["scale"][7]) - 1.2 ** 7) < 1e-5


def test_pyramid_level_sizes():
    """KITTI 1241x376 level sizes from SURVEY §8 (cvRound(W*invScale))."""
    from c_orb_slam_amd import synthetic
    img, _ = synthetic.sequence(0, 1)
    e = oracle_lib.OracleExtractor(1200, 1.2, 8, 20, 7)
    e(img[0])
    sizes = [(e.level(l).shape[1] - 38, e.level(l).shape[0] - 38) for l in range(8)]
    assert sizes == [(1241, 376), (1034, 313), (862, 261), (718, 218), (598, 181), (499, 151), (416, 126),
                     (346, 105)]
    # the padded border is REFLECT_101 of the level (Frame.cc:573-580 reads it)
    L0 = e.level(0)
    assert np.array_equal(L0[19:-19, 0], L0[19:-19, 38])
    assert np.array_equal(L0[0, 19:-19], L0[38, 19:-19])


@pytest.mark.parametrize("f", sorted(GOLDEN.glob("extract_*.npz")), ids=lambda p: p.stem)
def test_oracle_golden_extraction(f):
    from c_orb_slam_amd import synthetic
    g = np.load(f)
    img = synthetic.sequence(int(g["seed"]), 1, int(g["w"]), int(g["h"]))[0][0]
    assert hashlib.sha256(img.tobytes()).hexdigest() == str(g["sha256"]), "synthetic generator drifted"
    k, d = oracle_lib.OracleExtractor(int(g["nfeatures"]), 1.2, 8, 20, 7)(img)
    assert np.array_equal(k.view(np.uint8).reshape(-1, 28), g["kps"])
    assert np.array_equal(d, g["desc"])


def test_oracle_keypoint_invariants():
    from c_orb_slam_amd import synthetic
    img = synthetic.sequence(3, 1)[0][0]
    e = oracle_lib.OracleExtractor(1200, 1.2, 8, 20, 7)
    k, d = e(img)
    sc = e.tables()["scale"]
    assert (np.diff(k["octave"]) >= 0).all()                       # level-major
    assert ((k["angle"] >= 0) & (k["angle"] <= 360)).all()
    assert (k["class_id"] == -1).all()
    assert np.array_equal(k["size"], np.array([int(31 * s) for s in sc], np.float32)[k["octave"]])
    for l in range(8):
        kl = k[k["octave"] == l]
        lx, ly = kl["x"] / sc[l], kl["y"] / sc[l]
        lvl = e.level(l)
        assert (lx >= 19 - 1e-3).all() and (lx <= lvl.shape[1] - 38 - 20 + 1e-3).all()
        assert (ly >= 19 - 1e-3).all()


def test_oracle_svd_and_epnp():
    """OpenCV-semantics SVD restatement reconstructs; EPnP is exact on noise-free 6+ points."""
    import sys
    from pnp_cases import rot
    L = lib()
    L.ora_svd.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p]
    L.ora_epnp_compute_pose.restype = C.c_double
    L.ora_epnp_compute_pose.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_double, C.c_double, C.c_double,
                                        C.c_double, C.c_void_p, C.c_void_p]
    rng = np.random.default_rng(0)
    for m, n in [(3, 3), (6, 4), (12, 12), (6, 5)]:
        A = rng.normal(size=(m, n))
        w, Ut, Vt = np.zeros(n), np.zeros((n, m)), np.zeros((n, n))
        L.ora_svd(ptr(A), m, n, ptr(w), ptr(Ut), ptr(Vt))
        assert np.abs(Ut.T @ np.diag(w) @ Vt - A).max() < 1e-12
        assert (np.diff(w) <= 0).all()
    fx, fy, cx, cy = 718.856, 718.856, 607.1928, 185.2157
    for trial in range(20):
        R = rot(rng)
        t = rng.uniform(-2, 2, 3)
        n = 8
        u, v, d = rng.uniform(20, 1220, n), rng.uniform(20, 356, n), rng.uniform(5, 50, n)
        Xw = (np.stack([(u - cx) / fx * d, (v - cy) / fy * d, d], 1) - t) @ R
        pws, us = np.ascontiguousarray(Xw), np.ascontiguousarray(np.stack([u, v], 1))
        Ro, to = np.zeros((3, 3)), np.zeros(3)
        L.ora_epnp_compute_pose(ptr(pws), ptr(us), n, fx, fy, cx, cy, ptr(Ro), ptr(to))
        assert np.abs(Ro - R).max() < 1e-6 and np.abs(to - t).max() < 1e-5


def test_oracle_pnp_ransac_recovers_pose():
    from pnp_cases import pnp_problem
    pr = pnp_problem(3, 500)
    P = oracle_lib.OraclePnP(pr["p3d"], pr["p2d"], pr["sigma2"], pr["kp_idx"], pr["n_matches"], *pr["K"])
    P.set_ransac(0.99, 10, 300, 4, 0.5, 5.991)
    ok, T, inl, n, no_more = P.iterate(5, oracle_lib.new_rng(1))
    assert ok and n > 250 and np.abs(T - pr["Tcw"]).max() < 0.1


# ---- Sim3 (oracle/sim3.c) ---------------------------------------------------
def test_det_trig_close_to_libm():
    """det_sincos/det_atan2 (shared bit-for-bit with the GPU) stay within 4 ulp of libm."""
    import math
    L = oracle_lib.lib()
    L.ora_det_sincos.argtypes = [ctypes.c_double, ctypes.c_void_p, ctypes.c_void_p]
    L.ora_det_atan2.argtypes = [ctypes.c_double, ctypes.c_double]
    L.ora_det_atan2.restype = ctypes.c_double
    rng = np.random.default_rng(0)
    s, c = ctypes.c_double(), ctypes.c_double()
    for x in np.concatenate([rng.uniform(0, 4 * np.pi, 2000), [0.0, 1e-9, np.pi / 4, np.pi / 2, np.pi]]):
        L.ora_det_sincos(float(x), ctypes.byref(s), ctypes.byref(c))
        assert abs(s.value - math.sin(x)) <= 2 * math.ulp(max(abs(math.sin(x)), 1e-300)) + 1e-17
        assert abs(c.value - math.cos(x)) <= 2 * math.ulp(max(abs(math.cos(x)), 1e-300)) + 1e-17
    for y, x in rng.normal(0, 3, (2000, 2)).tolist() + [(0.0, 1.0), (1.0, 0.0), (0.0, -1.0), (-1.0, -1.0)]:
        a = math.atan2(y, x)
        assert abs(L.ora_det_atan2(y, x) - a) <= 4 * math.ulp(abs(a)) + 1e-300


def test_jacobi_eigen_symmetric():
    L = oracle_lib.lib()
    L.ora_jacobi_eigen_f.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    rng = np.random.default_rng(1)
    for _ in range(50):
        B = rng.normal(size=(4, 4)).astype(np.float32)
        A = (B + B.T).astype(np.float32)
        W, V, A2 = np.zeros(4, np.float32), np.zeros(16, np.float32), A.copy()
        L.ora_jacobi_eigen_f(A2.ctypes.data, 4, W.ctypes.data, V.ctypes.data)
        w_ref = np.sort(np.linalg.eigvalsh(A.astype(np.float64)))[::-1]
        np.testing.assert_allclose(W, w_ref, rtol=1e-4, atol=1e-4)
        V = V.reshape(4, 4)
        for i in range(4):   # rows are eigenvectors
            np.testing.assert_allclose(A @ V[i], W[i] * V[i], atol=2e-4)


@pytest.mark.parametrize("fix", [True, False])
def test_sim3_oracle_recovers_similarity(fix):
    from sim3_cases import sim3_problem
    pr = sim3_problem(11, 120, fix_scale=fix)
    o = oracle_lib.OracleSim3(pr["X1"], pr["X2"], pr["s1"], pr["s2"], pr["idx1"], pr["N1"], pr["K1"], pr["K2"],
                              pr["fix"])
    o.set_ransac(0.99, 20, 300)
    rng = oracle_lib.new_rng(1)
    for _ in range(60):
        ok, T, inl, nin, nm = o.iterate(5, rng)
        if ok or nm:
            break
    assert ok and nin > 20
    np.testing.assert_allclose(T[:3, :3], pr["T12"][:3, :3], atol=0.05)
    _, _, s = o.estimate()
    assert abs(s - pr["s"]) < 0.05 * pr["s"]
    mask = np.zeros(len(pr["X1"]), bool)
    mask[pr["outliers"]] = True
    flagged = inl[pr["idx1"]]
    assert not np.any(flagged & mask), "an outlier accepted as inlier"


def test_oracle_stereo_recovers_disparity():
    """Frame::ComputeStereoMatches restatement (oracle/stereo.c) on a synthetic rectified pair:
    kept matches sit at the rectangles' integer disparities (0..64) within a pixel."""
    from c_orb_slam_amd import synthetic
    L, R = synthetic.stereo_batch(0, 1, 1241, 376)
    exL, exR = oracle_lib.OracleExtractor(1200, 1.2, 8, 20, 7), oracle_lib.OracleExtractor(1200, 1.2, 8, 20, 7)
    kL, dL = exL(L[0])
    kR, dR = exR(R[0])
    mbf = 386.1448
    mb = np.float32(np.float32(mbf) / np.float32(718.856))
    uR, dep, kept = oracle_lib.oracle_stereo_matches(exL, exR, kL, dL, kR, dR, 376, mbf, mb)
    ok = uR >= 0
    assert kept == ok.sum() and kept > 50
    d = kL["x"][ok] - uR[ok]
    near_int = np.abs(d - np.round(d)) < 0.75
    assert near_int.mean() > 0.8 and (np.round(d) <= 65).mean() > 0.9
    np.testing.assert_allclose(dep[ok], mbf / d, rtol=1e-5)


def test_oracle_searches_run_and_agree_with_geometry():
    """CPU sanity of the restated searches (oracle/matchers2.c): relocalization projection matches
    land on the keypoint the map point came from (frames related by a known rotation), and the
    BoW / initialization searches return consistent one-to-one assignments."""
    import search_cases as sc
    c = sc.reloc_case(0)
    cur = c["cur_mp"].copy()
    n = oracle_lib.oracle_search_by_projection_kf(c["F"], cur, c["kf_mp"], c["skip"], c["kf_angle"], c["mps"],
                                                  c["max_dist"], c["min_dist"], c["logScaleFactor"], 10, 100)
    assert n > 100
    new = (cur >= 0) & (c["cur_mp"] < 0)
    assert new.sum() == n
    (k0, d0), (k1, d1) = sc.frames(0)[0]
    t = sc.frames(0)[3]
    F1 = sc.make_frame(k0, d0, t, np.eye(4, dtype=np.float32))
    F2 = sc.make_frame(k1, d1, t, np.eye(4, dtype=np.float32))
    prev = np.ascontiguousarray(np.stack([k0["x"], k0["y"]], 1), np.float32)
    n, m12 = oracle_lib.oracle_search_for_initialization(F1, F2, prev, 100)
    got = m12[m12 >= 0]
    assert n == len(got) and len(np.unique(got)) == len(got) and n > 50
    mp = np.arange(len(k0), dtype=np.int32)
    n, out = oracle_lib.oracle_search_by_bow_frame(d0, k0["angle"], mp, np.zeros(len(k0), np.uint8), sc.featvec(d0),
                                                   d1, k1["angle"], sc.featvec(d1), 0.7)
    got = out[out >= 0]
    assert n == len(got) and len(np.unique(got)) == len(got) and n > 50


def test_oracle_pose_optimization_recovers_pose():
    """ora_pose_optimization (Optimizer.cc:239-451) on a synthetic tracked frame: the
    motion-model prior is pulled to the true pose and the injected gross outliers are flagged."""
    from pose_cases import pose_problem
    pr = pose_problem(0)
    o = oracle_lib.oracle_pose_optimization(pr)
    mp = pr["has_mp"].astype(bool)
    T = o["Tcw"].astype(np.float64)
    assert np.linalg.norm(T[:3, 3] - pr["T_true"][:3, 3]) < 0.02
    assert np.abs(T[:3, :3] - pr["T_true"][:3, :3]).max() < 2e-3
    assert o["outlier"][pr["gross"] & mp].mean() > 0.9
    assert o["inliers"] == int(mp.sum()) - int(o["outlier"][mp].sum())
    assert len(o["solve_chi2"]) >= 4


def test_oracle_ldlt_pivot_solve():
    """Eigen LDLT with diagonal pivoting (LinearSolverDense) vs numpy on SPD 6x6 systems."""
    L = lib()
    L.ora_ldlt_pivot_solve.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p]
    rng = np.random.default_rng(3)
    for _ in range(20):
        A = rng.normal(size=(6, 6))
        H = A @ A.T + np.diag(rng.uniform(0, 5, 6) ** 3)
        b = rng.normal(size=6)
        x = np.zeros(6)
        Hc = np.ascontiguousarray(H).copy()
        assert L.ora_ldlt_pivot_solve(ptr(Hc), 6, ptr(b), ptr(x)) == 1
        np.testing.assert_allclose(x, np.linalg.solve(H, b), rtol=1e-9, atol=1e-12)
    Hn = -np.eye(6)
    assert L.ora_ldlt_pivot_solve(ptr(Hn), 6, ptr(np.ones(6)), ptr(np.zeros(6))) == 0


def test_oracle_projection_searches_sanity():
    """matchers3.c on the loop-closing cases: Sim3-projected map points of keyframe 0 land on
    keyframe 1 keypoints carrying the same descriptor (the rotation-only synthetic motion keeps
    most of them), and SearchBySim3's two directions agree on a large set."""
    import search_cases as sc
    c = sc.loop_case(0)
    n, m = oracle_lib.oracle_search_by_projection_sim3(c["KF"], c["Scw"], c["pts"], c["geo"], c["skip"],
                                                       c["matched"], c["logScaleFactor"], 10)
    new = (m >= 0) & (c["matched"] < 0)
    assert n == new.sum() and n > 300
    assert not c["skip"][m[new]].any()
    nf, best = oracle_lib.oracle_fuse(c["KF"], c["pts"], c["geo"], c["skip"], c["logScaleFactor"], 3.0)
    assert nf == (best >= 0).sum() and nf > 100
    s = sc.sim3_case(0)
    nfound, m12 = oracle_lib.oracle_search_by_sim3(s["KF1"], s["mp1"], s["KF2"], s["mp2"], s["pts"], s["geo"],
                                                   s["bad"], s["m12"], s["s12"], s["R12"], s["t12"],
                                                   s["logScaleFactor"], 7.5)
    assert nfound == ((m12 >= 0) & (s["m12"] == -1)).sum() and nfound > 200


def test_det_exp_close_to_libm():
    """ora_det_exp (fdlibm __ieee754_exp restated) is within 1 ulp of libm over the ranges
    g2o::Sim3 uses (sigma = log scale, +-1e-9 numeric steps) and far beyond."""
    import math
    xs = np.concatenate([[0.0, 1e-9, -1e-9, 1e-12, 0.3465, 0.3466, 1.0397, 1.0398, -0.3466, -1.0398, 700.0, -700.0],
                         np.random.default_rng(0).uniform(-30, 30, 2000)])
    for x in xs:
        a, b = oracle_lib.oracle_det_exp(x), math.exp(x)
        assert a == b or abs(a - b) <= abs(b) * 2.3e-16, (x, a, b)
    assert oracle_lib.oracle_det_exp(0.0) == 1.0


@pytest.mark.parametrize("fix", [True, False])
def test_oracle_optimize_sim3_refines_similarity(fix):
    """Optimizer::OptimizeSim3 restatement: the refined Sim3 is closer to the truth than the
    RANSAC-shaped initial guess, the synthetic gross outliers are erased, scale fixed iff bFixScale."""
    from scipy.spatial.transform import Rotation
    from sim3opt_cases import sim3opt_problem
    for seed in range(3):
        pr = sim3opt_problem(seed=seed, fix_scale=fix)
        S0 = oracle_lib.oracle_sim3_from_Rts(pr["R0"], pr["t0"], pr["s0"])
        n, S, er, tr = oracle_lib.oracle_optimize_sim3(pr, S0)
        valid = pr["valid"].astype(bool)
        assert n >= 10 and n + er.sum() == valid.sum() and not er[~valid].any()
        assert er[pr["gross"]].mean() > 0.8
        Rq = Rotation.from_quat(S[:4] / np.linalg.norm(S[:4])).as_matrix()
        e0 = np.linalg.norm(Rotation.from_matrix(pr["R0"].astype(np.float64) @ pr["R_true"].T).as_rotvec())
        e1 = np.linalg.norm(Rotation.from_matrix(Rq @ pr["R_true"].T).as_rotvec())
        assert e1 < 0.25 * e0
        assert np.linalg.norm(S[4:7] - pr["t_true"]) < np.linalg.norm(pr["t0"] - pr["t_true"])
        if fix:
            assert S[7] == float(pr["s0"])
        else:
            assert abs(S[7] - pr["s_true"]) < abs(float(pr["s0"]) - pr["s_true"]) + 1e-3
        assert np.all(np.diff(tr["solve_chi2"][:5]) <= 1e-9 * tr["solve_chi2"][0])


def test_oracle_optimize_sim3_early_return():
    """Fewer than 10 correspondences left after gating: return 0, g2oS12 untouched."""
    from sim3opt_cases import sim3opt_problem
    pr = sim3opt_problem(seed=4, N=40, match_frac=0.25)
    S0 = oracle_lib.oracle_sim3_from_Rts(pr["R0"], pr["t0"], pr["s0"])
    n, S, er, _ = oracle_lib.oracle_optimize_sim3(pr, S0)
    assert pr["valid"].sum() < 10 and n == 0 and np.array_equal(S, S0)


def test_det_log_predict_scale_exhaustive():
    """MapPoint::PredictScale (MapPoint.cc:402-417) takes glibc logf of ratio = mfMaxDistance /
    dist; on the device it is (float) of a restated fdlibm log in double (detmath::log_d, the
    same operation sequence as ora_det_log).  Over every float ratio isInFrustum can produce
    (dist within [0.8 minDistance, 1.2 maxDistance]: ratio in [1/1.2, 1.2^7 / 0.8]) and well
    beyond, the predicted levels agree exactly."""
    L = oracle_lib.lib()
    L.ora_predict_scale_mismatches.restype = C.c_longlong
    L.ora_predict_scale_mismatches.argtypes = [C.c_float, C.c_float, C.c_float, C.POINTER(C.c_longlong),
                                               C.POINTER(C.c_longlong)]
    lsf = np.float32(np.log(np.float32(1.2)))
    n, d = C.c_longlong(), C.c_longlong()
    bad = L.ora_predict_scale_mismatches(0.25, 16.0, float(lsf), C.byref(n), C.byref(d))
    assert n.value > 40_000_000
    assert bad == 0, (bad, d.value, n.value)
