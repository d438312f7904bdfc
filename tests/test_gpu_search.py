"""The remaining ORBmatcher searches on the GPU vs the CPU oracle (reference src/ORBmatcher.cc):
SearchByProjection(Frame, KeyFrame) 1472-1599, SearchForInitialization 405-520, SearchByBoW
(KF, F) 159-288 and (KF, KF) 522-655, SearchForTriangulation 657-823.  Integer outputs
(match indices, map point assignments, counts, pairs) must be identical."""
import numpy as np
import pytest

import oracle_lib
import search_cases as sc
from c_orb_slam_amd import synthetic

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("seed,th,orbdist,check", [(0, 10, 100, True), (1, 3, 64, True), (2, 10, 100, False)])
def test_search_by_projection_keyframe(gpu, seed, th, orbdist, check):
    c = sc.reloc_case(seed)
    m = gpu.ORBmatcher(0.9, check)
    cur = c["cur_mp"].copy()
    n = m.SearchByProjection_KeyFrame(c["F"], cur, c["kf_mp"], c["skip"], c["kf_angle"], c["mps"], c["max_dist"],
                                      c["min_dist"], c["logScaleFactor"], th, orbdist)
    ocur = c["cur_mp"].copy()
    on = oracle_lib.oracle_search_by_projection_kf(c["F"], ocur, c["kf_mp"], c["skip"], c["kf_angle"], c["mps"],
                                                   c["max_dist"], c["min_dist"], c["logScaleFactor"], th, orbdist,
                                                   check)
    assert n == on and np.array_equal(cur, ocur)
    assert n > 100, n


@pytest.mark.parametrize("seed,window,nnratio", [(0, 100, 0.9), (3, 50, 0.9), (4, 100, 0.6)])
def test_search_for_initialization(gpu, seed, window, nnratio):
    (k0, d0), (k1, d1) = sc.frames(seed)[0]
    t = sc.frames(seed)[3]
    F1 = sc.make_frame(k0, d0, t, np.eye(4, dtype=np.float32))
    F2 = sc.make_frame(k1, d1, t, np.eye(4, dtype=np.float32))
    prev = np.ascontiguousarray(np.stack([k0["x"], k0["y"]], 1), np.float32)
    m = gpu.ORBmatcher(nnratio, True)
    p1 = prev.copy()
    n, m12 = m.SearchForInitialization(F1, F2, p1, window)
    p2 = prev.copy()
    on, om12 = oracle_lib.oracle_search_for_initialization(F1, F2, p2, window, nnratio, True)
    assert n == on and np.array_equal(m12, om12) and np.array_equal(p1, p2)
    assert n > 50, n


@pytest.mark.parametrize("seed,nnratio,check", [(0, 0.7, True), (5, 0.75, True), (6, 0.9, False)])
def test_search_by_bow_frame(gpu, seed, nnratio, check):
    (k0, d0), (k1, d1) = sc.frames(seed)[0]
    rng = np.random.default_rng(seed)
    kf_mp = np.where(rng.random(len(k0)) < 0.8, rng.permutation(len(k0)), -1).astype(np.int32)
    bad = (rng.random(len(k0)) < 0.05).astype(np.uint8)
    m = gpu.ORBmatcher(nnratio, check)
    n, out = m.SearchByBoW_Frame(d0, k0["angle"], kf_mp, bad, sc.featvec(d0), d1, k1["angle"], sc.featvec(d1))
    on, oout = oracle_lib.oracle_search_by_bow_frame(d0, k0["angle"], kf_mp, bad, sc.featvec(d0), d1, k1["angle"],
                                                     sc.featvec(d1), nnratio, check)
    assert n == on and np.array_equal(out, oout)
    assert n > 50, n


@pytest.mark.parametrize("seed,nnratio", [(0, 0.75), (7, 0.9)])
def test_search_by_bow_keyframes(gpu, seed, nnratio):
    (k0, d0), (k1, d1) = sc.frames(seed)[0]
    rng = np.random.default_rng(seed + 1)
    mp1 = np.where(rng.random(len(k0)) < 0.8, np.arange(len(k0)), -1).astype(np.int32)
    mp2 = np.where(rng.random(len(k1)) < 0.8, 10000 + np.arange(len(k1)), -1).astype(np.int32)
    b1 = (rng.random(len(k0)) < 0.03).astype(np.uint8)
    b2 = (rng.random(len(k1)) < 0.03).astype(np.uint8)
    m = gpu.ORBmatcher(nnratio, True)
    n, out = m.SearchByBoW_KeyFrames(d0, k0["angle"], mp1, b1, sc.featvec(d0), d1, k1["angle"], mp2, b2,
                                     sc.featvec(d1))
    on, oout = oracle_lib.oracle_search_by_bow_kf(d0, k0["angle"], mp1, b1, sc.featvec(d0), d1, k1["angle"], mp2, b2,
                                                  sc.featvec(d1), nnratio, True)
    assert n == on and np.array_equal(out, oout)
    assert n > 50, n


def _tri_case(seed, stereo_frac):
    (k0, d0), (k1, d1) = sc.frames(seed)[0]
    t = sc.frames(seed)[3]
    rng = np.random.default_rng(seed + 2)
    T1 = np.eye(4, dtype=np.float32)
    T2 = np.eye(4, dtype=np.float32)
    T2[:3, :3] = synthetic.small_rotation(rng, 718.856)
    T2[:3, 3] = [-0.5, 0.02, -0.1]
    uR1 = np.where(rng.random(len(k0)) < stereo_frac, k0["x"] - 20, -1).astype(np.float32)
    uR2 = np.where(rng.random(len(k1)) < stereo_frac, k1["x"] - 20, -1).astype(np.float32)
    KF1 = sc.make_frame(k0, d0, t, T1, uRight=uR1)
    KF2 = sc.make_frame(k1, d1, t, T2, uRight=uR2)
    # F12 = K1^-T [t12]x R12 K2^-1 (KeyFrame-pair fundamental matrix, LocalMapping.cc:ComputeF12)
    R1w, t1w, R2w, t2w = T1[:3, :3], T1[:3, 3], T2[:3, :3], T2[:3, 3]
    R12 = R1w @ R2w.T
    t12 = -R1w @ R2w.T @ t2w + t1w
    fx, fy, cx, cy = synthetic.intrinsics(sc.W, sc.H)
    K = np.array([[fx, 0, cx], [0, fy, cy], [0, 0, 1]])
    F12 = (np.linalg.inv(K).T @ sc.skew(t12) @ R12 @ np.linalg.inv(K)).astype(np.float32)
    h1 = (rng.random(len(k0)) < 0.3).astype(np.uint8)
    h2 = (rng.random(len(k1)) < 0.3).astype(np.uint8)
    return KF1, h1, sc.featvec(d0), KF2, h2, sc.featvec(d1), t["sigma2"], F12


@pytest.mark.parametrize("seed,stereo_frac,only_stereo", [(0, 0.0, False), (8, 0.5, False), (9, 0.6, True)])
def test_search_for_triangulation(gpu, seed, stereo_frac, only_stereo):
    KF1, h1, fv1, KF2, h2, fv2, s2, F12 = _tri_case(seed, stereo_frac)
    m = gpu.ORBmatcher(0.6, True)
    pairs = m.SearchForTriangulation(KF1, h1, fv1, KF2, h2, fv2, s2, F12, only_stereo)
    opairs = oracle_lib.oracle_search_for_triangulation(KF1, h1, fv1, KF2, h2, fv2, s2, F12, only_stereo, True)
    assert np.array_equal(pairs, opairs)
    assert len(pairs) > 10, len(pairs)


def test_searches_refuse_device_pointers(gpu):
    from c_orb_slam_amd._lib import OrbGpuError, lib
    c = sc.reloc_case(0)
    m = gpu.ORBmatcher(0.9, True)
    lib().ORBmatcher_set_device_pointers(m._h, 1)
    with pytest.raises(OrbGpuError):
        m.SearchByProjection_KeyFrame(c["F"], c["cur_mp"].copy(), c["kf_mp"], c["skip"], c["kf_angle"], c["mps"],
                                      c["max_dist"], c["min_dist"], c["logScaleFactor"], 10, 100)


# ---- LocalMapping / LoopClosing projection searches (ORBmatcher.cc:290-403, 825-1326) ----
@pytest.mark.parametrize("seed,scale,th", [(0, 1.3, 10), (3, 0.7, 10), (5, 1.0, 5)])
def test_search_by_projection_sim3(gpu, seed, scale, th):
    c = sc.loop_case(seed, scale=scale)
    m = gpu.ORBmatcher(0.75, True)
    matched = c["matched"].copy()
    n = m.SearchByProjection_Sim3(c["KF"], c["Scw"], c["pts"], c["geo"], c["skip"], matched, c["logScaleFactor"], th)
    on, om = oracle_lib.oracle_search_by_projection_sim3(c["KF"], c["Scw"], c["pts"], c["geo"], c["skip"],
                                                         c["matched"], c["logScaleFactor"], th)
    assert n == on and np.array_equal(matched, om)
    assert n > 100, n


@pytest.mark.parametrize("seed,stereo_frac,th", [(0, 0.5, 3.0), (4, 0.0, 3.0), (6, 1.0, 5.0)])
def test_fuse(gpu, seed, stereo_frac, th):
    c = sc.loop_case(seed, stereo_frac=stereo_frac)
    m = gpu.ORBmatcher(0.6, True)
    n, best = m.Fuse(c["KF"], c["pts"], c["geo"], c["skip"], c["logScaleFactor"], th)
    on, ob = oracle_lib.oracle_fuse(c["KF"], c["pts"], c["geo"], c["skip"], c["logScaleFactor"], th)
    assert n == on and np.array_equal(best, ob)
    assert n > 50, n


@pytest.mark.parametrize("seed,scale", [(1, 1.3), (2, 0.5)])
def test_fuse_sim3(gpu, seed, scale):
    c = sc.loop_case(seed, scale=scale)
    m = gpu.ORBmatcher(0.8, True)
    n, best = m.Fuse_Sim3(c["KF"], c["Scw"], c["pts"], c["geo"], c["skip"], c["logScaleFactor"], 4.0)
    on, ob = oracle_lib.oracle_fuse_sim3(c["KF"], c["Scw"], c["pts"], c["geo"], c["skip"], c["logScaleFactor"], 4.0)
    assert n == on and np.array_equal(best, ob)
    assert n > 100, n


@pytest.mark.parametrize("seed,s12", [(0, 1.02), (7, 0.9), (8, 1.0)])
def test_search_by_sim3(gpu, seed, s12):
    s = sc.sim3_case(seed, s12=s12)
    m = gpu.ORBmatcher(0.75, True)
    m12 = s["m12"].copy()
    n = m.SearchBySim3(s["KF1"], s["mp1"], s["KF2"], s["mp2"], s["pts"], s["geo"], s["bad"], m12, s["s12"],
                       s["R12"], s["t12"], s["logScaleFactor"], 7.5)
    on, om = oracle_lib.oracle_search_by_sim3(s["KF1"], s["mp1"], s["KF2"], s["mp2"], s["pts"], s["geo"], s["bad"],
                                              s["m12"], s["s12"], s["R12"], s["t12"], s["logScaleFactor"], 7.5)
    assert n == on and np.array_equal(m12, om)
    assert n > 50, n


def test_projection_searches_empty_inputs(gpu):
    from c_orb_slam_amd.orb import MapPointGeo, MapPoints
    c = sc.loop_case(0)
    m = gpu.ORBmatcher(0.75, True)
    empty = MapPoints(np.zeros((0, 3)), np.zeros((0, 32)), np.zeros(0))
    eg = MapPointGeo(np.zeros(0), np.zeros(0), np.zeros((0, 3)))
    matched = c["matched"].copy()
    assert m.SearchByProjection_Sim3(c["KF"], c["Scw"], empty, eg, np.zeros(0), matched, c["logScaleFactor"], 10) == 0
    assert np.array_equal(matched, c["matched"])
    assert m.Fuse(c["KF"], empty, eg, np.zeros(0), c["logScaleFactor"], 3.0)[0] == 0
    allskip = np.ones(c["pts"].n, np.uint8)
    n, best = m.Fuse_Sim3(c["KF"], c["Scw"], c["pts"], c["geo"], allskip, c["logScaleFactor"], 4.0)
    assert n == 0 and (best == -1).all()
