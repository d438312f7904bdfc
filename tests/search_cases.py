"""Inputs for the remaining ORBmatcher searches, built from real (oracle) extractor output on
synthetic KITTI-shaped frames: frame t+1 is frame t under a camera rotation (synthetic.sequence).

Vocabulary: ORBvoc.txt is not shipped with the reference, so FeatureVectors come
from a stand-in node assignment -- the low 6 bits of descriptor byte 0 -- which, like DBoW2's
levelsup node, puts near-identical descriptors in the same node."""
import numpy as np

import oracle_lib
from c_orb_slam_amd import synthetic
from c_orb_slam_amd.orb import FeatureVector, Frame, MapPoints

W, H = 1241, 376


def frames(seed=0, n=2, nfeat=1200):
    imgs, Hs, Rs = synthetic.sequence(seed, n, W, H, return_rotations=True)
    ex = oracle_lib.OracleExtractor(nfeat, 1.2, 8, 20, 7)
    out = [ex(im) for im in imgs]
    t = ex.tables()
    return out, Rs, Hs, t


def node_ids(desc):
    return (np.asarray(desc)[:, 0] & 0x3F).astype(np.int64)


def featvec(desc):
    return FeatureVector(node_ids(desc))


def make_frame(kps, desc, t, Tcw, uRight=None):
    fx, fy, cx, cy = synthetic.intrinsics(W, H)
    return Frame(kps, desc, t["scale"], Tcw, fx, fy, cx, cy, synthetic.KITTI_BF, W, H, uRight=uRight)


def reloc_case(seed=0, occ_frac=0.1, skip_frac=0.05):
    """SearchByProjection(CurrentFrame, pKF, sAlreadyFound, th, ORBdist) (Tracking.cc:1452)."""
    (k0, d0), (k1, d1) = frames(seed)[0]
    _, Rs, _, t = frames(seed)
    rng = np.random.default_rng(seed + 100)
    fx, fy, cx, cy = synthetic.intrinsics(W, H)
    X = synthetic.lift_map_points(rng, k0, (fx, fy, cx, cy))
    n0 = len(k0)
    kf_mp = np.where(rng.random(n0) < 0.9, np.arange(n0), -1).astype(np.int32)
    skip = (rng.random(n0) < skip_frac).astype(np.uint8)
    dist = np.linalg.norm(X, axis=1).astype(np.float32)          # keyframe 0 is the world origin
    lvl_scale = t["scale"][k0["octave"]]
    max_dist = (dist * lvl_scale).astype(np.float32)              # UpdateNormalAndDepth (MapPoint.cc:366-368)
    min_dist = (max_dist / t["scale"][-1]).astype(np.float32)
    mps = MapPoints(X, d0, np.ones(n0, np.int32))
    F = make_frame(k1, d1, t, synthetic.pose_from_rotation(Rs[0]))
    cur_mp = np.where(rng.random(len(k1)) < occ_frac, rng.integers(0, n0, len(k1)), -1).astype(np.int32)
    log_sf = np.float32(np.log(np.float32(1.2)))
    return dict(F=F, cur_mp=cur_mp, kf_mp=kf_mp, skip=skip, kf_angle=k0["angle"].copy(), mps=mps,
                max_dist=max_dist, min_dist=min_dist, logScaleFactor=log_sf)


def skew(v):
    return np.array([[0, -v[2], v[1]], [v[2], 0, -v[0]], [-v[1], v[0], 0]])


def _geo(X, kps, t, center=(0.0, 0.0, 0.0)):
    """MapPoint::UpdateNormalAndDepth (MapPoint.cc:334-371) for one observing keyframe."""
    from c_orb_slam_amd.orb import MapPointGeo
    PC = X - np.asarray(center, np.float32)
    dist = np.linalg.norm(PC, axis=1).astype(np.float32)
    normal = (PC / dist[:, None]).astype(np.float32)
    max_dist = (dist * t["scale"][kps["octave"]]).astype(np.float32)
    min_dist = (max_dist / t["scale"][-1]).astype(np.float32)
    return MapPointGeo(max_dist, min_dist, normal)


def loop_case(seed=0, scale=1.3, skip_frac=0.05, occ_frac=0.1, stereo_frac=0.5):
    """Map points of keyframe 0 (world = KF0 camera) seen from keyframe 1 (a rotation later):
    Scw = scale * [R | t] for the Sim3 searches, KF1 with partial stereo for Fuse."""
    (k0, d0), (k1, d1) = frames(seed)[0]
    _, Rs, _, t = frames(seed)
    rng = np.random.default_rng(seed + 200)
    K4 = synthetic.intrinsics(W, H)
    X = synthetic.lift_map_points(rng, k0, K4)
    n0 = len(k0)
    pts = MapPoints(X, d0, np.ones(n0, np.int32))
    geo = _geo(X, k0, t)
    Tcw = synthetic.pose_from_rotation(Rs[0])
    Scw = Tcw.copy()
    Scw[:3, :] *= np.float32(scale)
    depth = np.float32(20.0)
    uR = np.where(rng.random(len(k1)) < stereo_frac,
                  k1["x"] - np.float32(synthetic.KITTI_BF) / depth * rng.uniform(0.5, 2.0, len(k1)), -1.0)
    KF = make_frame(k1, d1, t, Tcw, uRight=uR.astype(np.float32))
    skip = (rng.random(n0) < skip_frac).astype(np.uint8)
    matched = np.where(rng.random(len(k1)) < occ_frac, rng.integers(0, n0, len(k1)), -1).astype(np.int32)
    log_sf = np.float32(np.log(np.float32(1.2)))
    return dict(KF=KF, Scw=Scw, pts=pts, geo=geo, skip=skip, matched=matched, logScaleFactor=log_sf)


def sim3_case(seed=0, s12=1.02, bad_frac=0.03, pre_frac=0.05):
    """SearchBySim3(pKF1, pKF2, ...) (LoopClosing.cc:393): KF1 = frame 1 (pose R), KF2 = frame 0
    (identity); points of both keyframes in one table; S12 = (s12, R, 0) maps camera 2 to 1."""
    (k0, d0), (k1, d1) = frames(seed)[0]
    _, Rs, _, t = frames(seed)
    rng = np.random.default_rng(seed + 300)
    K4 = synthetic.intrinsics(W, H)
    R = np.asarray(Rs[0], np.float32)
    X2 = synthetic.lift_map_points(rng, k0, K4)                  # KF2 = world
    X1 = (synthetic.lift_map_points(rng, k1, K4) @ R).astype(np.float32)   # Xw = R^T Xc1
    pts = MapPoints(np.concatenate([X2, X1]), np.concatenate([d0, d1]), np.ones(len(k0) + len(k1), np.int32))
    from c_orb_slam_amd.orb import MapPointGeo
    g2, g1 = _geo(X2, k0, t), _geo(X1, k1, t)
    geo = MapPointGeo(np.concatenate([g2.max_dist, g1.max_dist]), np.concatenate([g2.min_dist, g1.min_dist]),
                      np.concatenate([g2.normal, g1.normal]))
    n2, n1 = len(k0), len(k1)
    mp2 = np.where(rng.random(n2) < 0.9, np.arange(n2), -1).astype(np.int32)
    mp1 = np.where(rng.random(n1) < 0.9, n2 + np.arange(n1), -1).astype(np.int32)
    bad = (rng.random(n2 + n1) < bad_frac).astype(np.uint8)
    m12 = np.full(n1, -1, np.int32)
    pre = rng.random(n1) < pre_frac
    m12[pre] = np.where(rng.random(pre.sum()) < 0.5, rng.integers(0, n2, pre.sum()), -2)
    KF1 = make_frame(k1, d1, t, synthetic.pose_from_rotation(R))
    KF2 = make_frame(k0, d0, t, np.eye(4, dtype=np.float32))
    log_sf = np.float32(np.log(np.float32(1.2)))
    return dict(KF1=KF1, mp1=mp1, KF2=KF2, mp2=mp2, pts=pts, geo=geo, bad=bad, m12=m12, s12=np.float32(s12),
                R12=R, t12=np.zeros(3, np.float32), logScaleFactor=log_sf)
