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
