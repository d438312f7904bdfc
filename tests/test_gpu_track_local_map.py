"""TrackLocalMap's device path (Tracking.cc:930-974) vs the CPU oracle:

* Frame::isInFrustum(pMP, 0.5) (Frame.cc:269-325) with MapPoint::PredictScale
  (MapPoint.cc:402-417) for every local map point -- in-view flags and the tracking fields
  (mTrackProjX / XR / Y, mnTrackScaleLevel, mTrackViewCos) bit-exact, every rejection branch
  exercised (behind the camera, outside the image, outside the scale-invariance distance,
  viewing angle, skipped points);
* Tracking::SearchLocalPoints (Tracking.cc:1143-1193): isInFrustum + SearchByProjection(F,
  mvpLocalMapPoints, th) with ORBmatcher(0.8) -- match indices and counts bit-exact, batched
  over frames in one launch set."""
import numpy as np
import pytest

import oracle_lib
from c_orb_slam_amd import synthetic
from c_orb_slam_amd.orb import Frame

pytestmark = pytest.mark.gpu

W, H = 1241, 376


@pytest.fixture(scope="module")
def seq(gpu):
    frames, Hs, Rs = synthetic.sequence(33, 4, return_rotations=True)
    ex = gpu.ORBextractor(1200, 1.2, 8, 20, 7, max_width=W, max_height=H, max_batch=4)
    res = ex.extract_batch(frames)
    return Rs, res, ex.GetScaleFactors()


def local_map(rng, kps, desc, scale, Twc=np.eye(4, dtype=np.float32), extra=300):
    """Map points lifted from a keyframe's keypoints (world = that frame's camera, then Twc), with
    the MapPoint fields UpdateNormalAndDepth sets (MapPoint.cc:349-371), plus points that fail
    each isInFrustum test."""
    fx, fy, cx, cy = synthetic.intrinsics(W, H)
    n = len(kps)
    d = rng.uniform(4.0, 60.0, n)
    Xc = np.stack([(kps["x"] - cx) / fx * d, (kps["y"] - cy) / fy * d, d], 1)
    oct_ = kps["octave"].astype(int)
    # extras: behind the camera, far outside the image, scale-invariance misses, oblique normals
    e = rng.integers(0, 4, extra)
    Xe = rng.normal(0, 1, (extra, 3)) * [10, 5, 20]
    Xe[e == 0, 2] = -np.abs(Xe[e == 0, 2]) - 1
    Xe[e == 1, :2] *= 50
    Xe[e >= 2, 2] = np.abs(Xe[e >= 2, 2]) + 5
    X = np.vstack([Xc, Xe])
    oct_all = np.concatenate([oct_, rng.integers(0, 8, extra)])
    dist = np.linalg.norm(X, axis=1)
    mx = dist * scale[oct_all]
    mx[n:][e[:] == 2] *= rng.choice([0.3, 3.0], int((e == 2).sum()))      # outside [0.8 min, 1.2 max]
    mn = mx / scale[7]
    nrm = X / dist[:, None]
    tilt = np.where(np.concatenate([rng.random(n) < 0.05, e == 3]), 1.5, 0.1)
    nrm = nrm + rng.normal(0, 1, nrm.shape) * tilt[:, None]
    nrm /= np.linalg.norm(nrm, axis=1, keepdims=True)
    R, t = Twc[:3, :3].astype(np.float64), Twc[:3, 3].astype(np.float64)
    Xw = X @ R.T + t
    nw = nrm @ R.T
    m = len(Xw)
    dsc = np.vstack([desc, rng.integers(0, 256, (extra, 32), dtype=np.uint8)])
    return dict(pos=Xw.astype(np.float32), desc=dsc, obs=rng.integers(0, 5, m).astype(np.int32),
                max_dist=mx.astype(np.float32), min_dist=mn.astype(np.float32), normal=nw.astype(np.float32),
                skip=(rng.random(m) < 0.08).astype(np.uint8))


def cur_frame(rng, k1, d1, scale, Rs, stereo=True):
    fx, fy, cx, cy = synthetic.intrinsics(W, H)
    bf = synthetic.KITTI_BF
    uR = None
    if stereo:
        dd = rng.uniform(5, 50, len(k1)).astype(np.float32)
        uR = np.where(rng.random(len(k1)) < 0.6, k1["x"] - np.float32(bf) / dd, -1).astype(np.float32)
    T = synthetic.pose_from_rotation(Rs)
    return Frame(k1, d1, scale, T, fx, fy, cx, cy, bf if stereo else 0.0, W, H, uRight=uR)


def test_is_in_frustum_matches_oracle(gpu, seq):
    Rs, res, scale = seq
    lsf = np.float32(np.log(np.float32(1.2)))
    rng = np.random.default_rng(1)
    frames, maps = [], []
    for f in range(3):
        (k0, d0), (k1, d1) = res[f], res[f + 1]
        maps.append(local_map(rng, k0, d0, scale))
        frames.append(cur_frame(rng, k1, d1, scale, Rs[f]))
    maps.append(dict(pos=np.zeros((0, 3), np.float32), desc=np.zeros((0, 32), np.uint8), obs=np.zeros(0, np.int32),
                     max_dist=np.zeros(0, np.float32), min_dist=np.zeros(0, np.float32),
                     normal=np.zeros((0, 3), np.float32), skip=np.zeros(0, np.uint8)))   # empty local map
    frames.append(frames[0])
    m = gpu.ORBmatcher(0.8, False)
    g = m.isInFrustum(frames, maps, lsf)
    for F, M, gr in zip(frames, maps, g):
        o = oracle_lib.oracle_is_in_frustum(F, M, lsf)
        assert gr["nvisible"] == o["nvisible"]
        assert np.array_equal(gr["in_view"], o["in_view"])
        v = o["in_view"].astype(bool)
        for k in ("proj_x", "proj_xr", "proj_y", "level", "view_cos"):
            assert np.array_equal(gr[k][v], o[k][v]), k
    # every rejection branch and the acceptance path were taken
    o = oracle_lib.oracle_is_in_frustum(frames[0], maps[0], lsf)
    assert 0 < o["nvisible"] < len(maps[0]["pos"]) - maps[0]["skip"].sum()
    assert len(np.unique(o["level"][o["in_view"].astype(bool)])) >= 4


@pytest.mark.parametrize("th", [1.0, 3.0, 5.0])
def test_search_local_points_matches_oracle(gpu, seq, th):
    Rs, res, scale = seq
    lsf = np.float32(np.log(np.float32(1.2)))
    rng = np.random.default_rng(int(th * 10))
    frames, maps, cms = [], [], []
    for f in range(3):
        (k0, d0), (k1, d1) = res[f], res[f + 1]
        M = local_map(rng, k0, d0, scale)
        F = cur_frame(rng, k1, d1, scale, Rs[f], stereo=f != 1)
        cm = np.where(rng.random(F.N) < 0.15, rng.integers(0, len(M["pos"]), F.N), -1).astype(np.int32)
        M["skip"][cm[cm >= 0]] = 1            # points already in the frame (mnLastFrameSeen)
        frames.append(F)
        maps.append(M)
        cms.append(cm)
    m = gpu.ORBmatcher(0.8, False)
    g = [c.copy() for c in cms]
    nm, nv = m.SearchLocalPoints(frames, g, maps, lsf, th)
    gd = [c.copy() for c in cms]   # the deferred chain form gives the same matches and counts
    nmd, nvd = m.SearchLocalPoints(frames, gd, maps, lsf, th, deferred=True)
    assert np.array_equal(nm, nmd) and np.array_equal(nv, nvd)
    assert all(np.array_equal(a, b) for a, b in zip(g, gd))
    for F, M, c0, gc, n1, n2 in zip(frames, maps, cms, g, nm, nv):
        oc = c0.copy()
        no, nvo = oracle_lib.oracle_search_local_points(F, oc, M, lsf, th, 0.8)
        assert n2 == nvo and n1 == no
        assert np.array_equal(gc, oc), np.nonzero(gc != oc)[0][:10]
        assert no > 50


def test_search_local_points_ratio_override(gpu, seq):
    """The reference's SearchLocalPoints builds ORBmatcher(0.8) (Tracking.cc:1184) while TrackWithMotionModel's
    matcher is ORBmatcher(0.9, true) (Tracking.cc:869): a 0.9-constructed matcher given nnratio=0.8 for the call must
    give the oracle's 0.8 result (so one deferred chain serves both searches), and 0.9 where it differs."""
    Rs, res, scale = seq
    lsf = np.float32(np.log(np.float32(1.2)))
    rng = np.random.default_rng(77)
    frames, maps, cms = [], [], []
    for f in range(3):
        (k0, d0), (k1, d1) = res[f], res[f + 1]
        M = local_map(rng, k0, d0, scale)
        frames.append(cur_frame(rng, k1, d1, scale, Rs[f], stereo=True))
        maps.append(M)
        cms.append(np.full(frames[-1].N, -1, np.int32))
    m = gpu.ORBmatcher(0.9, True)
    for ratio, deferred in ((0.8, False), (0.8, True), (0.0, False)):
        g = [c.copy() for c in cms]
        nm, nv = m.SearchLocalPoints(frames, g, maps, lsf, 1.0, deferred=deferred, nnratio=ratio)
        want = ratio if ratio > 0 else 0.9
        for F, M, c0, gc, n1, n2 in zip(frames, maps, cms, g, nm, nv):
            oc = c0.copy()
            no, nvo = oracle_lib.oracle_search_local_points(F, oc, M, lsf, 1.0, want)
            assert (n1, n2) == (no, nvo), (ratio, n1, no)
            assert np.array_equal(gc, oc)


def test_create_stereo_points_and_local_prep(gpu):
    """MapPoint_CreateStereo_batch_device (UnprojectStereo + UpdateNormalAndDepth for one
    observation) against the oracle's UnprojectStereo and the float / double convention written
    out in numpy; Tracking_PrepareLocalSearch_batch_device against its definition."""
    import ctypes as C
    import torch
    from c_orb_slam_amd._lib import lib, orb_newpoints, orb_localprep
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(3)
    fx, fy, cx, cy = synthetic.intrinsics(W, H)
    n = 1800
    k = np.zeros(n, oracle_lib.KP_DTYPE)
    k["x"] = rng.uniform(0, W, n)
    k["y"] = rng.uniform(0, H, n)
    k["octave"] = rng.integers(0, 8, n)
    dep = rng.uniform(-5, 60, n).astype(np.float32)
    a = rng.normal(0, 0.2, 3)
    Rm = np.linalg.qr(np.eye(3) + np.array([[0, -a[2], a[1]], [a[2], 0, -a[0]], [-a[1], a[0], 0]]))[0]
    Twc = np.eye(4, dtype=np.float32)
    Twc[:3, :3] = Rm
    Twc[:3, 3] = rng.normal(0, 3, 3)
    scale = (np.float32(1.2) ** np.arange(8)).astype(np.float32)
    t = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(dev)
    dk, dd, dT, ds = t(k.view(np.int32).reshape(n, 7)), t(dep), t(Twc.reshape(16)), t(scale)
    X = torch.zeros((n, 3), device=dev)
    row = torch.full((n,), -7, dtype=torch.int32, device=dev)
    nrm = torch.zeros((n, 3), device=dev)
    mx, mn = torch.zeros(n, device=dev), torch.zeros(n, device=dev)
    m = gpu.ORBmatcher(0.8, False)
    q = orb_newpoints(n, dk.data_ptr(), dd.data_ptr(), dT.data_ptr(), float(fx), float(fy), float(cx), float(cy),
                      ds.data_ptr(), 8, 100, X.data_ptr(), row.data_ptr(), nrm.data_ptr(), mx.data_ptr(), mn.data_ptr())
    assert lib().MapPoint_CreateStereo_batch_device(m._h, 1, C.byref(q)) == 0
    torch.cuda.synchronize()
    x3, slot = oracle_lib.oracle_unproject_stereo(k, dep, Twc, fx, fy, cx, cy)
    ok = dep > 0
    assert np.array_equal(row.cpu().numpy(), np.where(ok, 100 + np.arange(n), -1))
    assert np.array_equal(X.cpu().numpy()[ok], x3[ok])
    PO = (x3[ok] - Twc[:3, 3]).astype(np.float32)
    nd = np.sqrt((PO[:, 0].astype(np.float64) * PO[:, 0] + PO[:, 1].astype(np.float64) * PO[:, 1]) +
                 PO[:, 2].astype(np.float64) * PO[:, 2])
    inv = (1.0 / nd).astype(np.float32)
    assert np.array_equal(nrm.cpu().numpy()[ok], PO * inv[:, None])
    mxo = nd.astype(np.float32) * scale[k["octave"][ok]]
    assert np.array_equal(mx.cpu().numpy()[ok], mxo)
    assert np.array_equal(mn.cpu().numpy()[ok], (mxo / scale[7]).astype(np.float32))
    # PrepareLocalSearch: skip = no map point | in the frame; outliers dropped
    nr, N = 5000, 1200
    rows = np.where(rng.random(nr) < 0.2, -1, np.arange(nr)).astype(np.int32)
    cm = np.where(rng.random(N) < 0.5, rng.integers(0, nr, N), -1).astype(np.int32)
    outl = (rng.random(N) < 0.1).astype(np.uint8)
    dcm, dout, drow = t(cm), t(outl), t(rows)
    dskip = torch.full((nr,), 9, dtype=torch.uint8, device=dev)
    pq = orb_localprep(N, dcm.data_ptr(), dout.data_ptr(), nr, drow.data_ptr(), dskip.data_ptr())
    assert lib().Tracking_PrepareLocalSearch_batch_device(m._h, 1, C.byref(pq)) == 0
    sk = (rows < 0).astype(np.uint8)
    sk[cm[cm >= 0]] = 1
    assert np.array_equal(dskip.cpu().numpy(), sk)
    assert np.array_equal(dcm.cpu().numpy(), np.where((cm >= 0) & (outl == 1), -1, cm))
