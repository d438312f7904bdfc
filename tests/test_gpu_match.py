"""GPU guided matching vs the CPU oracle: bit-exact match indices and counts.

Reference: ORBmatcher::SearchByProjection (src/ORBmatcher.cc:45-129, 1328-1470),
Frame::GetFeaturesInArea (src/Frame.cc:327-380), DescriptorDistance (1647-1663).
"""
import numpy as np
import pytest

import oracle_lib
from c_orb_slam_amd import synthetic
from match_cases import frame_pair, local_queries

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def kitti_frames(gpu):
    frames, Hs, Rs = synthetic.sequence(21, 3, return_rotations=True)
    ex = gpu.ORBextractor(1200, 1.2, 8, 20, 7, max_width=1241, max_height=376, max_batch=3)
    res = ex.extract_batch(frames)
    return frames, Hs, Rs, res, ex.GetScaleFactors()


def test_descriptor_distance(gpu):
    rng = np.random.default_rng(0)
    a = rng.integers(0, 256, (500, 32), dtype=np.uint8)
    b = rng.integers(0, 256, (500, 32), dtype=np.uint8)
    for i in range(500):
        d = gpu.ORBmatcher.DescriptorDistance(a[i], b[i])
        assert d == oracle_lib.lib().ora_descriptor_distance(oracle_lib.ptr(a[i]), oracle_lib.ptr(b[i]))
        assert d == int(np.unpackbits(a[i] ^ b[i]).sum())
    assert gpu.ORBmatcher.DescriptorDistance(a[0], a[0]) == 0
    assert gpu.ORBmatcher.DescriptorDistance(np.zeros(32, np.uint8), np.full(32, 255, np.uint8)) == 256


@pytest.mark.parametrize("stereo,th,checkOri", [(False, 15.0, True), (False, 7.0, False), (True, 7.0, True),
                                                (False, 30.0, True)])
def test_search_by_projection_last(gpu, kitti_frames, stereo, th, checkOri):
    frames, Hs, Rs, res, scale = kitti_frames
    K4 = synthetic.intrinsics(1241, 376)
    rng = np.random.default_rng(int(th) * 7 + stereo)
    (k0, d0), (k1, d1) = res[0], res[1]
    cur, last, mps, last_mp, last_out = frame_pair(k0, d0, k1, d1, Rs[0], K4, 1241, 376, scale, rng, stereo=stereo)
    m = gpu.ORBmatcher(0.9, checkOri)
    cur_mp_g = np.full(cur.N, -1, np.int32)
    cur_mp_o = cur_mp_g.copy()
    ng = m.SearchByProjection_LastFrame(cur, cur_mp_g, last, k0, last_mp, last_out, mps, th, not stereo)
    no = oracle_lib.oracle_search_last(cur, cur_mp_o, last, k0, last_mp, last_out, mps, th, not stereo, 0.9,
                                       checkOri)
    assert ng == no
    assert np.array_equal(cur_mp_g, cur_mp_o), np.nonzero(cur_mp_g != cur_mp_o)[0][:10]
    assert no > 0.3 * len(k1), f"synthetic pair should match well ({no} of {len(k1)})"


def test_search_by_projection_last_preoccupied(gpu, kitti_frames):
    """Occupancy rule: candidates holding a map point with Observations()>0 are skipped."""
    frames, Hs, Rs, res, scale = kitti_frames
    K4 = synthetic.intrinsics(1241, 376)
    rng = np.random.default_rng(99)
    (k0, d0), (k1, d1) = res[1], res[2]
    cur, last, mps, last_mp, last_out = frame_pair(k0, d0, k1, d1, Rs[1], K4, 1241, 376, scale, rng,
                                                   obs_zero_fraction=0.4)
    init = np.where(rng.random(cur.N) < 0.3, rng.integers(0, mps.n, cur.N), -1).astype(np.int32)
    m = gpu.ORBmatcher(0.9, True)
    g, o = init.copy(), init.copy()
    ng = m.SearchByProjection_LastFrame(cur, g, last, k0, last_mp, last_out, mps, 15.0, True)
    no = oracle_lib.oracle_search_last(cur, o, last, k0, last_mp, last_out, mps, 15.0, True, 0.9, True)
    assert ng == no and np.array_equal(g, o)


@pytest.mark.parametrize("th,nnratio", [(1.0, 0.8), (3.0, 0.8), (5.0, 0.8), (10.0, 0.6)])
def test_search_by_projection_local(gpu, kitti_frames, th, nnratio):
    frames, Hs, Rs, res, scale = kitti_frames
    K4 = synthetic.intrinsics(1241, 376)
    rng = np.random.default_rng(int(th * 10))
    (k0, d0), (k1, d1) = res[0], res[1]
    cur, last, mps, last_mp, last_out = frame_pair(k0, d0, k1, d1, Rs[0], K4, 1241, 376, scale, rng, stereo=True)
    iv, px, pxr, py, lvl, vc = local_queries(k0, d0, Hs[0], rng)
    mp_index = np.arange(len(k0), dtype=np.int32)
    init = np.where(rng.random(cur.N) < 0.2, rng.integers(0, mps.n, cur.N), -1).astype(np.int32)
    m = gpu.ORBmatcher(nnratio, True)
    g, o = init.copy(), init.copy()
    ng = m.SearchByProjection_MapPoints(cur, g, iv, px, pxr, py, lvl, vc, mp_index, mps, th)
    no = oracle_lib.oracle_search_local(cur, o, mps.obs, iv, px, pxr, py, lvl, vc, mps.desc[mp_index], mp_index,
                                        th, nnratio)
    assert ng == no
    assert np.array_equal(g, o), np.nonzero(g != o)[0][:10]


def test_search_candidates_csr(gpu):
    rng = np.random.default_rng(5)
    q = rng.integers(0, 256, (300, 32), dtype=np.uint8)
    t = rng.integers(0, 256, (900, 32), dtype=np.uint8)
    t[::7] = t[3]  # duplicates -> equal distances exercise the earliest-wins tie rule
    counts = rng.integers(0, 150, 300)
    counts[5] = 0
    off = np.concatenate([[0], np.cumsum(counts)]).astype(np.int32)
    cand = rng.integers(0, 900, off[-1]).astype(np.int32)
    m = gpu.ORBmatcher()
    dist, bi, bd, sd = m.SearchCandidates(q, t, off, cand)
    ref = np.array([int(np.unpackbits(q[i] ^ t[c]).sum()) for i in range(300) for c in cand[off[i]:off[i + 1]]])
    assert np.array_equal(dist, ref)
    for i in range(300):
        ds = ref[off[i]:off[i + 1]]
        if len(ds) == 0:
            assert bi[i] == -1 and bd[i] == 256 and sd[i] == 256
            continue
        j = int(np.argmin(ds))  # first minimum
        assert bi[i] == cand[off[i] + j] and bd[i] == ds[j]
        assert sd[i] == (np.sort(ds)[1] if len(ds) > 1 else 256)


def test_batched_pairs_equal_single(gpu, kitti_frames):
    import ctypes as C
    from c_orb_slam_amd._lib import lib, ptr, KP_DTYPE
    frames, Hs, Rs, res, scale = kitti_frames
    K4 = synthetic.intrinsics(1241, 376)
    probs = []
    for p in range(2):
        rng = np.random.default_rng(300 + p)
        (k0, d0), (k1, d1) = res[p], res[p + 1]
        probs.append((frame_pair(k0, d0, k1, d1, Rs[p], K4, 1241, 376, scale, rng), k0))
    m = gpu.ORBmatcher(0.9, True)
    singles = []
    for (cur, last, mps, lm, lo), k0 in probs:
        g = np.full(cur.N, -1, np.int32)
        n = m.SearchByProjection_LastFrame(cur, g, last, k0, lm, lo, mps, 15.0, True)
        singles.append((n, g))
    # batch call through the C ABI
    from c_orb_slam_amd._lib import orb_frame, orb_mappoints
    curs = (orb_frame * 2)(*[p[0][0].cstruct() for p in probs])
    lasts = (orb_frame * 2)(*[p[0][1].cstruct() for p in probs])
    mpss = (orb_mappoints * 2)(*[p[0][2].cstruct() for p in probs])
    outs = [np.full(p[0][0].N, -1, np.int32) for p in probs]
    lks = [np.ascontiguousarray(p[1], KP_DTYPE) for p in probs]
    arr = lambda xs: (C.c_void_p * 2)(*[x.ctypes.data for x in xs])
    nm = np.zeros(2, np.int32)
    rc = lib().ORBmatcher_SearchByProjection_LastFrame_batch(m._h, 2, curs, arr(outs), lasts, arr(lks),
                                                             arr([p[0][3] for p in probs]),
                                                             arr([p[0][4] for p in probs]), mpss, 15.0, 1, ptr(nm))
    assert rc == 0
    for p in range(2):
        assert nm[p] == singles[p][0] and np.array_equal(outs[p], singles[p][1])


@pytest.mark.parametrize("frac", [0.6, 1.0])
def test_search_by_projection_clustered_cell(gpu, kitti_frames, frac):
    """Many keypoints in one grid cell (AssignFeaturesToGrid, Frame.cc:230-245): the device grid
    keeps index order inside a crowded cell, so GetFeaturesInArea enumerates (and breaks
    distance ties) as the reference does."""
    frames, Hs, Rs, res, scale = kitti_frames
    K4 = synthetic.intrinsics(1241, 376)
    rng = np.random.default_rng(int(frac * 10) + 5)
    (k0, d0), (k1, d1) = res[0], res[1]
    k1 = k1.copy()
    sel = rng.random(len(k1)) < frac
    k1["x"][sel] = rng.uniform(620.0, 629.0, sel.sum()).astype(np.float32)   # grid cell (32, 24)
    k1["y"][sel] = rng.uniform(187.8, 191.0, sel.sum()).astype(np.float32)
    d1 = d1.copy()
    d1[sel] = d0[rng.integers(0, len(d0), sel.sum())]   # equal descriptors: many distance ties
    cur, last, mps, last_mp, last_out = frame_pair(k0, d0, k1, d1, Rs[0], K4, 1241, 376, scale, rng)
    m = gpu.ORBmatcher(0.9, True)
    for th in (15.0, 100.0):
        g = np.full(cur.N, -1, np.int32)
        o = g.copy()
        ng = m.SearchByProjection_LastFrame(cur, g, last, k0, last_mp, last_out, mps, th, True)
        no = oracle_lib.oracle_search_last(cur, o, last, k0, last_mp, last_out, mps, th, True, 0.9, True)
        assert ng == no and np.array_equal(g, o), (th, ng, no)


def _dense_ref(q, t):
    """The reference loop over train rows in order (ORBmatcher.cc:1647-1663 distance; best on a
    strictly smaller distance, an equal one becomes the second), vectorised with numpy."""
    if len(t) == 0:
        return np.full(len(q), -1), np.full(len(q), 256), np.full(len(q), 256)
    d = np.unpackbits(q[:, None, :] ^ t[None, :, :], axis=2).sum(2)
    bi = d.argmin(1)                                  # first index of the minimum
    bd = d.min(1)
    sd = np.partition(d, 1, axis=1)[:, 1] if d.shape[1] > 1 else np.full(len(q), 256)
    return bi, bd, sd


def test_search_dense_matches_reference_loop(gpu):
    """Brute-force matching with LDS-resident train blocks: every query's best index, best and
    second distance equal the sequential loop's, across block edges (train counts around the
    256-row block), duplicate descriptors (ties), an empty train set and a one-row train set."""
    import oracle_lib
    rng = np.random.default_rng(41)
    shapes = [(1200, 1200), (257, 256), (300, 257), (513, 511), (64, 1), (40, 0), (1, 700)]
    qs, ts = [], []
    for nq, nt in shapes:
        q = rng.integers(0, 256, (nq, 32), dtype=np.uint8)
        t = rng.integers(0, 256, (nt, 32), dtype=np.uint8)
        if nt > 10:
            t[nt // 2] = t[3]                        # duplicate rows: equal distances, earliest wins
            q[: min(nq, 5)] = t[3]                   # exact matches (distance 0) at a duplicated row
        qs.append(q)
        ts.append(t)
    m = gpu.ORBmatcher(0.9, True)
    out = m.SearchDense(qs, ts)
    for q, t, (bi, bd, sd) in zip(qs, ts, out):
        rbi, rbd, rsd = _dense_ref(q, t)
        assert np.array_equal(bi, rbi) and np.array_equal(bd, rbd) and np.array_equal(sd, rsd)
    q, t = qs[1], ts[1]   # the distance itself is the oracle's DescriptorDistance
    for k in range(0, len(q), 37):
        L = oracle_lib.lib()
        assert out[1][1][k] == min(L.ora_descriptor_distance(oracle_lib.ptr(np.ascontiguousarray(q[k])),
                                                             oracle_lib.ptr(np.ascontiguousarray(t[j])))
                                   for j in range(len(t)))
