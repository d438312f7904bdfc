"""GPU ORB extraction vs the CPU oracle: bit-exact keypoints, descriptors, pyramid.

Reference: ORBextractor::operator() (src/ORBextractor.cc:1043-1105).  Inputs are
seeded synthetic images (SURVEY.md §8d config 2 generator) at KITTI (1241x376),
EuRoC (752x480) and TUM (640x480) sizes.
"""
import numpy as np
import pytest

import oracle_lib
from c_orb_slam_amd import synthetic

pytestmark = pytest.mark.gpu

CASES = [  # (w, h, nfeatures, seed)
    (1241, 376, 1200, 0),
    (1241, 376, 2000, 1),
    (752, 480, 1200, 2),
    (640, 480, 1000, 3),
]


def _diag(gk, gd, ok, od):
    msg = [f"gpu n={len(gk)} oracle n={len(ok)}"]
    for l in range(8):
        a, b = gk[gk["octave"] == l], ok[ok["octave"] == l]
        if len(a) != len(b) or not np.array_equal(a.view(np.uint8), b.view(np.uint8)):
            msg.append(f" level {l}: gpu {len(a)} oracle {len(b)}")
            n = min(len(a), len(b))
            for f in ("x", "y", "angle", "response"):
                bad = np.nonzero(a[f][:n] != b[f][:n])[0]
                if len(bad):
                    i = bad[0]
                    msg.append(f"   first {f} mismatch at {i}: gpu {a[i]} oracle {b[i]}")
                    break
            break
    return "\n".join(msg)


@pytest.mark.parametrize("w,h,nf,seed", CASES)
def test_extract_bit_exact(gpu, w, h, nf, seed):
    frames, _ = synthetic.sequence(seed, 1, w, h)
    img = frames[0]
    ex = gpu.ORBextractor(nf, 1.2, 8, 20, 7, max_width=w, max_height=h)
    orc = oracle_lib.OracleExtractor(nf, 1.2, 8, 20, 7)
    gk, gd = ex(img)
    ok, od = orc(img)
    # pyramid (with its border) first: it localises any divergence
    for l in range(8):
        gl = ex.image_pyramid_level(l)
        ol = orc.level(l)
        assert gl.shape == ol.shape
        assert np.array_equal(gl, ol), f"pyramid level {l} differs at {np.argwhere(gl != ol)[:5]}"
    for l in range(8):
        gb, ob = ex.blurred_level(l), orc.blurred(l)
        assert np.array_equal(gb, ob), f"blurred level {l} differs at {np.argwhere(gb != ob)[:5]}"
    assert len(gk) == len(ok) and np.array_equal(gk.view(np.uint8), ok.view(np.uint8)), _diag(gk, gd, ok, od)
    assert np.array_equal(gd, od)


def test_extract_batch_matches_single(gpu):
    frames, _ = synthetic.sequence(11, 4, 1241, 376)
    ex = gpu.ORBextractor(1200, 1.2, 8, 20, 7, max_width=1241, max_height=376, max_batch=4)
    orc = oracle_lib.OracleExtractor(1200, 1.2, 8, 20, 7)
    res = ex.extract_batch(frames)
    for b in range(4):
        ok, od = orc(frames[b])
        k, d = res[b]
        assert np.array_equal(k.view(np.uint8), ok.view(np.uint8)), f"image {b}"
        assert np.array_equal(d, od), f"image {b}"


def test_extractor_tables(gpu):
    ex = gpu.ORBextractor(1200, 1.2, 8, 20, 7, max_width=640, max_height=480)
    t = oracle_lib.OracleExtractor(1200, 1.2, 8, 20, 7).tables()
    assert np.array_equal(ex.GetScaleFactors(), t["scale"])
    assert np.array_equal(ex.GetInverseScaleFactors(), t["inv_scale"])
    assert np.array_equal(ex.GetScaleSigmaSquares(), t["sigma2"])
    assert np.array_equal(ex.GetInverseScaleSigmaSquares(), t["inv_sigma2"])
    assert np.array_equal(ex.features_per_level(), t["n_per_level"])
    assert ex.GetLevels() == 8 and abs(ex.GetScaleFactor() - 1.2) < 1e-7


def test_extract_edge_cases(gpu):
    ex = gpu.ORBextractor(500, 1.2, 8, 20, 7, max_width=640, max_height=480)
    # empty image: operator() returns immediately (ORBextractor.cc:1046-1047)
    k, d = ex(np.zeros((0, 0), np.uint8))
    assert len(k) == 0 and d is None
    # flat image: no corners at all -> zero keypoints, descriptors released (1064-1065)
    k, d = ex(np.full((480, 640), 128, np.uint8))
    assert len(k) == 0 and d is None
    # image larger than the declared maximum is rejected, not overrun
    with pytest.raises(gpu.OrbGpuError):
        ex(np.zeros((481, 640), np.uint8))


def test_extract_non_contiguous_stride(gpu):
    frames, _ = synthetic.sequence(5, 1, 640, 480)
    big = np.zeros((480, 700), np.uint8)
    big[:, :640] = frames[0]
    view = big[:, :640]
    ex = gpu.ORBextractor(1000, 1.2, 8, 20, 7, max_width=640, max_height=480)
    import ctypes as C
    from c_orb_slam_amd._lib import KP_DTYPE, lib, ptr
    kps = np.zeros(4096, KP_DTYPE)
    desc = np.zeros((4096, 32), np.uint8)
    n = C.c_int()
    assert lib().ORBextractor_extract(ex._h, C.c_void_p(view.ctypes.data), 640, 480, 700, ptr(kps), ptr(desc),
                                      4096, C.byref(n)) == 0
    ok, od = oracle_lib.OracleExtractor(1000, 1.2, 8, 20, 7)(frames[0])
    assert np.array_equal(kps[:n.value].view(np.uint8), ok.view(np.uint8))
    assert np.array_equal(desc[:n.value], od)


def test_extract_images_separate_host_buffers(gpu):
    """ORBextractor_extract_images: Frame(imLeft, imRight)'s two host images at unrelated addresses
    (one with a padded row stride) in one call; each image's keypoints / descriptors equal the
    oracle's, over two calls (the pinned staging block reused); a null image is rejected."""
    import ctypes as C
    from c_orb_slam_amd._lib import KP_DTYPE, lib, ptr
    frames, _ = synthetic.sequence(21, 4, 1241, 376)
    ex = gpu.ORBextractor(1200, 1.2, 8, 20, 7, max_width=1241, max_height=376, max_batch=2)
    orc = oracle_lib.OracleExtractor(1200, 1.2, 8, 20, 7)
    cap = 4096
    for call in range(2):
        a = np.ascontiguousarray(frames[2 * call])
        big = np.zeros((376, 1300), np.uint8)   # the second image inside a wider buffer: row stride 1300
        big[:, :1241] = frames[2 * call + 1]
        # both images share the row stride of the call: copy the first into a 1300-wide buffer too
        abig = np.zeros((376, 1300), np.uint8)
        abig[:, :1241] = a
        lst = (C.c_void_p * 2)(abig.ctypes.data, big.ctypes.data)
        kps = np.zeros(2 * cap, KP_DTYPE)
        desc = np.zeros((2 * cap, 32), np.uint8)
        n = np.zeros(2, np.int32)
        assert lib().ORBextractor_extract_images(ex._h, lst, 2, 1241, 376, 1300, ptr(kps), ptr(desc), cap, 0,
                                                 ptr(n)) == 0
        for b in range(2):
            ok, od = orc(frames[2 * call + b])
            got = kps[b * cap:b * cap + n[b]]
            assert n[b] == len(ok) and np.array_equal(got.view(np.uint8), ok.view(np.uint8)), f"call {call} image {b}"
            assert np.array_equal(desc[b * cap:b * cap + n[b]], od), f"call {call} image {b}"
    bad = (C.c_void_p * 2)(abig.ctypes.data, None)
    assert lib().ORBextractor_extract_images(ex._h, bad, 2, 1241, 376, 1300, ptr(kps), ptr(desc), cap, 0,
                                             ptr(n)) != 0


def _sparse_image(seed, w=1241, h=376, nrect=12):
    rng = np.random.default_rng(seed)
    img = np.full((h, w), 90, np.uint8)
    for _ in range(nrect):
        x0, y0 = rng.integers(0, w - 60), rng.integers(0, h - 40)
        img[y0:y0 + rng.integers(10, 40), x0:x0 + rng.integers(10, 60)] = rng.integers(150, 255)
    return img


@pytest.mark.parametrize("kind,nf", [("noise", 1200), ("noise", 2000), ("sparse", 1200), ("sparse", 500)])
def test_extract_octree_regimes(gpu, kind, nf):
    """DistributeOctTree regimes on the device octree: pure-noise frames put >40k FAST
    candidates on level 0 (> the LDS key budget -> global-scratch path, phase 2 from the
    first round); sparse frames end phase 1 with every node holding one key."""
    rng = np.random.default_rng(7)
    img = rng.integers(0, 256, (376, 1241), dtype=np.uint8) if kind == "noise" else _sparse_image(7)
    ex = gpu.ORBextractor(nf, 1.2, 8, 20, 7, max_width=1241, max_height=376)
    gk, gd = ex(img)
    ok, od = oracle_lib.OracleExtractor(nf, 1.2, 8, 20, 7)(img)
    assert len(gk) == len(ok) and np.array_equal(gk.view(np.uint8), ok.view(np.uint8)), _diag(gk, gd, ok, od)
    if len(ok):
        assert np.array_equal(gd, od)


@pytest.mark.parametrize("flow", [0, 1])
@pytest.mark.parametrize("B", [3, 12])
def test_pyramid_flow_alternating_batches(gpu, B, flow, monkeypatch):
    """Alternate two different batches (and a smaller one) through one extractor: every padded
    level of every image byte-exact.  flow = 1 builds the pyramid with k_pyr_flow (opt-in
    ORBGPU_PYR_FLOW=1, read when the extractor is created), which hands pyramid rows between
    workgroups of one launch, so a row read before its producer finished would show the previous
    call's bytes.  B = 3 and 12 take the two tile-height variants (16 / 32 rows)."""
    monkeypatch.setenv("ORBGPU_PYR_FLOW", str(flow))
    frames, _ = synthetic.sequence(21, 2 * B, 1241, 376)
    sets = [frames[:B], frames[B:], frames[:B][::-1], frames[B:][: max(1, B // 2)]]
    ex = gpu.ORBextractor(1200, 1.2, 8, 20, 7, max_width=1241, max_height=376, max_batch=B)
    orc = oracle_lib.OracleExtractor(1200, 1.2, 8, 20, 7)
    want = {}
    for imgs in sets:
        ex.extract_batch(np.ascontiguousarray(imgs))
        for b, img in enumerate(imgs):
            key = img.tobytes()[:4096] + bytes([b % 256])
            if key not in want:
                orc(img)
                want[key] = [orc.level(l).copy() for l in range(8)]
            for l in range(8):
                gl = ex.image_pyramid_level(l, b)
                assert np.array_equal(gl, want[key][l]), f"image {b} level {l} differs at {np.argwhere(gl != want[key][l])[:5]}"


def test_extractors_sharing_a_stream(gpu):
    """ORBextractor_share_stream: two extractors launching on one stream (the second one's calls
    queue behind the first one's) keep their own buffers: each batch bit-exact against the oracle,
    and CU reservation (which recreates a stream) is refused on both."""
    from c_orb_slam_amd._lib import lib
    frames, _ = synthetic.sequence(13, 4, 1241, 376)
    a = gpu.ORBextractor(1200, 1.2, 8, 20, 7, max_width=1241, max_height=376, max_batch=2)
    b = gpu.ORBextractor(1200, 1.2, 8, 20, 7, max_width=1241, max_height=376, max_batch=2)
    assert lib().ORBextractor_share_stream(b._h, a._h) == 0
    assert lib().ORBextractor_stream(b._h) == lib().ORBextractor_stream(a._h)
    assert lib().ORBextractor_reserve_cus(b._h, 8) != 0
    assert lib().ORBextractor_reserve_cus(a._h, 8) != 0   # (it would recreate the stream b launches on)
    orc = oracle_lib.OracleExtractor(1200, 1.2, 8, 20, 7)
    for rep in range(2):
        ra = a.extract_batch(frames[:2])
        rb = b.extract_batch(frames[2:])
        for imgs, res in ((frames[:2], ra), (frames[2:], rb)):
            for img, (k, d) in zip(imgs, res):
                ok, od = orc(img)
                assert np.array_equal(k.view(np.uint8), ok.view(np.uint8)), rep
                assert np.array_equal(d, od), rep
    del rb, b   # the borrower goes first (the stream's owner must outlive it)
