"""Frame::ComputeStereoMatches (reference src/Frame.cc:466-640) on the GPU vs the CPU oracle.

Bit-exact: mvuRight / mvDepth floats and the kept-match count, on synthetic rectified pairs
(per-rectangle integer disparities 0..64) at KITTI and EuRoC sizes;
batched == single; edge cases (no right keypoints, identical images -> the disparity <= 0
branch, tiny images).  The pyramids come from the GPU extractors of the same images, which
are bit-exact with the oracle extractors (test_gpu_extract.py)."""
import numpy as np
import pytest

import oracle_lib
from c_orb_slam_amd import synthetic

pytestmark = pytest.mark.gpu

KITTI_BF, KITTI_FX = 386.1448, 718.856


def _pair(gpu, left, right, nfeat=1200, mbf=KITTI_BF, fx=KITTI_FX):
    h, w = left.shape
    exL = gpu.ORBextractor(nfeat, 1.2, 8, 20, 7, max_width=w, max_height=h)
    exR = gpu.ORBextractor(nfeat, 1.2, 8, 20, 7, max_width=w, max_height=h)
    kL, dL = exL(left)
    kR, dR = exR(right)
    m = gpu.ORBmatcher(0.6, True)
    mb = np.float32(np.float32(mbf) / np.float32(fx))
    uR, dep, n = m.ComputeStereoMatches(exL, exR, kL, dL, kR, dR, mbf, mb)
    oL, oR = oracle_lib.OracleExtractor(nfeat, 1.2, 8, 20, 7), oracle_lib.OracleExtractor(nfeat, 1.2, 8, 20, 7)
    okL, odL = oL(left)
    okR, odR = oR(right)
    assert np.array_equal(okL.view(np.uint8), kL.view(np.uint8)) and np.array_equal(okR.view(np.uint8), kR.view(np.uint8))
    ouR, odep, on = oracle_lib.oracle_stereo_matches(oL, oR, kL, dL, kR, dR, h, mbf, mb)
    return (uR, dep, n), (ouR, odep, on), (kL, kR)


@pytest.mark.parametrize("seed,w,h", [(0, 1241, 376), (1, 1241, 376), (2, 752, 480), (3, 640, 480)])
def test_stereo_bit_exact(gpu, seed, w, h):
    L, R = synthetic.stereo_batch(seed, 1, w, h)
    (uR, dep, n), (ouR, odep, on), (kL, _) = _pair(gpu, L[0], R[0])
    assert n == on
    assert np.array_equal(uR.view(np.uint32), ouR.view(np.uint32))
    assert np.array_equal(dep.view(np.uint32), odep.view(np.uint32))
    assert n > 50, n
    # sanity: the recovered disparities are the synthetic ones (integers 0..64)
    ok = uR >= 0
    d = kL["x"][ok] - uR[ok]
    assert np.median(d) > 0 and np.percentile(d, 90) < 70


def test_stereo_identical_images_zero_disparity(gpu):
    L, _ = synthetic.stereo_batch(5, 1, 640, 480)
    (uR, dep, n), (ouR, odep, on), _ = _pair(gpu, L[0], L[0])
    assert n == on and np.array_equal(uR.view(np.uint32), ouR.view(np.uint32))
    assert np.array_equal(dep.view(np.uint32), odep.view(np.uint32))


def test_stereo_no_right_keypoints(gpu):
    L, _ = synthetic.stereo_batch(6, 1, 640, 480)
    flat = np.full_like(L[0], 128)
    (uR, dep, n), (ouR, odep, on), _ = _pair(gpu, L[0], flat)
    assert n == on == 0 and (uR == -1).all() and (dep == -1).all()


def test_stereo_batch_matches_single(gpu):
    Ls, Rs = synthetic.stereo_batch(9, 3, 752, 480)
    exL = gpu.ORBextractor(1200, 1.2, 8, 20, 7, max_width=752, max_height=480, max_batch=3)
    exR = gpu.ORBextractor(1200, 1.2, 8, 20, 7, max_width=752, max_height=480, max_batch=3)
    kdL = exL.extract_batch(Ls)
    kdR = exR.extract_batch(Rs)
    m = gpu.ORBmatcher(0.6, True)
    mbf, mb = 47.9064, np.float32(47.9064 / 435.2047)
    uRs, deps, ns = m.ComputeStereoMatches_batch(exL, exR, [k for k, _ in kdL], [d for _, d in kdL],
                                                 [k for k, _ in kdR], [d for _, d in kdR], mbf, mb)
    for b in range(3):
        e1 = gpu.ORBextractor(1200, 1.2, 8, 20, 7, max_width=752, max_height=480)
        e2 = gpu.ORBextractor(1200, 1.2, 8, 20, 7, max_width=752, max_height=480)
        kL, dL = e1(Ls[b])
        kR, dR = e2(Rs[b])
        uR, dep, n = m.ComputeStereoMatches(e1, e2, kL, dL, kR, dR, mbf, mb)
        assert n == ns[b]
        assert np.array_equal(uR.view(np.uint32), uRs[b].view(np.uint32))
        assert np.array_equal(dep.view(np.uint32), deps[b].view(np.uint32))


def test_stereo_one_extractor_batch(gpu):
    """Frame(imLeft, imRight)'s two extractions as ONE batch call over [lefts..., rights...] on one
    extractor (the bench's --stereo-batch pipeline): ComputeStereoMatches_batch_at pairs image b
    with image P + b, and every pair is bit-identical to the two-extractor batch."""
    P = 3
    Ls, Rs = synthetic.stereo_batch(11, P, 1241, 376)
    one = gpu.ORBextractor(1200, 1.2, 8, 20, 7, max_width=1241, max_height=376, max_batch=2 * P)
    kd = one.extract_batch(np.concatenate([Ls, Rs]))
    exL = gpu.ORBextractor(1200, 1.2, 8, 20, 7, max_width=1241, max_height=376, max_batch=P)
    exR = gpu.ORBextractor(1200, 1.2, 8, 20, 7, max_width=1241, max_height=376, max_batch=P)
    kdL = exL.extract_batch(Ls)
    kdR = exR.extract_batch(Rs)
    for b in range(P):   # the extractions themselves are per-image bit-exact
        assert np.array_equal(kd[b][0].view(np.uint8), kdL[b][0].view(np.uint8))
        assert np.array_equal(kd[P + b][1], kdR[b][1])
    m = gpu.ORBmatcher(0.6, True)
    mb = np.float32(np.float32(KITTI_BF) / np.float32(KITTI_FX))
    args = lambda kl, kr: ([k for k, _ in kl], [d for _, d in kl], [k for k, _ in kr], [d for _, d in kr], KITTI_BF, mb)
    u1, d1, n1 = m.ComputeStereoMatches_batch(one, one, *args(kd[:P], kd[P:]), first_left=0, first_right=P)
    u2, d2, n2 = m.ComputeStereoMatches_batch(exL, exR, *args(kdL, kdR))
    assert np.array_equal(n1, n2) and n1.min() > 50
    for b in range(P):
        assert np.array_equal(u1[b].view(np.uint32), u2[b].view(np.uint32))
        assert np.array_equal(d1[b].view(np.uint32), d2[b].view(np.uint32))
