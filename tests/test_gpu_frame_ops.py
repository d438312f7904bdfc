"""Frame-level device ops on the tracking path vs the CPU oracle.

* Frame::UnprojectStereo (reference src/Frame.cc:666-680) -- bit-exact x3D and slot indices
  over a batch (empty frame, all-negative depths, random Twc), rows with depth <= 0 untouched.
* Optimizer::PoseOptimization(Frame*) in the frame form (map points as indices into a table,
  keypoints, mvuRight, the mvInvLevelSigma2 table; Optimizer.cc:255-347) -- identical to the
  packed device form and to the oracle (Tcw bits, outlier flags, nInliers)."""
import sys
from pathlib import Path

import numpy as np
import pytest

import oracle_lib
from pose_cases import pose_problem

pytestmark = pytest.mark.gpu

KITTI = (718.856, 718.856, 607.1928, 185.2157)


def _rand_T(rng):
    a = rng.normal(0, 0.3, 3)
    th = np.linalg.norm(a)
    k = a / th
    K = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
    T = np.eye(4)
    T[:3, :3] = np.eye(3) + np.sin(th) * K + (1 - np.cos(th)) * K @ K
    T[:3, 3] = rng.normal(0, 5, 3)
    return T.astype(np.float32)


def _kps(rng, n):
    k = np.zeros(n, oracle_lib.KP_DTYPE)
    k["x"] = rng.uniform(0, 1241, n).astype(np.float32)
    k["y"] = rng.uniform(0, 376, n).astype(np.float32)
    k["octave"] = rng.integers(0, 8, n)
    return k


def test_unproject_stereo_matches_oracle(gpu):
    import torch
    import c_orb_slam_amd as orb
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(5)
    sizes = [1500, 0, 7, 300]
    frames, host = [], []
    for f, n in enumerate(sizes):
        k = _kps(rng, n)
        dep = rng.uniform(-5, 60, n).astype(np.float32)
        if f == 2:
            dep[:] = -1.0
        Twc = _rand_T(rng)
        x3, mp = oracle_lib.oracle_unproject_stereo(k, dep, Twc, *KITTI)
        host.append((x3, mp, dep))
        frames.append(dict(keysUn=torch.from_numpy(k.view(np.int32).reshape(n, 7).copy()).to(dev),
                           depth=torch.from_numpy(dep).to(dev), Twc=torch.from_numpy(Twc.reshape(16)).to(dev),
                           x3D=torch.full((n, 3), 7.0, dtype=torch.float32, device=dev),
                           mp=torch.full((n,), -7, dtype=torch.int32, device=dev), cam=KITTI))
    m = orb.ORBmatcher(0.9, True)
    m.UnprojectStereo_device(frames)
    torch.cuda.synchronize()
    for (x3, mp, dep), fr in zip(host, frames):
        gx = fr["x3D"].cpu().numpy()
        gm = fr["mp"].cpu().numpy()
        assert np.array_equal(gm, mp)
        ok = dep > 0
        assert np.array_equal(gx[ok].view(np.uint32), x3[ok].view(np.uint32))
        assert (gx[~ok] == 7.0).all()


def _octaves(inv_sigma2):
    tab = (np.float32(1.0) / np.float32(1.2) ** (2 * np.arange(8))).astype(np.float32)
    return np.array([int(np.flatnonzero(tab == v)[0]) for v in inv_sigma2], np.int32), tab


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_pose_frames_form_equals_packed_and_oracle(gpu, seed):
    import torch
    from c_orb_slam_amd.optimizer import PoseOptimizationBatchDevice, PoseOptimizationFramesDevice
    dev = torch.device("cuda", 0)
    frames = [pose_problem(100 * seed + s, N=400 + 500 * s) for s in range(3)]
    packed, framed = [], []
    for fr in frames:
        N = len(fr["has_mp"])
        octv, tab = _octaves(fr["inv_sigma2"])
        k = np.zeros(N, oracle_lib.KP_DTYPE)
        k["x"], k["y"], k["octave"] = fr["obs"][:, 0], fr["obs"][:, 1], octv
        # map point table in a shuffled order: the frame form gathers rows by index
        perm = np.random.default_rng(seed).permutation(N)
        table = np.zeros((N, 3), np.float32)
        table[perm] = fr["Xw"]
        mp = np.where(fr["has_mp"] > 0, perm, -1).astype(np.int32)
        T = torch.from_numpy(np.ascontiguousarray(fr["Tcw"], np.float32).reshape(16)).to(dev)
        packed.append(dict(Tcw=T, has_mp=torch.from_numpy(fr["has_mp"]).to(dev), Xw=torch.from_numpy(fr["Xw"]).to(dev),
                           obs=torch.from_numpy(fr["obs"]).to(dev), inv_sigma2=torch.from_numpy(fr["inv_sigma2"]).to(dev),
                           cam=fr["cam"]))
        framed.append(dict(Tcw=T, mp=torch.from_numpy(mp).to(dev), mp_pos=torch.from_numpy(table).to(dev),
                           keysUn=torch.from_numpy(k.view(np.int32).reshape(N, 7).copy()).to(dev),
                           uRight=torch.from_numpy(np.ascontiguousarray(fr["obs"][:, 2])).to(dev),
                           invLevelSigma2=torch.from_numpy(tab).to(dev), cam=fr["cam"]))
    Tp = [torch.zeros(16, dtype=torch.float32, device=dev) for _ in frames]
    Tf = [torch.zeros(16, dtype=torch.float32, device=dev) for _ in frames]
    op = [torch.full((len(f["has_mp"]),), 9, dtype=torch.uint8, device=dev) for f in frames]
    of = [torch.full((len(f["has_mp"]),), 9, dtype=torch.uint8, device=dev) for f in frames]
    n_p = PoseOptimizationBatchDevice(packed, Tp, op)
    n_f = PoseOptimizationFramesDevice(framed, Tf, of)
    assert np.array_equal(n_p, n_f)
    for f, fr in enumerate(frames):
        assert np.array_equal(Tp[f].cpu().numpy(), Tf[f].cpu().numpy())
        assert np.array_equal(op[f].cpu().numpy(), of[f].cpu().numpy())
        o = oracle_lib.oracle_pose_optimization(fr)
        assert int(n_f[f]) == int(o["inliers"])
        assert np.array_equal(Tf[f].cpu().numpy().reshape(4, 4), o["Tcw"])


def test_deferred_chain_equals_synchronous(gpu):
    """ORBmatcher_set_deferred: two PoseOptimization batches queued on the matcher's stream
    without a host sync in between give the synchronous call's poses, outliers and counts, and
    the counts land only at ORBmatcher_finish."""
    import torch
    from c_orb_slam_amd._lib import check, lib
    from c_orb_slam_amd.optimizer import PoseOptimizationFramesDevice
    dev = torch.device("cuda", 0)
    frames = [pose_problem(700 + s, N=300 + 400 * s) for s in range(3)]
    framed = []
    for fr in frames:
        N = len(fr["has_mp"])
        octv, tab = _octaves(fr["inv_sigma2"])
        k = np.zeros(N, oracle_lib.KP_DTYPE)
        k["x"], k["y"], k["octave"] = fr["obs"][:, 0], fr["obs"][:, 1], octv
        mp = np.where(fr["has_mp"] > 0, np.arange(N), -1).astype(np.int32)
        framed.append(dict(Tcw=torch.from_numpy(np.ascontiguousarray(fr["Tcw"], np.float32).reshape(16)).to(dev),
                           mp=torch.from_numpy(mp).to(dev), mp_pos=torch.from_numpy(fr["Xw"]).to(dev),
                           keysUn=torch.from_numpy(k.view(np.int32).reshape(N, 7).copy()).to(dev),
                           uRight=torch.from_numpy(np.ascontiguousarray(fr["obs"][:, 2])).to(dev),
                           invLevelSigma2=torch.from_numpy(tab).to(dev), cam=fr["cam"]))
    mk = lambda fill: [torch.full((len(f["has_mp"]),), fill, dtype=torch.uint8, device=dev) for f in frames]
    T0 = [torch.zeros(16, dtype=torch.float32, device=dev) for _ in frames]
    o0 = mk(9)
    n0 = PoseOptimizationFramesDevice(framed, T0, o0)
    m = gpu.ORBmatcher(0.8, False)
    L = lib()
    check(L.ORBmatcher_set_device_pointers(m._h, 1))
    T1 = [torch.zeros(16, dtype=torch.float32, device=dev) for _ in frames]
    T2 = [torch.zeros(16, dtype=torch.float32, device=dev) for _ in frames]
    o1, o2 = mk(9), mk(9)   # entries of keypoints without a map point keep the caller's value
    n1, n2 = np.full(3, -9, np.int32), np.full(3, -9, np.int32)
    check(L.ORBmatcher_set_deferred(m._h, 1))
    PoseOptimizationFramesDevice(framed, T1, o1, chain=m, n_out=n1)
    PoseOptimizationFramesDevice(framed, T2, o2, chain=m, n_out=n2)
    assert (n1 == -9).all() and (n2 == -9).all()      # nothing lands before finish
    check(L.ORBmatcher_finish(m._h))
    # overlapping chains: close one epoch, queue the next behind it, wait for the first from
    # another host thread (device work only), then finish them in order
    import ctypes as C
    import threading
    T3 = [torch.zeros(16, dtype=torch.float32, device=dev) for _ in frames]
    T4 = [torch.zeros(16, dtype=torch.float32, device=dev) for _ in frames]
    o3, o4 = mk(9), mk(9)
    n3, n4 = np.full(3, -9, np.int32), np.full(3, -9, np.int32)
    e3, e4 = C.c_longlong(0), C.c_longlong(0)
    PoseOptimizationFramesDevice(framed, T3, o3, chain=m, n_out=n3)
    check(L.ORBmatcher_chain_close(m._h, C.byref(e3)))
    PoseOptimizationFramesDevice(framed, T4, o4, chain=m, n_out=n4)
    check(L.ORBmatcher_chain_close(m._h, C.byref(e4)))
    assert e4.value == e3.value + 1
    th = threading.Thread(target=lambda: check(L.ORBmatcher_chain_wait(m._h, e3.value)))
    th.start()
    th.join()
    assert (n3 == -9).all()                           # waiting writes nothing
    check(L.ORBmatcher_chain_finish(m._h, e3.value))
    assert np.array_equal(n3, n0) and (n4 == -9).all()
    check(L.ORBmatcher_chain_finish(m._h, e4.value))
    assert np.array_equal(n4, n0)
    check(L.ORBmatcher_set_deferred(m._h, 0))
    for f in range(3):
        assert np.array_equal(T3[f].cpu().numpy(), T0[f].cpu().numpy())
        assert np.array_equal(T4[f].cpu().numpy(), T0[f].cpu().numpy())
    for n, T, o in ((n1, T1, o1), (n2, T2, o2)):
        assert np.array_equal(n, n0)
        for f in range(3):
            assert np.array_equal(T[f].cpu().numpy(), T0[f].cpu().numpy())
            assert np.array_equal(o[f].cpu().numpy(), o0[f].cpu().numpy())


def test_deferred_and_synchronous_pose_interleaved(gpu):
    """The pose engine's device arena is shared by every PoseOptimization call of a host thread.
    A deferred batch still queued on one matcher's stream, then a synchronous batch (larger, so
    the arena grows), then a deferred batch on a second matcher: each must give its own
    standalone result (the arena's next user waits for the queued kernels that read it)."""
    import torch
    from c_orb_slam_amd._lib import check, lib
    from c_orb_slam_amd.optimizer import PoseOptimizationFramesDevice
    dev = torch.device("cuda", 0)

    def framed_of(seeds, base_n):
        out = []
        for i, s in enumerate(seeds):
            fr = pose_problem(s, N=base_n + 350 * i)
            N = len(fr["has_mp"])
            octv, tab = _octaves(fr["inv_sigma2"])
            k = np.zeros(N, oracle_lib.KP_DTYPE)
            k["x"], k["y"], k["octave"] = fr["obs"][:, 0], fr["obs"][:, 1], octv
            mp = np.where(fr["has_mp"] > 0, np.arange(N), -1).astype(np.int32)
            out.append(dict(Tcw=torch.from_numpy(np.ascontiguousarray(fr["Tcw"], np.float32).reshape(16)).to(dev),
                            mp=torch.from_numpy(mp).to(dev), mp_pos=torch.from_numpy(fr["Xw"]).to(dev),
                            keysUn=torch.from_numpy(k.view(np.int32).reshape(N, 7).copy()).to(dev),
                            uRight=torch.from_numpy(np.ascontiguousarray(fr["obs"][:, 2])).to(dev),
                            invLevelSigma2=torch.from_numpy(tab).to(dev), cam=fr["cam"]))
        return out

    A = framed_of([910, 911], 300)
    B = framed_of([920, 921, 922, 923, 924, 925], 900)     # more edges than A: the arena grows
    Cf = framed_of([930, 931, 932], 500)
    outs = lambda fs: ([torch.zeros(16, dtype=torch.float32, device=dev) for _ in fs],
                       [torch.full((f["mp"].numel(),), 9, dtype=torch.uint8, device=dev) for f in fs])
    ref = {}
    for name, fs in (("A", A), ("B", B), ("C", Cf)):
        T, o = outs(fs)
        n = PoseOptimizationFramesDevice(fs, T, o)
        ref[name] = (n, [t.cpu().numpy() for t in T], [x.cpu().numpy() for x in o])
    L = lib()
    m1, m2 = gpu.ORBmatcher(0.8, False), gpu.ORBmatcher(0.8, False)
    for m in (m1, m2):
        check(L.ORBmatcher_set_device_pointers(m._h, 1))
        check(L.ORBmatcher_set_deferred(m._h, 1))
    TA, oA = outs(A)
    nA = np.full(len(A), -9, np.int32)
    PoseOptimizationFramesDevice(A, TA, oA, chain=m1, n_out=nA)        # queued, not finished
    TB, oB = outs(B)
    nB = PoseOptimizationFramesDevice(B, TB, oB)                        # synchronous, own stream
    TC, oC = outs(Cf)
    nC = np.full(len(Cf), -9, np.int32)
    PoseOptimizationFramesDevice(Cf, TC, oC, chain=m2, n_out=nC)       # another matcher's stream
    check(L.ORBmatcher_finish(m2._h))
    check(L.ORBmatcher_finish(m1._h))
    for m in (m1, m2):
        check(L.ORBmatcher_set_deferred(m._h, 0))
    for name, n, T, o in (("A", nA, TA, oA), ("B", nB, TB, oB), ("C", nC, TC, oC)):
        rn, rT, ro = ref[name]
        assert np.array_equal(np.asarray(n), np.asarray(rn)), name
        for f in range(len(T)):
            assert np.array_equal(T[f].cpu().numpy(), rT[f]), (name, f)
            assert np.array_equal(o[f].cpu().numpy(), ro[f]), (name, f)


@pytest.mark.parametrize("seed", [3, 4])
def test_pose_output_in_pinned_host_memory_visible_on_return(gpu, seed):
    """Optimizer_PoseOptimization_frames_device with Tcw_out in pinned host memory (torch's default,
    non-coherent pinned pages, and coherent ones): the pose the host reads the moment the call
    returns (the library's polled stream drain) equals the same call's device-buffer output read
    after a blocking device synchronisation, and the oracle's pose (bench.py's latency leg reads
    its final pose this way)."""
    import torch
    from c_orb_slam_amd.optimizer import PoseOptimizationFramesDevice
    sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
    from bench import _coherent_host_f32
    dev = torch.device("cuda", 0)
    frames = [pose_problem(900 + 10 * seed + s, N=350 + 300 * s) for s in range(4)]
    framed = []
    for fr in frames:
        N = len(fr["has_mp"])
        octv, tab = _octaves(fr["inv_sigma2"])
        k = np.zeros(N, oracle_lib.KP_DTYPE)
        k["x"], k["y"], k["octave"] = fr["obs"][:, 0], fr["obs"][:, 1], octv
        mp = np.where(fr["has_mp"] > 0, np.arange(N), -1).astype(np.int32)
        framed.append(dict(Tcw=torch.from_numpy(np.ascontiguousarray(fr["Tcw"], np.float32).reshape(16)).to(dev),
                           mp=torch.from_numpy(mp).to(dev), mp_pos=torch.from_numpy(fr["Xw"]).to(dev),
                           keysUn=torch.from_numpy(k.view(np.int32).reshape(N, 7).copy()).to(dev),
                           uRight=torch.from_numpy(np.ascontiguousarray(fr["obs"][:, 2])).to(dev),
                           invLevelSigma2=torch.from_numpy(tab).to(dev), cam=fr["cam"]))
    outl = lambda: [torch.zeros(len(f["has_mp"]), dtype=torch.uint8, device=dev) for f in frames]
    Td = [torch.zeros(16, dtype=torch.float32, device=dev) for _ in frames]
    PoseOptimizationFramesDevice(framed, Td, outl())
    torch.cuda.synchronize()
    ref = [t.cpu().numpy().copy() for t in Td]
    for alloc in ("pinned", "coherent"):
        for rep in range(3):
            Th = [(torch.full((16,), -7.0, dtype=torch.float32).pin_memory() if alloc == "pinned"
                   else _coherent_host_f32(16).fill_(-7.0)) for _ in frames]
            PoseOptimizationFramesDevice(framed, Th, outl())
            got = [t.numpy().copy() for t in Th]   # no synchronisation after the call
            for f, fr in enumerate(frames):
                assert np.array_equal(got[f], ref[f]), (alloc, rep, f)
                o = oracle_lib.oracle_pose_optimization(fr)
                assert np.array_equal(got[f].reshape(4, 4), o["Tcw"])
