"""Host mirror of ORB_SLAM2::Optimizer (LocalBundleAdjustment, BundleAdjustment) over the C ABI.

LocalBundleAdjustment(...) takes the arrays the reference gathers from the
covisibility graph (Optimizer.cc:456-653, see include/orbslam_gpu.h ba_problem)
and returns what it writes back: keyframe poses, map point positions and the
(keyframe, map point) observations to erase.  BundleAdjustment(...) is
Optimizer::BundleAdjustment (Optimizer.cc:49-237, GlobalBundleAdjustemnt's body).

Keyframe-block sharding across GPUs: partition_points() assigns
every map point to the rank owning its reference keyframe's block,
shard_problem() cuts a rank's shard (all keyframes, own points and their
edges), the *_sharded calls run the LM with one all-reduce of the partial
Schur complement per trial (RCCL across processes, or an in-process group of
threads on one device), and merge_shards() reassembles the full result.
"""
import ctypes as C
import threading

import numpy as np

from ._lib import ba_problem, ba_result, check, lib, pose_problem, ptr, sim3opt_problem

_FIELDS = (("kf_id", np.int32), ("kf_Tcw", np.float32), ("kf_local", np.uint8), ("kf_cam", np.float32),
           ("pt_id", np.int32), ("pt_pos", np.float32), ("edge_pt", np.int32), ("edge_kf", np.int32),
           ("edge_obs", np.float32), ("edge_inv_sigma2", np.float32))
FIELDS = tuple(n for n, _ in _FIELDS)


class _Packed:
    """Contiguous copies of a problem + its ba_problem/ba_result structs (kept alive together)."""

    def __init__(self, arrays):
        a = {}
        for (name, dt), v in zip(_FIELDS, arrays):
            a[name] = np.ascontiguousarray(v, dt)
        self.a = a
        self.nkf, self.npt, self.ne = len(a["kf_id"]), len(a["pt_id"]), len(a["edge_pt"])
        self.P = ba_problem(self.nkf, ptr(a["kf_id"]), ptr(a["kf_Tcw"]), ptr(a["kf_local"]), ptr(a["kf_cam"]),
                            self.npt, ptr(a["pt_id"]), ptr(a["pt_pos"]), self.ne, ptr(a["edge_pt"]),
                            ptr(a["edge_kf"]), ptr(a["edge_obs"]), ptr(a["edge_inv_sigma2"]))
        self.T = np.zeros((self.nkf, 16), np.float32)
        self.X = np.zeros((self.npt, 3), np.float32)
        self.er = np.zeros(max(self.ne, 1), np.uint8)
        self.R = ba_result(ptr(self.T), ptr(self.X), ptr(self.er))

    def result(self, trace):
        R = self.R
        out = dict(kf_Tcw=self.T, pt_pos=self.X, edge_erase=self.er[:self.ne].astype(bool),
                   iterations=tuple(R.iterations), n_erased=R.n_erased, aborted=bool(R.aborted))
        if trace:
            out.update(last_trace())
        return out


def _args(problem):
    return [problem[k] for k in FIELDS]


def last_trace():
    """LM trace of the calling thread's last run (per solve: initial/final chi2; per trial: chi2, lambda)."""
    cap = 4096
    si, sc, tc, tl = (np.zeros(cap) for _ in range(4))
    ns, nt = C.c_int(), C.c_int()
    check(lib().Optimizer_last_trace(ptr(si), ptr(sc), cap, C.byref(ns), ptr(tc), ptr(tl), cap, C.byref(nt)))
    return dict(solve_ini_chi2=si[:ns.value], solve_chi2=sc[:ns.value], trial_chi2=tc[:nt.value],
                trial_lambda=tl[:nt.value])


def _stop_ref(stop):
    return C.byref(stop) if stop is not None else None


def LocalBundleAdjustment(kf_id, kf_Tcw, kf_local, kf_cam, pt_id, pt_pos, edge_pt, edge_kf, edge_obs, edge_inv_sigma2,
                          stop=None, trace=False):
    """-> dict(kf_Tcw, pt_pos, edge_erase, iterations, n_erased, aborted[, trace])

    stop: optional ctypes.c_bool shared with another thread (pbStopFlag)."""
    k = _Packed((kf_id, kf_Tcw, kf_local, kf_cam, pt_id, pt_pos, edge_pt, edge_kf, edge_obs, edge_inv_sigma2))
    check(lib().Optimizer_LocalBundleAdjustment(C.byref(k.P), _stop_ref(stop), C.byref(k.R)),
          "Optimizer_LocalBundleAdjustment")
    return k.result(trace)


def BundleAdjustment(problem, nIterations=10, bRobust=False, stop=None, trace=False):
    """Optimizer::BundleAdjustment(vpKFs, vpMP, nIterations, pbStopFlag, nLoopKF, bRobust) (Optimizer.cc:49).
    LoopClosing runs it with nIterations=10, bRobust=false (LoopClosing.cc:650)."""
    k = _Packed(_args(problem))
    check(lib().Optimizer_BundleAdjustment(C.byref(k.P), int(nIterations), int(bool(bRobust)), _stop_ref(stop),
                                           C.byref(k.R)), "Optimizer_BundleAdjustment")
    return k.result(trace)


def last_timings():
    ms = np.zeros(2)
    check(lib().Optimizer_last_timings(ptr(ms)))
    return ms


# ------------------------------------------------------------------ OptimizeSim3
_SIM3OPT = (("valid", np.uint8), ("X1c", np.float32), ("X2c", np.float32), ("obs1", np.float32),
            ("obs2", np.float32), ("inv_sigma2_1", np.float32), ("inv_sigma2_2", np.float32))


def _sim3opt_struct(pr, keep):
    a = {k: np.ascontiguousarray(pr[k], dt) for k, dt in _SIM3OPT}
    keep.append(a)
    N = len(a["valid"])
    if (a["X1c"].shape != (N, 3) or a["X2c"].shape != (N, 3) or a["obs1"].shape != (N, 2)
            or a["obs2"].shape != (N, 2) or a["inv_sigma2_1"].shape != (N,) or a["inv_sigma2_2"].shape != (N,)):
        raise ValueError("OptimizeSim3: inconsistent correspondence arrays")
    P = sim3opt_problem()
    P.N = N
    for k, _ in _SIM3OPT:
        setattr(P, k, ptr(a[k]))
    P.K1 = (C.c_float * 4)(*[float(v) for v in pr["K1"]])
    P.K2 = (C.c_float * 4)(*[float(v) for v in pr["K2"]])
    P.th2 = float(pr.get("th2", 10.0))
    P.bFixScale = int(bool(pr["bFixScale"]))
    return P


def OptimizeSim3(problem, S12):
    """Optimizer::OptimizeSim3(pKF1, pKF2, vpMatches1, g2oS12, th2, bFixScale) (Optimizer.cc:1046-1241).

    problem: dict with valid (N), X1c / X2c (N x 3 camera-frame points), obs1 / obs2 (N x 2 undistorted
    keypoints), inv_sigma2_1 / inv_sigma2_2 (N), K1 / K2 (fx fy cx cy), th2, bFixScale.
    S12: g2o::Sim3 as 8 doubles (quaternion x y z w, t, s).
    -> (nIn, S12 out, erased mask: vpMatches1[i] set to NULL)."""
    n, S, e = OptimizeSim3Batch([problem], [S12])
    return int(n[0]), S[0], e[0]


def OptimizeSim3Batch(problems, S12s):
    """One launch for many loop candidates (one workgroup each) -> (nIn[C], S12[C, 8], [erased_c])."""
    keep = []
    F = len(problems)
    probs = (sim3opt_problem * max(F, 1))(*[_sim3opt_struct(p, keep) for p in problems])
    S = np.zeros((max(F, 1), 8), np.float64)
    for i, s in enumerate(S12s):
        S[i] = np.asarray(s, np.float64).reshape(8)
    er = [np.zeros(max(len(k["valid"]), 1), np.uint8) for k in keep]
    eptr = (C.c_void_p * max(F, 1))(*[e.ctypes.data for e in er])
    n = np.zeros(max(F, 1), np.int32)
    check(lib().Optimizer_OptimizeSim3_batch(F, probs, ptr(S), eptr, ptr(n)), "Optimizer_OptimizeSim3")
    return n[:F], S[:F], [e[:len(k["valid"])].astype(bool) for e, k in zip(er, keep)]


# ------------------------------------------------------------------ PoseOptimization
_POSE = (("Tcw", np.float32), ("has_mp", np.uint8), ("Xw", np.float32), ("obs", np.float32),
         ("inv_sigma2", np.float32))


def _pose_struct(frame, keep):
    a = {k: np.ascontiguousarray(frame[k], dt) for k, dt in _POSE}
    keep.append(a)
    N = len(a["has_mp"])
    if a["Tcw"].size != 16 or a["Xw"].shape != (N, 3) or a["obs"].shape != (N, 3) or a["inv_sigma2"].shape != (N,):
        raise ValueError("PoseOptimization: inconsistent frame arrays")
    fx, fy, cx, cy, bf = (float(v) for v in frame["cam"])
    return pose_problem(N, ptr(a["Tcw"]), ptr(a["has_mp"]), ptr(a["Xw"]), ptr(a["obs"]), ptr(a["inv_sigma2"]),
                        fx, fy, cx, cy, bf)


def PoseOptimization(frame, outlier=None):
    """Optimizer::PoseOptimization(Frame*) (Optimizer.cc:239-451).

    frame: dict with Tcw (4x4), has_mp (N), Xw (N x 3), obs (N x 3: kpUn.x, kpUn.y, mvuRight),
    inv_sigma2 (N), cam (fx, fy, cx, cy, mbf).  outlier: mvbOutlier (N, in/out; rows without
    a map point are left as given).  -> (nInliers, Tcw 4x4, outlier)."""
    n, T, o = PoseOptimizationBatch([frame], None if outlier is None else [outlier])
    return int(n[0]), T[0], o[0]


def PoseOptimizationBatch(frames, outliers=None):
    """One launch for many frames (one workgroup per frame) -> (nInliers[F], Tcw[F,4,4], [outlier_f])."""
    keep = []
    F = len(frames)
    probs = (pose_problem * max(F, 1))(*[_pose_struct(f, keep) for f in frames])
    outs = [np.ascontiguousarray(outliers[i] if outliers is not None else np.zeros(len(keep[i]["has_mp"])),
                                 np.uint8).copy() for i in range(F)]
    optr = (C.c_void_p * max(F, 1))(*[o.ctypes.data for o in outs])
    T = np.zeros((max(F, 1), 16), np.float32)
    n = np.zeros(max(F, 1), np.int32)
    check(lib().Optimizer_PoseOptimization_batch(F, probs, ptr(T), optr, ptr(n)), "Optimizer_PoseOptimization")
    return n[:F], T[:F].reshape(F, 4, 4), outs


def PoseOptimizationBatchDevice(frames, Tcw_out, outliers):
    """Device-resident batch: frames[f] holds torch device tensors Tcw (16 f32), has_mp (N u8),
    Xw (N x 3 f32), obs (N x 3 f32), inv_sigma2 (N f32) and cam (5 floats, host); Tcw_out[f]
    (16 f32) and outliers[f] (N u8, in/out) are device tensors.  -> nInliers[F] (host)."""
    F = len(frames)
    ps = []
    for f in frames:
        for k, dt in _POSE:
            t = f[k]
            if not t.is_contiguous() or t.element_size() != np.dtype(dt).itemsize:
                raise ValueError(f"PoseOptimizationBatchDevice: {k} must be contiguous {np.dtype(dt).name}")
        fx, fy, cx, cy, bf = (float(v) for v in f["cam"])
        ps.append(pose_problem(int(f["has_mp"].numel()), f["Tcw"].data_ptr(), f["has_mp"].data_ptr(),
                               f["Xw"].data_ptr(), f["obs"].data_ptr(), f["inv_sigma2"].data_ptr(),
                               fx, fy, cx, cy, bf))
    probs = (pose_problem * max(F, 1))(*ps)
    tptr = (C.c_void_p * max(F, 1))(*[t.data_ptr() for t in Tcw_out])
    optr = (C.c_void_p * max(F, 1))(*[o.data_ptr() for o in outliers])
    n = np.zeros(max(F, 1), np.int32)
    check(lib().Optimizer_PoseOptimization_batch_device(F, probs, tptr, optr, ptr(n)),
          "Optimizer_PoseOptimization_batch_device")
    return n[:F]


def PoseOptimizationFramesDevice(frames, Tcw_out, outliers, chain=None, n_out=None):
    """Optimizer::PoseOptimization(Frame*) on device-resident frames as the reference reads them
    (Optimizer.cc:255-347): frames[f] holds torch device tensors Tcw (16 f32), mp (N i32 indices
    into mp_pos, -1 = NULL), mp_pos (M x 3 f32), keysUn (N x 7 words, cv::KeyPoint layout),
    uRight (N f32), invLevelSigma2 (nlevels f32) and cam (5 floats, host).  -> nInliers[F].
    chain: an ORBmatcher in deferred mode (ORBmatcher_set_deferred): the call is queued on its
    stream and n_out (int32 numpy, F) is written by ORBmatcher_finish."""
    from ._lib import pose_frame
    F = len(frames)
    ps = []
    for f in frames:
        for k in ("Tcw", "mp", "mp_pos", "keysUn", "uRight", "invLevelSigma2"):
            if not f[k].is_contiguous() or f[k].element_size() != 4:
                raise ValueError(f"PoseOptimizationFramesDevice: {k} must be contiguous 4-byte elements")
        fx, fy, cx, cy, bf = (float(v) for v in f["cam"])
        ps.append(pose_frame(int(f["mp"].numel()), f["Tcw"].data_ptr(), f["mp"].data_ptr(), f["mp_pos"].data_ptr(),
                             f["keysUn"].data_ptr(), f["uRight"].data_ptr(), f["invLevelSigma2"].data_ptr(),
                             int(f["invLevelSigma2"].numel()), fx, fy, cx, cy, bf))
    probs = (pose_frame * max(F, 1))(*ps)
    tptr = (C.c_void_p * max(F, 1))(*[t.data_ptr() for t in Tcw_out])
    optr = (C.c_void_p * max(F, 1))(*[o.data_ptr() for o in outliers])
    if chain is not None:
        check(lib().Optimizer_PoseOptimization_frames_device_deferred(chain._h, F, probs, tptr, optr, ptr(n_out)),
              "Optimizer_PoseOptimization_frames_device_deferred")
        return n_out
    n = np.zeros(max(F, 1), np.int32)
    check(lib().Optimizer_PoseOptimization_frames_device(F, probs, tptr, optr, ptr(n)),
          "Optimizer_PoseOptimization_frames_device")
    return n[:F]


# ------------------------------------------------------------------ sharding
def partition_points(problem, nranks):
    """pt_rank[p]: keyframe-block owner of every map point (Optimizer_partition_points, host only)."""
    k = _Packed(_args(problem))
    out = np.zeros(max(k.npt, 1), np.int32)
    check(lib().Optimizer_partition_points(C.byref(k.P), int(nranks), ptr(out)), "Optimizer_partition_points")
    return out[:k.npt]


def partition_points_nd(problem, nranks, with_kf_owner=False):
    """pt_rank[p] for the sharded factorisation of a global BA: whole subtrees of the pose
    graph's nested dissection per rank, a point with the rank of the first subtree pose it
    observes (Optimizer_partition_points_nd, host only).  with_kf_owner: also the rank of each
    keyframe's subtree (-1 separator, -2 no free pose)."""
    k = _Packed(_args(problem))
    out = np.zeros(max(k.npt, 1), np.int32)
    kfo = np.zeros(max(len(problem["kf_id"]), 1), np.int32)
    check(lib().Optimizer_partition_points_nd(C.byref(k.P), int(nranks), ptr(out), ptr(kfo)),
          "Optimizer_partition_points_nd")
    return (out[:k.npt], kfo[:len(problem["kf_id"])]) if with_kf_owner else out[:k.npt]


def last_lm_path():
    """The calling thread's last BA run: steps of the device-resident LM, trials the host loop decided
    after a readback, and whether it was sharded (Optimizer_last_lm_path)."""
    v = np.zeros(4, np.int32)
    check(lib().Optimizer_last_lm_path(ptr(v)), "Optimizer_last_lm_path")
    return dict(device_steps=int(v[0]), host_trials=int(v[1]), sharded=bool(v[2]))


def last_sharding():
    """The calling thread's last BA run: (sharded factorisation used, separator tiles exchanged
    per trial, separator rows, Schur-pattern tiles the replicated path would all-reduce)."""
    v = np.zeros(4, np.int32)
    check(lib().Optimizer_last_sharding(ptr(v)), "Optimizer_last_sharding")
    return tuple(int(x) for x in v)


def shard_problem(problem, pt_rank, rank):
    """Rank `rank`'s shard: every keyframe, its own points and all of their edges, in the original
    (reference creation) order.  Adds pt_index / edge_index: positions in the full problem."""
    pts = np.flatnonzero(np.asarray(pt_rank) == rank).astype(np.int64)
    remap = np.full(len(problem["pt_id"]), -1, np.int64)
    remap[pts] = np.arange(len(pts))
    ep = np.asarray(problem["edge_pt"])
    edges = np.flatnonzero(remap[ep] >= 0)
    sh = {k: problem[k] for k in ("kf_id", "kf_Tcw", "kf_local", "kf_cam")}
    sh["pt_id"] = np.asarray(problem["pt_id"])[pts]
    sh["pt_pos"] = np.asarray(problem["pt_pos"])[pts]
    sh["edge_pt"] = remap[ep[edges]].astype(np.int32)
    sh["edge_kf"] = np.asarray(problem["edge_kf"])[edges]
    sh["edge_obs"] = np.asarray(problem["edge_obs"])[edges]
    sh["edge_inv_sigma2"] = np.asarray(problem["edge_inv_sigma2"])[edges]
    sh["pt_index"] = pts
    sh["edge_index"] = edges
    return sh


def merge_shards(problem, shards, results):
    """Full-problem outputs from per-rank results (poses are identical on every rank: take rank 0's)."""
    npt, ne = len(problem["pt_id"]), len(problem["edge_pt"])
    X = np.zeros((npt, 3), np.float32)
    er = np.zeros(ne, bool)
    for sh, r in zip(shards, results):
        X[sh["pt_index"]] = r["pt_pos"]
        er[sh["edge_index"]] = r["edge_erase"]
    r0 = results[0]
    out = dict(kf_Tcw=r0["kf_Tcw"], pt_pos=X, edge_erase=er, iterations=r0["iterations"],
               n_erased=int(er.sum()), aborted=r0["aborted"])
    for k in ("solve_ini_chi2", "solve_chi2", "trial_chi2", "trial_lambda"):
        if k in r0:
            out[k] = r0[k]
    return out


class Comm:
    """Exchange handle of a sharded BA rank (orbgpu_comm_h)."""

    def __init__(self, h):
        self._h = h

    @staticmethod
    def unique_id():
        """RCCL unique id (rank 0); distribute the 128 bytes to every rank."""
        buf = (C.c_uint8 * 128)()
        check(lib().orbgpu_comm_unique_id(buf), "orbgpu_comm_unique_id")
        return bytes(buf)

    @classmethod
    def rccl(cls, nranks, rank, uid):
        h = C.c_void_p()
        check(lib().orbgpu_comm_init_rccl(int(nranks), int(rank), (C.c_uint8 * 128)(*uid), C.byref(h)),
              "orbgpu_comm_init_rccl")
        return cls(h)

    @classmethod
    def local_group(cls, nranks):
        hs = (C.c_void_p * nranks)()
        check(lib().orbgpu_comm_init_local(int(nranks), hs), "orbgpu_comm_init_local")
        return [cls(C.c_void_p(h)) for h in hs]

    @classmethod
    def shm(cls, name, nranks, rank, max_doubles):
        """One process per rank on one host (orbgpu_comm_init_shm): every rank passes the same fresh
        name ("/..."), nranks and max_doubles (the largest exchange in doubles)."""
        h = C.c_void_p()
        check(lib().orbgpu_comm_init_shm(name.encode(), int(nranks), int(rank), int(max_doubles), C.byref(h)),
              "orbgpu_comm_init_shm")
        return cls(h)

    @property
    def rank_size(self):
        r, s = C.c_int(), C.c_int()
        check(lib().orbgpu_comm_rank(self._h, C.byref(r), C.byref(s)))
        return r.value, s.value

    def close(self):
        if getattr(self, "_h", None):
            lib().orbgpu_comm_destroy(self._h)
            self._h = None

    __del__ = close


def LocalBundleAdjustmentSharded(shard, comm, stop=None, trace=False):
    k = _Packed(_args(shard))
    check(lib().Optimizer_LocalBundleAdjustment_sharded(C.byref(k.P), comm._h, _stop_ref(stop), C.byref(k.R)),
          "Optimizer_LocalBundleAdjustment_sharded")
    return k.result(trace)


def BundleAdjustmentSharded(shard, comm, nIterations=10, bRobust=False, stop=None, trace=False):
    k = _Packed(_args(shard))
    check(lib().Optimizer_BundleAdjustment_sharded(C.byref(k.P), comm._h, int(nIterations), int(bool(bRobust)),
                                                   _stop_ref(stop), C.byref(k.R)),
          "Optimizer_BundleAdjustment_sharded")
    return k.result(trace)


def run_sharded_local(problem, nranks, mode="local", nIterations=10, bRobust=False, trace=False, pt_rank=None,
                      partition="block"):
    """Run the sharded protocol with `nranks` in-process ranks (threads) on the current device;
    returns (merged result, per-rank results).  mode: "local" or "global"; partition: "block"
    (keyframe blocks) or "nd" (separator-tree subtrees: the sharded factorisation).  Each rank's
    result carries `sharding` (last_sharding())."""
    if pt_rank is None:
        pt_rank = partition_points_nd(problem, nranks) if partition == "nd" else partition_points(problem, nranks)
    shards = [shard_problem(problem, pt_rank, r) for r in range(nranks)]
    comms = Comm.local_group(nranks)
    results = [None] * nranks
    errors = [None] * nranks

    def work(r):
        try:
            if mode == "local":
                results[r] = LocalBundleAdjustmentSharded(shards[r], comms[r], trace=trace)
            else:
                results[r] = BundleAdjustmentSharded(shards[r], comms[r], nIterations, bRobust, trace=trace)
            results[r]["sharding"] = last_sharding()
            results[r]["lm_path"] = last_lm_path()
        except Exception as e:  # noqa: BLE001 -- re-raised below
            errors[r] = e

    ts = [threading.Thread(target=work, args=(r,)) for r in range(nranks)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    for c in comms:
        c.close()
    for e in errors:
        if e is not None:
            raise e
    return merge_shards(problem, shards, results), results
