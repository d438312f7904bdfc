"""Host mirror of ORB_SLAM2::Optimizer::LocalBundleAdjustment over the C ABI.

LocalBundleAdjustment(...) takes the arrays the reference gathers from the
covisibility graph (Optimizer.cc:456-653, see include/orbslam_gpu.h ba_problem)
and returns what it writes back: keyframe poses, map point positions and the
(keyframe, map point) observations to erase.
"""
import ctypes as C

import numpy as np

from ._lib import ba_problem, ba_result, check, lib, ptr

_FIELDS = (("kf_id", np.int32), ("kf_Tcw", np.float32), ("kf_local", np.uint8), ("kf_cam", np.float32),
           ("pt_id", np.int32), ("pt_pos", np.float32), ("edge_pt", np.int32), ("edge_kf", np.int32),
           ("edge_obs", np.float32), ("edge_inv_sigma2", np.float32))


def LocalBundleAdjustment(kf_id, kf_Tcw, kf_local, kf_cam, pt_id, pt_pos, edge_pt, edge_kf, edge_obs, edge_inv_sigma2,
                          stop=None, trace=False):
    """-> dict(kf_Tcw, pt_pos, edge_erase, iterations, n_erased, aborted[, trace])

    stop: optional ctypes.c_bool shared with another thread (pbStopFlag)."""
    L = lib()
    a = {}
    for (name, dt), v in zip(_FIELDS, (kf_id, kf_Tcw, kf_local, kf_cam, pt_id, pt_pos, edge_pt, edge_kf, edge_obs,
                                       edge_inv_sigma2)):
        a[name] = np.ascontiguousarray(v, dt)
    nkf, npt, ne = len(a["kf_id"]), len(a["pt_id"]), len(a["edge_pt"])
    P = ba_problem(nkf, ptr(a["kf_id"]), ptr(a["kf_Tcw"]), ptr(a["kf_local"]), ptr(a["kf_cam"]), npt, ptr(a["pt_id"]),
                   ptr(a["pt_pos"]), ne, ptr(a["edge_pt"]), ptr(a["edge_kf"]), ptr(a["edge_obs"]),
                   ptr(a["edge_inv_sigma2"]))
    T = np.zeros((nkf, 16), np.float32)
    X = np.zeros((npt, 3), np.float32)
    er = np.zeros(max(ne, 1), np.uint8)
    R = ba_result(ptr(T), ptr(X), ptr(er))
    check(L.Optimizer_LocalBundleAdjustment(C.byref(P), C.byref(stop) if stop is not None else None, C.byref(R)),
          "Optimizer_LocalBundleAdjustment")
    out = dict(kf_Tcw=T, pt_pos=X, edge_erase=er[:ne].astype(bool), iterations=tuple(R.iterations),
               n_erased=R.n_erased, aborted=bool(R.aborted))
    if trace:
        cap = 4096
        si, sc, tc, tl = (np.zeros(cap) for _ in range(4))
        ns, nt = C.c_int(), C.c_int()
        check(L.Optimizer_last_trace(ptr(si), ptr(sc), cap, C.byref(ns), ptr(tc), ptr(tl), cap, C.byref(nt)))
        out.update(solve_ini_chi2=si[:ns.value], solve_chi2=sc[:ns.value], trial_chi2=tc[:nt.value],
                   trial_lambda=tl[:nt.value])
    return out


def last_timings():
    ms = np.zeros(2)
    check(lib().Optimizer_last_timings(ptr(ms)))
    return ms
