"""Host mirror of ORB_SLAM2::PnPsolver, ORB_SLAM2::Sim3Solver and
DUtils::Random over the C ABI.

PnPsolver(...) takes the packed correspondences the reference constructor
builds from a Frame and its map-point matches (PnPsolver.cc:67-110);
Sim3Solver(...) the camera-frame pairs its constructor builds from two
keyframes and vpMatched12 (Sim3Solver.cc:37-112).
"""
import ctypes as C

import numpy as np

from ._lib import check, lib, orb_rng, ptr


class Rng:
    """glibc rand() stream (srand(seed)); the reference's process RNG, made explicit."""

    def __init__(self, seed=1):
        self.s = orb_rng()
        lib().orb_rng_seed(C.byref(self.s), seed)

    def rand(self):
        return lib().orb_rng_rand(C.byref(self.s))

    def state(self):
        return (tuple(self.s.tbl), self.s.f, self.s.r)


class PnPsolver:
    def __init__(self, p3d, p2d, sigma2, kp_index, n_matches, fx, fy, cx, cy):
        self._L = lib()
        self.p3d = np.ascontiguousarray(p3d, np.float32).reshape(-1, 3)
        self.p2d = np.ascontiguousarray(p2d, np.float32).reshape(-1, 2)
        self.sigma2 = np.ascontiguousarray(sigma2, np.float32)
        self.kp = np.ascontiguousarray(kp_index, np.int32)
        self.n_matches = int(n_matches)
        h = C.c_void_p()
        check(self._L.PnPsolver_create(len(self.p3d), ptr(self.p3d), ptr(self.p2d), ptr(self.sigma2), ptr(self.kp),
                                       self.n_matches, fx, fy, cx, cy, C.byref(h)), "PnPsolver_create")
        self._h = h

    def close(self):
        if getattr(self, "_h", None):
            self._L.PnPsolver_destroy(self._h)
            self._h = None

    __del__ = close

    def SetRansacParameters(self, probability=0.99, minInliers=8, maxIterations=300, minSet=4, epsilon=0.4,
                            th2=5.991):
        check(self._L.PnPsolver_set_ransac(self._h, probability, minInliers, maxIterations, minSet, epsilon, th2))

    def iterate(self, nIterations, rng: Rng):
        """-> (Tcw or None, bNoMore, vbInliers, nInliers)"""
        no_more, nin, has = C.c_int(), C.c_int(), C.c_int()
        inl = np.zeros(max(self.n_matches, 1), np.uint8)
        T = np.zeros(16, np.float32)
        check(self._L.PnPsolver_iterate(self._h, nIterations, C.byref(rng.s), C.byref(no_more), ptr(inl),
                                        C.byref(nin), ptr(T), C.byref(has)), "PnPsolver_iterate")
        return (T.reshape(4, 4) if has.value else None), bool(no_more.value), inl[:self.n_matches].astype(bool), \
            nin.value

    def state(self):
        a, b, c = C.c_int(), C.c_int(), C.c_int()
        check(self._L.PnPsolver_get_state(self._h, C.byref(a), C.byref(b), C.byref(c)))
        return a.value, b.value, c.value


def iterate_batch(solvers, nIterations, rngs):
    """PnPsolver_iterate_batch: one hypothesis launch for all solvers."""
    L = lib()
    n = len(solvers)
    hs = (C.c_void_p * n)(*[s._h.value for s in solvers])
    rp = (C.c_void_p * n)(*[C.cast(C.byref(r.s), C.c_void_p).value for r in rngs])
    bufs = [np.zeros(max(s.n_matches, 1), np.uint8) for s in solvers]
    ip = (C.c_void_p * n)(*[b.ctypes.data for b in bufs])
    nm, nin, has = (np.zeros(n, np.int32) for _ in range(3))
    T = np.zeros((n, 16), np.float32)
    check(L.PnPsolver_iterate_batch(n, hs, nIterations, rp, ptr(nm), ip, ptr(nin), ptr(T), ptr(has)),
          "PnPsolver_iterate_batch")
    return [((T[k].reshape(4, 4) if has[k] else None), bool(nm[k]), bufs[k][:solvers[k].n_matches].astype(bool),
             int(nin[k])) for k in range(n)]


class Sim3Solver:
    """ORB_SLAM2::Sim3Solver (include/Sim3Solver.h:39-137) on the GPU."""

    def __init__(self, X1c, X2c, sigma2_1, sigma2_2, idx1, N1, K1, K2, bFixScale=True):
        self._L = lib()
        self.X1 = np.ascontiguousarray(X1c, np.float32).reshape(-1, 3)
        self.X2 = np.ascontiguousarray(X2c, np.float32).reshape(-1, 3)
        self.s1 = np.ascontiguousarray(sigma2_1, np.float32)
        self.s2 = np.ascontiguousarray(sigma2_2, np.float32)
        self.idx1 = np.ascontiguousarray(idx1, np.int32)
        self.K1 = np.ascontiguousarray(K1, np.float32)
        self.K2 = np.ascontiguousarray(K2, np.float32)
        self.n_matches = int(N1)
        h = C.c_void_p()
        check(self._L.Sim3Solver_create(len(self.X1), ptr(self.X1), ptr(self.X2), ptr(self.s1), ptr(self.s2),
                                        ptr(self.idx1), self.n_matches, ptr(self.K1), ptr(self.K2), int(bFixScale),
                                        C.byref(h)), "Sim3Solver_create")
        self._h = h

    def close(self):
        if getattr(self, "_h", None):
            self._L.Sim3Solver_destroy(self._h)
            self._h = None

    __del__ = close

    def SetRansacParameters(self, probability=0.99, minInliers=6, maxIterations=300):
        check(self._L.Sim3Solver_set_ransac(self._h, probability, minInliers, maxIterations))

    def iterate(self, nIterations, rng: Rng):
        """-> (T12 or None, bNoMore, vbInliers, nInliers)"""
        no_more, nin, has = C.c_int(), C.c_int(), C.c_int()
        inl = np.zeros(max(self.n_matches, 1), np.uint8)
        T = np.zeros(16, np.float32)
        check(self._L.Sim3Solver_iterate(self._h, nIterations, C.byref(rng.s), C.byref(no_more), ptr(inl),
                                         C.byref(nin), ptr(T), C.byref(has)), "Sim3Solver_iterate")
        return (T.reshape(4, 4) if has.value else None), bool(no_more.value), inl[:self.n_matches].astype(bool), \
            nin.value

    def _estimate(self):
        R, t, s = np.zeros(9, np.float32), np.zeros(3, np.float32), np.zeros(1, np.float32)
        check(self._L.Sim3Solver_get_estimate(self._h, ptr(R), ptr(t), ptr(s)))
        return R.reshape(3, 3), t.reshape(3, 1), float(s[0])

    def GetEstimatedRotation(self):
        return self._estimate()[0]

    def GetEstimatedTranslation(self):
        return self._estimate()[1]

    def GetEstimatedScale(self):
        return self._estimate()[2]

    def state(self):
        a, b, c = C.c_int(), C.c_int(), C.c_int()
        check(self._L.Sim3Solver_get_state(self._h, C.byref(a), C.byref(b), C.byref(c)))
        return a.value, b.value, c.value


def sim3_iterate_batch(solvers, nIterations, rngs):
    """Sim3Solver_iterate_batch: one hypothesis launch for all loop candidates."""
    L = lib()
    n = len(solvers)
    hs = (C.c_void_p * n)(*[s._h.value for s in solvers])
    rp = (C.c_void_p * n)(*[C.cast(C.byref(r.s), C.c_void_p).value for r in rngs])
    bufs = [np.zeros(max(s.n_matches, 1), np.uint8) for s in solvers]
    ip = (C.c_void_p * n)(*[b.ctypes.data for b in bufs])
    nm, nin, has = (np.zeros(n, np.int32) for _ in range(3))
    T = np.zeros((n, 16), np.float32)
    check(L.Sim3Solver_iterate_batch(n, hs, nIterations, rp, ptr(nm), ip, ptr(nin), ptr(T), ptr(has)),
          "Sim3Solver_iterate_batch")
    return [((T[k].reshape(4, 4) if has[k] else None), bool(nm[k]), bufs[k][:solvers[k].n_matches].astype(bool),
             int(nin[k])) for k in range(n)]


class BatchCall:
    """A batch entry (PnPsolver_iterate_batch / Sim3Solver_iterate_batch) with its argument
    arrays built once, as a C++ caller keeps them between calls: call() is the C call alone and
    leaves its results in has / no_more / n_inliers / T / inliers[k]."""

    def __init__(self, kind, solvers, nIterations, rngs):
        L = lib()
        self._fn = L.PnPsolver_iterate_batch if kind == "pnp" else L.Sim3Solver_iterate_batch
        self.n = n = len(solvers)
        self.nIterations = nIterations
        self._hs = (C.c_void_p * n)(*[s._h.value for s in solvers])
        self._rp = (C.c_void_p * n)(*[C.cast(C.byref(r.s), C.c_void_p).value for r in rngs])
        self.inliers = [np.zeros(max(s.n_matches, 1), np.uint8) for s in solvers]
        self._ip = (C.c_void_p * n)(*[b.ctypes.data for b in self.inliers])
        self.no_more, self.n_inliers, self.has = (np.zeros(n, np.int32) for _ in range(3))
        self.T = np.zeros((n, 16), np.float32)
        self._args = (n, self._hs, nIterations, self._rp, ptr(self.no_more), self._ip, ptr(self.n_inliers),
                      ptr(self.T), ptr(self.has))
        self._solvers = solvers   # the handles stay alive with the call
        self._rngs = rngs

    def __call__(self):
        check(self._fn(*self._args), "iterate_batch")
