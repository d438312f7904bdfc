"""ctypes binding of the CPU parity oracle (oracle/liborb_oracle.so).

TEST INFRASTRUCTURE ONLY -- the checker, never the thing measured.
"""
import ctypes as C
import os
import subprocess
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
ORACLE_DIR = ROOT / "oracle"
LIB_PATH = ORACLE_DIR / "liborb_oracle.so"

KP_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
                     ("response", "<f4"), ("octave", "<i4"), ("class_id", "<i4")])
assert KP_DTYPE.itemsize == 28


def build():
    subprocess.run(["make", "-s", "-C", str(ORACLE_DIR)], check=True)


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            build()
        L = C.CDLL(str(LIB_PATH))
        vp, i32, f32 = C.c_void_p, C.c_int, C.c_float
        L.ora_extractor_new.restype = vp
        L.ora_extractor_new.argtypes = [i32, f32, i32, i32, i32]
        L.ora_extractor_free.argtypes = [vp]
        L.ora_extract.argtypes = [vp, vp, i32, i32, i32, vp, vp, i32]
        L.ora_extract.restype = i32
        L.ora_extractor_level.argtypes = [vp, i32, C.POINTER(C.c_void_p), C.POINTER(i32), C.POINTER(i32), C.POINTER(i32)]
        L.ora_extractor_blurred.argtypes = [vp, i32, C.POINTER(C.c_void_p), C.POINTER(i32), C.POINTER(i32)]
        L.ora_extractor_candidates.argtypes = [vp, i32, vp, i32]
        L.ora_extractor_tables.argtypes = [vp, vp, vp, vp, vp, vp, vp]
        L.ora_fastAtan2.restype = f32
        L.ora_fastAtan2.argtypes = [f32, f32]
        L.ora_sinf.restype = f32
        L.ora_sinf.argtypes = [f32]
        L.ora_cosf.restype = f32
        L.ora_cosf.argtypes = [f32]
        L.ora_fast_score.argtypes = [vp, i32]
        L.ora_descriptor_distance.argtypes = [vp, vp]
        L.ora_gaussian7_taps.argtypes = [vp]
        L.ora_resize_linear_u8.argtypes = [vp, i32, i32, i32, vp, i32, i32, i32]
        L.ora_gaussian7_u8.argtypes = [vp, i32, i32, i32, vp, i32]
        L.ora_rng_seed.argtypes = [vp, C.c_uint]
        L.ora_rng_rand.argtypes = [vp]
        L.ora_rng_random_int.argtypes = [vp, i32, i32]
        _lib = L
    return _lib


def ptr(a):
    return a.ctypes.data_as(C.c_void_p)


class OracleExtractor:
    """ORBextractor(nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST) restated on CPU."""

    def __init__(self, nfeatures=1200, scale_factor=1.2, nlevels=8, ini_th=20, min_th=7):
        self.L = lib()
        self.h = self.L.ora_extractor_new(nfeatures, scale_factor, nlevels, ini_th, min_th)
        assert self.h
        self.nlevels = nlevels

    def __del__(self):
        if getattr(self, "h", None):
            self.L.ora_extractor_free(self.h)
            self.h = None

    def __call__(self, img):
        img = np.ascontiguousarray(img, dtype=np.uint8)
        cap = 8192
        while True:
            kps = np.zeros(cap, KP_DTYPE)
            desc = np.zeros((cap, 32), np.uint8)
            n = self.L.ora_extract(self.h, ptr(img), img.shape[1], img.shape[0], img.strides[0],
                                   ptr(kps), ptr(desc), cap)
            if n == -1 and cap > 0:
                raise RuntimeError("oracle extraction failed (image too small?)")
            if n < 0:
                cap = -n
                continue
            return kps[:n].copy(), desc[:n].copy()

    def level(self, l):
        d, pw, ph, st = C.c_void_p(), C.c_int(), C.c_int(), C.c_int()
        assert self.L.ora_extractor_level(self.h, l, C.byref(d), C.byref(pw), C.byref(ph), C.byref(st)) == 0
        buf = (C.c_uint8 * (st.value * ph.value)).from_address(d.value)
        return np.frombuffer(buf, np.uint8).reshape(ph.value, st.value)[:, :pw.value].copy()

    def blurred(self, l):
        d, w, h = C.c_void_p(), C.c_int(), C.c_int()
        assert self.L.ora_extractor_blurred(self.h, l, C.byref(d), C.byref(w), C.byref(h)) == 0
        buf = (C.c_uint8 * (w.value * h.value)).from_address(d.value)
        return np.frombuffer(buf, np.uint8).reshape(h.value, w.value).copy()

    def candidates(self, l):
        n = self.L.ora_extractor_candidates(self.h, l, None, 0)
        out = np.zeros(max(n, 1), KP_DTYPE)
        self.L.ora_extractor_candidates(self.h, l, ptr(out), n)
        return out[:n]

    def tables(self):
        nl = self.nlevels
        sc, isc, s2, is2 = (np.zeros(nl, np.float32) for _ in range(4))
        npl = np.zeros(nl, np.int32)
        umax = np.zeros(16, np.int32)
        self.L.ora_extractor_tables(self.h, ptr(sc), ptr(isc), ptr(s2), ptr(is2), ptr(npl), ptr(umax))
        return dict(scale=sc, inv_scale=isc, sigma2=s2, inv_sigma2=is2, n_per_level=npl, umax=umax)
