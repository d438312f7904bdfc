"""Host-side mirror of the reference's ORBVocabulary (DBoW2::TemplatedVocabulary<FORB::TDescriptor,
FORB>, include/ORBVocabulary.h): loadFromTextFile, transform (BowVector + FeatureVector, the
Frame::ComputeBoW call) and score.  Every call goes through the C ABI into the HIP library;
the text parse is host work, the tree walk, vector assembly and scoring run on the device."""
import ctypes as C
import os

import numpy as np

from ._lib import ORB_E_CAPACITY, check, lib, orb_bow, ptr
from .orb import FeatureVector

L1_NORM, L2_NORM, CHI_SQUARE, KL, BHATTACHARYYA, DOT_PRODUCT = range(6)   # BowVector.h:45-53
TF_IDF, TF, IDF, BINARY = range(4)                                          # BowVector.h:36-42


class BowVector:
    """DBoW2::BowVector: ascending word ids and their values."""

    def __init__(self, words, values):
        self.words = np.ascontiguousarray(words, np.uint32)
        self.values = np.ascontiguousarray(values, np.float64)

    def __len__(self):
        return len(self.words)

    def as_dict(self):
        return dict(zip(self.words.tolist(), self.values.tolist()))


class ORBVocabulary:
    def __init__(self):
        self._L = lib()
        h = C.c_void_p()
        check(self._L.ORBvocabulary_create(C.byref(h)), "ORBvocabulary_create")
        self._h = h

    def close(self):
        if getattr(self, "_h", None):
            self._L.ORBvocabulary_destroy(self._h)
            self._h = None

    __del__ = close

    def loadFromTextFile(self, path):
        """bool loadFromTextFile(const std::string&) (TemplatedVocabulary.h:1338)."""
        return self._L.ORBvocabulary_loadFromTextFile(self._h, os.fsencode(str(path))) == 0

    def info(self):
        v = [C.c_int() for _ in range(6)]
        check(self._L.ORBvocabulary_info(self._h, *[C.byref(x) for x in v]), "ORBvocabulary_info")
        return dict(zip(["k", "L", "scoring", "weighting", "nodes", "words"], [x.value for x in v]))

    def empty(self):
        return self.info()["words"] == 0

    def _out(self, n):
        cap = max(n, 1)
        bufs = dict(word=np.zeros(cap, np.uint32), value=np.zeros(cap, np.float64), fv_node=np.zeros(cap, np.uint32),
                    fv_start=np.zeros(cap + 1, np.int32), fv_feat=np.zeros(cap, np.int32))
        o = orb_bow(cap, ptr(bufs["word"]), ptr(bufs["value"]), 0, ptr(bufs["fv_node"]), ptr(bufs["fv_start"]),
                    ptr(bufs["fv_feat"]), 0)
        return o, bufs

    @staticmethod
    def _result(o, b):
        bow = BowVector(b["word"][:o.n_words].copy(), b["value"][:o.n_words].copy())
        fv = FeatureVector.__new__(FeatureVector)
        fv.node_id = b["fv_node"][:o.n_nodes].copy()
        fv.start = b["fv_start"][:o.n_nodes + 1].copy()
        fv.feat = b["fv_feat"][:int(fv.start[-1]) if o.n_nodes else 0].copy()
        return bow, fv

    def transform(self, desc, levelsup=4):
        """transform(features, BowVector&, FeatureVector&, levelsup) -> (BowVector, FeatureVector)."""
        d = np.ascontiguousarray(desc, np.uint8).reshape(-1, 32)
        o, b = self._out(len(d))
        check(self._L.ORBvocabulary_transform(self._h, ptr(d), len(d), int(levelsup), C.byref(o)),
              "ORBvocabulary_transform")
        return self._result(o, b)

    def transform_batch(self, descs, levelsup=4):
        ds = [np.ascontiguousarray(d, np.uint8).reshape(-1, 32) for d in descs]
        n = np.array([len(d) for d in ds], np.int32)
        outs = [self._out(len(d)) for d in ds]
        arr = (orb_bow * max(len(ds), 1))(*[o for o, _ in outs])
        dp = (C.c_void_p * max(len(ds), 1))(*[d.ctypes.data for d in ds])
        check(self._L.ORBvocabulary_transform_batch(self._h, len(ds), dp, ptr(n), int(levelsup), arr),
              "ORBvocabulary_transform_batch")
        return [self._result(arr[i], outs[i][1]) for i in range(len(ds))]

    def transform_features(self, desc, levelsup=4):
        """Per descriptor (word id, weight, node id at levelsup) -- transform(feature, ...)."""
        d = np.ascontiguousarray(desc, np.uint8).reshape(-1, 32)
        n = max(len(d), 1)
        w, wt, nd = np.zeros(n, np.uint32), np.zeros(n, np.float64), np.zeros(n, np.uint32)
        check(self._L.ORBvocabulary_transform_features(self._h, ptr(d), len(d), int(levelsup), ptr(w), ptr(wt),
                                                       ptr(nd)), "ORBvocabulary_transform_features")
        return w[:len(d)], wt[:len(d)], nd[:len(d)]

    def score(self, a: BowVector, candidates):
        """L1Scoring::score(a, c) for every candidate BowVector c (ScoringObject.cpp:21-66)."""
        cs = list(candidates) if not isinstance(candidates, BowVector) else [candidates]
        start = np.zeros(len(cs) + 1, np.int32)
        start[1:] = np.cumsum([len(c) for c in cs])
        cw = np.concatenate([c.words for c in cs] + [np.zeros(1, np.uint32)])
        cv = np.concatenate([c.values for c in cs] + [np.zeros(1)])
        out = np.zeros(max(len(cs), 1), np.float64)
        qw = a.words if len(a) else np.zeros(1, np.uint32)
        qv = a.values if len(a) else np.zeros(1)
        check(self._L.ORBvocabulary_score(self._h, ptr(qw), ptr(qv), len(a), len(cs), ptr(start), ptr(cw), ptr(cv),
                                          ptr(out)), "ORBvocabulary_score")
        return out[:len(cs)] if not isinstance(candidates, BowVector) else float(out[0])


__all__ = ["ORBVocabulary", "BowVector", "ORB_E_CAPACITY"]
