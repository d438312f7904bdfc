"""Host-side mirror of the reference ORBextractor / ORBmatcher interface.

Same names, argument meaning and error behaviour as the reference classes
(include/ORBextractor.h, include/ORBmatcher.h); every call goes through the
C ABI of include/orbslam_gpu.h into the HIP library.  cv::Mat / vector<KeyPoint>
become numpy arrays: keypoints are KP_DTYPE records (cv::KeyPoint layout),
descriptors (N, 32) uint8, map-point pointers int32 indices (-1 = NULL).
"""
import ctypes as C

import numpy as np

from ._lib import (KP_DTYPE, ORB_E_CAPACITY, OrbGpuError, check, lib, orb_featvec, orb_frame, orb_mappoint_geo, orb_mappoints, ptr)

FRAME_GRID_COLS, FRAME_GRID_ROWS = 64, 48   # Frame.h:37-38


class ORBextractor:
    """ORBextractor(nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST)  (ORBextractor.cc:410)."""

    def __init__(self, nfeatures, scaleFactor, nlevels, iniThFAST, minThFAST,
                 max_width=2048, max_height=2048, max_batch=1):
        self._L = lib()
        h = C.c_void_p()
        check(self._L.ORBextractor_create(int(nfeatures), float(scaleFactor), int(nlevels), int(iniThFAST),
                                          int(minThFAST), int(max_width), int(max_height), int(max_batch),
                                          C.byref(h)), "ORBextractor_create")
        self._h = h
        self.nfeatures, self.nlevels = int(nfeatures), int(nlevels)
        self.max_batch = int(max_batch)
        self._cap = max(64, 2 * int(nfeatures) + 64)

    def close(self):
        if getattr(self, "_h", None):
            self._L.ORBextractor_destroy(self._h)
            self._h = None

    __del__ = close

    # operator()(image, mask, keypoints, descriptors) -- ORBextractor.cc:1043
    def __call__(self, image, mask=None):
        img = np.ascontiguousarray(image, dtype=np.uint8)
        if img.size == 0:
            return np.zeros(0, KP_DTYPE), None
        while True:
            kps = np.zeros(self._cap, KP_DTYPE)
            desc = np.zeros((self._cap, 32), np.uint8)
            n = C.c_int()
            rc = self._L.ORBextractor_extract(self._h, ptr(img), img.shape[1], img.shape[0], img.strides[0],
                                              ptr(kps), ptr(desc), self._cap, C.byref(n))
            if rc == ORB_E_CAPACITY:
                self._cap *= 2
                continue
            check(rc, "ORBextractor_extract")
            n = n.value
            return kps[:n].copy(), (desc[:n].copy() if n else None)

    def extract_batch(self, images):
        imgs = np.ascontiguousarray(images, dtype=np.uint8)
        B, H, W = imgs.shape
        while True:
            kps = np.zeros((B, self._cap), KP_DTYPE)
            desc = np.zeros((B, self._cap, 32), np.uint8)
            n = np.zeros(B, np.int32)
            rc = self._L.ORBextractor_extract_batch(self._h, ptr(imgs), B, W, H, imgs.strides[1], imgs.strides[0],
                                                    0, ptr(kps), ptr(desc), self._cap, 0, ptr(n))
            if rc == ORB_E_CAPACITY:
                self._cap *= 2
                continue
            check(rc, "ORBextractor_extract_batch")
            return [(kps[b, :n[b]].copy(), desc[b, :n[b]].copy()) for b in range(B)]

    def extract_device(self, d_imgs_ptr, B, W, H, step, img_stride, d_kps_ptr, d_desc_ptr, cap):
        """HBM-resident form: all pointers are device addresses; returns per-image counts."""
        n = np.zeros(B, np.int32)
        check(self._L.ORBextractor_extract_batch(self._h, C.c_void_p(d_imgs_ptr), B, W, H, step, img_stride, 1,
                                                 C.c_void_p(d_kps_ptr), C.c_void_p(d_desc_ptr), cap, 1, ptr(n)),
              "ORBextractor_extract_batch(device)")
        return n

    def extract_host_to_device(self, image, d_kps_ptr, d_desc_ptr, cap):
        """operator() on a host (pageable) image, keypoints and descriptors left in HBM for the
        device-resident tracking calls: the H2D copy of the image is part of the call.  -> count."""
        img = np.ascontiguousarray(image, dtype=np.uint8)
        H, W = img.shape
        n = np.zeros(1, np.int32)
        check(self._L.ORBextractor_extract_batch(self._h, ptr(img), 1, W, H, img.strides[0], img.strides[0] * H, 0,
                                                 C.c_void_p(d_kps_ptr), C.c_void_p(d_desc_ptr), cap, 1, ptr(n)),
              "ORBextractor_extract_batch(host image)")
        return n

    def extract_host_images_to_device(self, images, d_kps_ptr, d_desc_ptr, cap):
        """Frame(imLeft, imRight)'s extractions (Frame.cc:78-81) in one call: the host images of
        equal size staged as one block, one H2D copy, keypoints / descriptors of image b left in HBM
        at d_kps_ptr + b*cap entries.  -> counts."""
        imgs = [np.ascontiguousarray(im, dtype=np.uint8) for im in images]
        H, W = imgs[0].shape
        if any(im.shape != (H, W) for im in imgs):
            raise ValueError("images of different sizes")
        lst = (C.c_void_p * len(imgs))(*[im.ctypes.data for im in imgs])
        n = np.zeros(len(imgs), np.int32)
        check(self._L.ORBextractor_extract_images(self._h, lst, len(imgs), W, H, imgs[0].strides[0],
                                                  C.c_void_p(d_kps_ptr), C.c_void_p(d_desc_ptr), cap, 1, ptr(n)),
              "ORBextractor_extract_images")
        return n

    def image_pyramid_level(self, level, index=0):
        """mvImagePyramid[level] WITH its 19-px border (ORBextractor.h:85)."""
        w, h = C.c_int(), C.c_int()
        check(self._L.ORBextractor_get_level(self._h, index, level, None, 0, C.byref(w), C.byref(h)), "get_level")
        out = np.zeros((h.value + 38, w.value + 38), np.uint8)
        check(self._L.ORBextractor_get_level(self._h, index, level, ptr(out), out.strides[0], C.byref(w),
                                             C.byref(h)), "get_level")
        return out

    def blurred_level(self, level, index=0):
        """GaussianBlur working image of `level` (diagnostic; ORBextractor.cc:1085-1086)."""
        w, h = C.c_int(), C.c_int()
        check(self._L.ORBextractor_get_blurred_level(self._h, index, level, None, 0, C.byref(w), C.byref(h)))
        out = np.zeros((h.value, w.value), np.uint8)
        check(self._L.ORBextractor_get_blurred_level(self._h, index, level, ptr(out), out.strides[0], C.byref(w),
                                                     C.byref(h)))
        return out

    def _tables(self):
        nl = self.nlevels
        t = [np.zeros(nl, np.float32) for _ in range(4)] + [np.zeros(nl, np.int32)]
        check(self._L.ORBextractor_get_scale_tables(self._h, *[ptr(a) for a in t]), "get_scale_tables")
        return t

    def GetLevels(self):
        return self.nlevels

    def GetScaleFactor(self):
        n, s = C.c_int(), C.c_float()
        check(self._L.ORBextractor_get_levels(self._h, C.byref(n), C.byref(s)))
        return s.value

    def GetScaleFactors(self):
        return self._tables()[0]

    def GetInverseScaleFactors(self):
        return self._tables()[1]

    def GetScaleSigmaSquares(self):
        return self._tables()[2]

    def GetInverseScaleSigmaSquares(self):
        return self._tables()[3]

    def features_per_level(self):
        return self._tables()[4]

    @property
    def stream(self):
        return self._L.ORBextractor_stream(self._h)

    def last_timings(self):
        t = np.zeros(6, np.float32)
        check(self._L.ORBextractor_last_timings(self._h, ptr(t)))
        return dict(zip(["pyramid", "blur", "fast_cells", "compact", "octree", "orient_desc"], t.tolist()))

    def last_corner_count(self):
        """FAST corners the last call kept (all its images), before DistributeOctTree."""
        n = np.zeros(1, np.int64)
        check(self._L.ORBextractor_last_corner_count(self._h, ptr(n)))
        return int(n[0])


class Frame:
    """The Frame fields the matcher reads (Frame.h).  Arrays are host numpy."""

    def __init__(self, keysUn, desc, scale_factors, Tcw, fx, fy, cx, cy, bf=0.0, width=None, height=None,
                 uRight=None, minX=0.0, maxX=None, minY=0.0, maxY=None):
        self.keysUn = np.ascontiguousarray(keysUn, KP_DTYPE)
        self.N = len(self.keysUn)
        self.desc = np.ascontiguousarray(desc if desc is not None else np.zeros((0, 32), np.uint8), np.uint8)
        self.uRight = None if uRight is None else np.ascontiguousarray(uRight, np.float32)
        self.scale = np.ascontiguousarray(scale_factors, np.float32)
        self.Tcw = np.ascontiguousarray(Tcw, np.float32).reshape(4, 4)
        self.fx, self.fy, self.cx, self.cy = (np.float32(v) for v in (fx, fy, cx, cy))
        self.bf = np.float32(bf)
        self.b = np.float32(np.float32(bf) / np.float32(fx))   # mb = mbf/fx (Frame.cc:114)
        # ComputeImageBounds (no distortion), Frame.cc:464-469
        self.minX, self.minY = np.float32(minX), np.float32(minY)
        self.maxX = np.float32(width if maxX is None else maxX)
        self.maxY = np.float32(height if maxY is None else maxY)
        self.gridWInv = np.float32(np.float32(FRAME_GRID_COLS) / (self.maxX - self.minX))
        self.gridHInv = np.float32(np.float32(FRAME_GRID_ROWS) / (self.maxY - self.minY))

    def cstruct(self):
        f = orb_frame()
        f.N = self.N
        f.keysUn = self.keysUn.ctypes.data if self.N else None
        f.desc = self.desc.ctypes.data if self.N else None
        f.uRight = None if self.uRight is None else self.uRight.ctypes.data
        f.minX, f.maxX, f.minY, f.maxY = self.minX, self.maxX, self.minY, self.maxY
        f.gridWInv, f.gridHInv = self.gridWInv, self.gridHInv
        f.scaleFactors = self.scale.ctypes.data
        f.nlevels = len(self.scale)
        f.fx, f.fy, f.cx, f.cy, f.bf, f.b = self.fx, self.fy, self.cx, self.cy, self.bf, self.b
        f.Tcw = self.Tcw.ctypes.data
        return f


class FeatureVector:
    """DBoW2::FeatureVector (map<NodeId, vector<unsigned>>) as CSR; built from per-feature node ids."""

    def __init__(self, node_of_feature):
        node = np.asarray(node_of_feature, np.int64)
        order = np.argsort(node, kind="stable")              # feature index order kept inside a node
        ids, counts = np.unique(node[order], return_counts=True)
        self.node_id = np.ascontiguousarray(ids, np.uint32)
        self.start = np.ascontiguousarray(np.concatenate([[0], np.cumsum(counts)]), np.int32)
        self.feat = np.ascontiguousarray(order, np.int32)

    def cstruct(self):
        v = orb_featvec()
        v.n_nodes = len(self.node_id)
        v.node_id = self.node_id.ctypes.data
        v.start = self.start.ctypes.data
        v.feat = self.feat.ctypes.data
        return v


class MapPoints:
    def __init__(self, pos, desc, observations):
        self.pos = np.ascontiguousarray(pos, np.float32).reshape(-1, 3)
        self.desc = np.ascontiguousarray(desc, np.uint8).reshape(-1, 32)
        self.obs = np.ascontiguousarray(observations, np.int32)
        self.n = len(self.pos)

    def cstruct(self):
        m = orb_mappoints()
        m.n = self.n
        m.pos = self.pos.ctypes.data if self.n else None
        m.desc = self.desc.ctypes.data if self.n else None
        m.observations = self.obs.ctypes.data if self.n else None
        return m


class MapPointGeo:
    """mfMaxDistance, mfMinDistance, GetNormal() of the rows of a MapPoints table."""

    def __init__(self, max_dist, min_dist, normal=None):
        self.max_dist = np.ascontiguousarray(max_dist, np.float32)
        self.min_dist = np.ascontiguousarray(min_dist, np.float32)
        self.normal = None if normal is None else np.ascontiguousarray(normal, np.float32).reshape(-1, 3)

    def cstruct(self):
        g = orb_mappoint_geo()
        g.max_dist = self.max_dist.ctypes.data if len(self.max_dist) else None
        g.min_dist = self.min_dist.ctypes.data if len(self.min_dist) else None
        g.normal = self.normal.ctypes.data if self.normal is not None and len(self.normal) else None
        return g


class ORBmatcher:
    """ORBmatcher(nnratio=0.6, checkOri=True)  (ORBmatcher.cc:41-43)."""

    TH_HIGH, TH_LOW, HISTO_LENGTH = 100, 50, 30

    def __init__(self, nnratio=0.6, checkOri=True):
        self._L = lib()
        h = C.c_void_p()
        check(self._L.ORBmatcher_create(float(nnratio), int(bool(checkOri)), C.byref(h)), "ORBmatcher_create")
        self._h = h
        self.mfNNratio, self.mbCheckOrientation = float(nnratio), bool(checkOri)

    def close(self):
        if getattr(self, "_h", None):
            self._L.ORBmatcher_destroy(self._h)
            self._h = None

    __del__ = close

    @staticmethod
    def DescriptorDistance(a, b):
        a = np.ascontiguousarray(a, np.uint8)
        b = np.ascontiguousarray(b, np.uint8)
        return lib().ORBmatcher_DescriptorDistance(ptr(a), ptr(b))

    def SearchDense(self, queries, trains):
        """Brute-force matching (ORBmatcher_SearchDense_batch): problem p matches every descriptor
        of queries[p] (n x 32 u8) against every row of trains[p]; host arrays.  -> list of
        (best_idx, best_dist, second_dist) int32 arrays (ORBmatcher.cc loop rule: strict '<')."""
        n = len(queries)
        qs = [np.ascontiguousarray(q, np.uint8).reshape(-1, 32) for q in queries]
        ts = [np.ascontiguousarray(t, np.uint8).reshape(-1, 32) for t in trains]
        outs = [tuple(np.zeros(len(q), np.int32) for _ in range(3)) for q in qs]
        arr = lambda xs: (C.c_void_p * max(n, 1))(*[x.ctypes.data if x.size else None for x in xs])
        nq = np.array([len(q) for q in qs] or [0], np.int32)
        nt = np.array([len(t) for t in ts] or [0], np.int32)
        check(self._L.ORBmatcher_set_device_pointers(self._h, 0))
        check(self._L.ORBmatcher_SearchDense_batch(self._h, n, arr(qs), ptr(nq), arr(ts), ptr(nt),
                                                   arr([o[0] for o in outs]), arr([o[1] for o in outs]),
                                                   arr([o[2] for o in outs])), "ORBmatcher_SearchDense_batch")
        return outs

    def SearchByProjection_LastFrame(self, cur: Frame, cur_mp, last: Frame, last_keys, last_mp, last_outlier,
                                     mps: MapPoints, th, bMono):
        """SearchByProjection(CurrentFrame, LastFrame, th, bMono) (ORBmatcher.cc:1328).
        cur_mp is updated in place (CurrentFrame.mvpMapPoints); returns nmatches."""
        assert cur_mp.dtype == np.int32 and cur_mp.flags.c_contiguous and len(cur_mp) == cur.N
        lk = np.ascontiguousarray(last_keys, KP_DTYPE)
        lm = np.ascontiguousarray(last_mp, np.int32)
        lo = np.ascontiguousarray(last_outlier, np.uint8)
        cf, lf, mp = cur.cstruct(), last.cstruct(), mps.cstruct()
        n = C.c_int()
        check(self._L.ORBmatcher_SearchByProjection_LastFrame(self._h, C.byref(cf), ptr(cur_mp), C.byref(lf),
                                                              ptr(lk), ptr(lm), ptr(lo), C.byref(mp),
                                                              float(th), int(bool(bMono)), C.byref(n)),
              "SearchByProjection(LastFrame)")
        return n.value

    def SearchByProjection_MapPoints(self, F: Frame, cur_mp, track_in_view, proj_x, proj_xr, proj_y, level,
                                     view_cos, mp_index, mps: MapPoints, th=1.0):
        """SearchByProjection(F, vpMapPoints, th) (ORBmatcher.cc:45); cur_mp updated in place."""
        assert cur_mp.dtype == np.int32 and len(cur_mp) == F.N
        a = [np.ascontiguousarray(track_in_view, np.uint8), np.ascontiguousarray(proj_x, np.float32),
             np.ascontiguousarray(proj_xr, np.float32), np.ascontiguousarray(proj_y, np.float32),
             np.ascontiguousarray(level, np.int32), np.ascontiguousarray(view_cos, np.float32),
             np.ascontiguousarray(mp_index, np.int32)]
        f, mp = F.cstruct(), mps.cstruct()
        n = C.c_int()
        check(self._L.ORBmatcher_SearchByProjection_MapPoints(self._h, C.byref(f), ptr(cur_mp), len(a[0]),
                                                              *[ptr(x) for x in a], C.byref(mp), float(th),
                                                              C.byref(n)), "SearchByProjection(MapPoints)")
        return n.value

    def ComputeStereoMatches(self, left, right, keysL, descL, keysR, descR, mbf, mb):
        """Frame::ComputeStereoMatches() (Frame.cc:466-640) for image 0 of the last call of the
        `left` / `right` ORBextractors (their mvImagePyramid).  -> (mvuRight, mvDepth, nmatches)."""
        kL = np.ascontiguousarray(keysL, KP_DTYPE)
        kR = np.ascontiguousarray(keysR, KP_DTYPE)
        dL = np.ascontiguousarray(descL if descL is not None else np.zeros((0, 32)), np.uint8)
        dR = np.ascontiguousarray(descR if descR is not None else np.zeros((0, 32)), np.uint8)
        uR = np.zeros(max(len(kL), 1), np.float32)
        dep = np.zeros(max(len(kL), 1), np.float32)
        n = C.c_int()
        check(self._L.ORBmatcher_ComputeStereoMatches(self._h, left._h, right._h, 0, len(kL), ptr(kL), ptr(dL),
                                                      len(kR), ptr(kR), ptr(dR), float(mbf), float(mb), ptr(uR),
                                                      ptr(dep), C.byref(n)), "ORBmatcher_ComputeStereoMatches")
        return uR[:len(kL)], dep[:len(kL)], n.value

    def ComputeStereoMatches_batch(self, left, right, keysL, descL, keysR, descR, mbf, mb, first_left=0,
                                   first_right=0):
        """Batched form over the images 0..P-1 of the last extract_batch of both extractors; pair p
        takes image first_left + p of `left` and first_right + p of `right` (one extractor's batch
        over [lefts..., rights...]: left is right, first_right = P)."""
        P = len(keysL)
        kL = [np.ascontiguousarray(k, KP_DTYPE) for k in keysL]
        kR = [np.ascontiguousarray(k, KP_DTYPE) for k in keysR]
        dL = [np.ascontiguousarray(d if d is not None else np.zeros((0, 32)), np.uint8) for d in descL]
        dR = [np.ascontiguousarray(d if d is not None else np.zeros((0, 32)), np.uint8) for d in descR]
        uR = [np.zeros(max(len(k), 1), np.float32) for k in kL]
        dep = [np.zeros(max(len(k), 1), np.float32) for k in kL]
        arr = lambda xs: (C.c_void_p * P)(*[x.ctypes.data for x in xs])
        NL = np.array([len(k) for k in kL], np.int32)
        NR = np.array([len(k) for k in kR], np.int32)
        n = np.zeros(P, np.int32)
        check(self._L.ORBmatcher_ComputeStereoMatches_batch_at(self._h, left._h, int(first_left), right._h,
                                                               int(first_right), P, ptr(NL), arr(kL), arr(dL),
                                                               ptr(NR), arr(kR), arr(dR), float(mbf), float(mb),
                                                               arr(uR), arr(dep), ptr(n)),
              "ORBmatcher_ComputeStereoMatches_batch_at")
        return [u[:len(k)] for u, k in zip(uR, kL)], [d[:len(k)] for d, k in zip(dep, kL)], n

    def _local_batch(self, frames, maps, dev, want_desc=True):
        """Device copies (torch) of host Frames and local maps (dicts of numpy arrays: pos, desc,
        obs, max_dist, min_dist, normal, skip) and their C structs."""
        import torch
        from ._lib import orb_frame, orb_localmap
        keep, fs, ms = [], [], []
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
        for F, M in zip(frames, maps):
            n = len(M["pos"])
            d = dict(k=t(F.keysUn.view(np.int32).reshape(F.N, 7) if F.N else np.zeros((1, 7), np.int32)),
                     desc=t(F.desc if F.N else np.zeros((1, 32), np.uint8)), scale=t(F.scale),
                     Tcw=t(F.Tcw.reshape(16)),
                     uR=None if F.uRight is None else t(F.uRight if F.N else np.zeros(1, np.float32)),
                     pos=t(np.asarray(M["pos"], np.float32).reshape(-1, 3) if n else np.zeros((1, 3), np.float32)),
                     mdesc=t(np.asarray(M.get("desc", np.zeros((n, 32))), np.uint8).reshape(-1, 32) if n
                             else np.zeros((1, 32), np.uint8)),
                     obs=t(np.asarray(M.get("obs", np.ones(n)), np.int32) if n else np.zeros(1, np.int32)),
                     mx=t(np.asarray(M["max_dist"], np.float32) if n else np.zeros(1, np.float32)),
                     mn=t(np.asarray(M["min_dist"], np.float32) if n else np.zeros(1, np.float32)),
                     nrm=t(np.asarray(M["normal"], np.float32).reshape(-1, 3) if n else np.zeros((1, 3), np.float32)),
                     skip=t(np.asarray(M["skip"], np.uint8) if n else np.zeros(1, np.uint8)))
            keep.append(d)
            f = orb_frame()
            f.N = F.N
            f.keysUn, f.desc = d["k"].data_ptr(), d["desc"].data_ptr()
            f.uRight = None if d["uR"] is None else d["uR"].data_ptr()
            f.minX, f.maxX, f.minY, f.maxY = F.minX, F.maxX, F.minY, F.maxY
            f.gridWInv, f.gridHInv = F.gridWInv, F.gridHInv
            f.scaleFactors, f.nlevels = d["scale"].data_ptr(), len(F.scale)
            f.fx, f.fy, f.cx, f.cy, f.bf, f.b = F.fx, F.fy, F.cx, F.cy, F.bf, F.b
            f.Tcw = d["Tcw"].data_ptr()
            fs.append(f)
            ms.append(orb_localmap(n, d["pos"].data_ptr(), d["mdesc"].data_ptr(), d["obs"].data_ptr(),
                                   d["mx"].data_ptr(), d["mn"].data_ptr(), d["nrm"].data_ptr(), d["skip"].data_ptr()))
        cnt = max(len(fs), 1)
        return keep, (orb_frame * cnt)(*fs), (orb_localmap * cnt)(*ms)

    def isInFrustum(self, frames, maps, logScaleFactor, viewingCosLimit=0.5):
        """Frame::isInFrustum (Frame.cc:269-325) of every local map point of maps[f] in frames[f]
        (host Frames / dicts) on the device -> per frame dict(in_view, proj_x, proj_xr, proj_y, level,
        view_cos, nvisible) as numpy."""
        import torch
        dev = torch.device("cuda", torch.cuda.current_device())
        keep, fa, ma = self._local_batch(frames, maps, dev)
        outs = []
        for M in maps:
            n = max(len(M["pos"]), 1)
            outs.append(dict(in_view=torch.full((n,), 7, dtype=torch.uint8, device=dev),
                             proj_x=torch.zeros(n, device=dev), proj_xr=torch.zeros(n, device=dev),
                             proj_y=torch.zeros(n, device=dev), level=torch.zeros(n, dtype=torch.int32, device=dev),
                             view_cos=torch.zeros(n, device=dev)))
        arr = lambda k: (C.c_void_p * max(len(outs), 1))(*[o[k].data_ptr() for o in outs])
        nv = np.zeros(max(len(frames), 1), np.int32)
        check(self._L.ORBmatcher_set_device_pointers(self._h, 1))
        try:
            check(self._L.Frame_isInFrustum_batch(self._h, len(frames), fa, ma, float(viewingCosLimit),
                                                  float(logScaleFactor), arr("in_view"), arr("proj_x"),
                                                  arr("proj_xr"), arr("proj_y"), arr("level"), arr("view_cos"),
                                                  ptr(nv)), "Frame_isInFrustum_batch")
        finally:
            check(self._L.ORBmatcher_set_device_pointers(self._h, 0))
        res = []
        for o, M, k in zip(outs, maps, nv):
            n = len(M["pos"])
            r = {key: v.cpu().numpy()[:n] for key, v in o.items()}
            r["nvisible"] = int(k)
            res.append(r)
        del keep
        return res

    def SearchLocalPoints(self, frames, cur_mps, maps, logScaleFactor, th=1.0, deferred=False, nnratio=0.0):
        """Tracking::SearchLocalPoints (Tracking.cc:1143-1193): isInFrustum(pMP, 0.5) + SearchByProjection(F,
        mvpLocalMapPoints, th) per frame on the device (ORBmatcher_SearchLocalPoints_batch); cur_mps[f] (int32
        numpy, F.N) updated in place.  nnratio > 0 overrides this matcher's ratio for the call (the reference
        uses ORBmatcher(0.8), Tracking.cc:1184).  -> (nmatches, nvisible) arrays."""
        import torch
        dev = torch.device("cuda", torch.cuda.current_device())
        keep, fa, ma = self._local_batch(frames, maps, dev)
        cm = [torch.from_numpy(np.ascontiguousarray(c, np.int32) if len(c) else np.full(1, -1, np.int32)).to(dev)
              for c in cur_mps]
        arr = (C.c_void_p * max(len(cm), 1))(*[c.data_ptr() for c in cm])
        nm = np.zeros(max(len(frames), 1), np.int32)
        nv = np.zeros(max(len(frames), 1), np.int32)
        check(self._L.ORBmatcher_set_device_pointers(self._h, 1))
        try:
            if deferred:   # queued on the stream; the counts land at finish (set_deferred(0))
                check(self._L.ORBmatcher_set_deferred(self._h, 1))
            check(self._L.ORBmatcher_SearchLocalPoints_batch(self._h, len(frames), fa, arr, ma, float(logScaleFactor),
                                                             float(th), float(nnratio), ptr(nm), ptr(nv)),
                  "ORBmatcher_SearchLocalPoints_batch")
        finally:
            if deferred:
                check(self._L.ORBmatcher_set_deferred(self._h, 0))
            check(self._L.ORBmatcher_set_device_pointers(self._h, 0))
        for c, d in zip(cur_mps, cm):
            c[:] = d.cpu().numpy()[:len(c)]
        del keep
        return nm[:len(frames)], nv[:len(frames)]

    def UnprojectStereo_device(self, frames):
        """Frame::UnprojectStereo (Frame.cc:666-680) for every keypoint of device-resident frames,
        enqueued on this matcher's stream (ORBmatcher_stream): frames[f] is a dict of torch device
        tensors keysUn (N x 7 words), depth (N f32), Twc (16 f32, [Rwc | Ow]), x3D (N x 3 f32, out),
        optional mp (N i32, out), and cam = (fx, fy, cx, cy)."""
        from ._lib import orb_unproject
        us = []
        for f in frames:
            fx, fy, cx, cy = (float(v) for v in f["cam"])
            mp = f.get("mp")
            us.append(orb_unproject(int(f["depth"].numel()), f["keysUn"].data_ptr(), f["depth"].data_ptr(),
                                    f["Twc"].data_ptr(), fx, fy, cx, cy, f["x3D"].data_ptr(),
                                    mp.data_ptr() if mp is not None else None))
        arr = (orb_unproject * max(len(us), 1))(*us)
        check(self._L.Frame_UnprojectStereo_batch_device(self._h, len(us), arr), "Frame_UnprojectStereo_batch_device")

    @staticmethod
    def _undistort_struct(N, keys_ptr, out_ptr, K, dist):
        from ._lib import orb_undistort
        K = np.ascontiguousarray(K, np.float32).reshape(-1)
        dist = np.ascontiguousarray(dist, np.float32).reshape(-1)
        if K.size != 9 or dist.size not in (4, 5, 8):
            raise ValueError("K must be 3x3 and mDistCoef 4, 5 or 8 coefficients")
        u = orb_undistort()
        u.N, u.keys, u.keysUn, u.ndist = int(N), keys_ptr, out_ptr, int(dist.size)
        u.K[:] = K.tolist()
        u.dist[:dist.size] = dist.tolist()
        return u

    def UndistortKeyPoints(self, keys, K, dist):
        """Frame::UndistortKeyPoints (Frame.cc:404-430): mvKeys (KP_DTYPE) -> mvKeysUn, through
        cv::undistortPoints(pts, pts, mK, mDistCoef, Mat(), mK) on the GPU."""
        keys = np.ascontiguousarray(keys, KP_DTYPE)
        out = np.zeros(max(len(keys), 1), KP_DTYPE)
        u = self._undistort_struct(len(keys), keys.ctypes.data if len(keys) else None, out.ctypes.data, K, dist)
        check(self._L.Frame_UndistortKeyPoints(self._h, C.byref(u)), "Frame_UndistortKeyPoints")
        return out[:len(keys)]

    def UndistortKeyPoints_device(self, frames):
        """The batch form over device-resident frames, enqueued on this matcher's stream: frames[f]
        = dict(keys, keysUn (torch device tensors, N x 7 words), K (3x3), dist)."""
        from ._lib import orb_undistort
        us = [self._undistort_struct(f["keys"].shape[0], f["keys"].data_ptr(), f["keysUn"].data_ptr(), f["K"], f["dist"])
              for f in frames]
        arr = (orb_undistort * max(len(us), 1))(*us)
        check(self._L.ORBmatcher_set_device_pointers(self._h, 1))
        try:
            check(self._L.Frame_UndistortKeyPoints_batch(self._h, len(us), arr), "Frame_UndistortKeyPoints_batch")
        finally:
            check(self._L.ORBmatcher_set_device_pointers(self._h, 0))

    def ComputeImageBounds(self, cols, rows, K, dist):
        """Frame::ComputeImageBounds (Frame.cc:436-464) + the grid factors (Frame.cc:155-156) ->
        (mnMinX, mnMaxX, mnMinY, mnMaxY, mfGridElementWidthInv, mfGridElementHeightInv)."""
        K = np.ascontiguousarray(K, np.float32).reshape(-1)
        dist = np.ascontiguousarray(dist, np.float32).reshape(-1)
        b = np.zeros(6, np.float32)
        check(self._L.Frame_ComputeImageBounds(self._h, int(cols), int(rows), ptr(K), ptr(dist), int(dist.size), ptr(b)),
              "Frame_ComputeImageBounds")
        return tuple(np.float32(v) for v in b)

    def SearchByProjection_KeyFrame(self, F: Frame, cur_mp, kf_mp, skip, kf_angle, mps: MapPoints, max_dist,
                                    min_dist, logScaleFactor, th, ORBdist):
        """SearchByProjection(CurrentFrame, pKF, sAlreadyFound, th, ORBdist) (ORBmatcher.cc:1472).
        cur_mp is updated in place; returns nmatches."""
        assert cur_mp.dtype == np.int32 and cur_mp.flags.c_contiguous and len(cur_mp) == F.N
        kf_mp = np.ascontiguousarray(kf_mp, np.int32)
        skip = np.ascontiguousarray(skip, np.uint8)
        kf_angle = np.ascontiguousarray(kf_angle, np.float32)
        mx = np.ascontiguousarray(max_dist, np.float32)
        mn = np.ascontiguousarray(min_dist, np.float32)
        f, m, n = F.cstruct(), mps.cstruct(), C.c_int()
        check(self._L.ORBmatcher_SearchByProjection_KeyFrame(self._h, C.byref(f), ptr(cur_mp), len(kf_mp), ptr(kf_mp),
                                                             ptr(skip), ptr(kf_angle), C.byref(m), ptr(mx), ptr(mn),
                                                             float(logScaleFactor), float(th), int(ORBdist),
                                                             C.byref(n)), "SearchByProjection_KeyFrame")
        return n.value

    def SearchByProjection_Sim3(self, KF: Frame, Scw, pts: MapPoints, geo: MapPointGeo, skip, matched,
                                logScaleFactor, th):
        """SearchByProjection(pKF, Scw, vpPoints, vpMatched, th) (ORBmatcher.cc:290-403).
        matched (KF.N int32, rows of pts or -1) is updated in place; returns nmatches."""
        assert matched.dtype == np.int32 and matched.flags.c_contiguous and len(matched) == KF.N
        S = np.ascontiguousarray(Scw, np.float32).reshape(16)
        skip = np.ascontiguousarray(skip, np.uint8)
        f, m, g, n = KF.cstruct(), pts.cstruct(), geo.cstruct(), C.c_int()
        check(self._L.ORBmatcher_SearchByProjection_Sim3(self._h, C.byref(f), ptr(S), C.byref(m), C.byref(g), ptr(skip),
                                                         float(logScaleFactor), int(th), ptr(matched), C.byref(n)),
              "SearchByProjection_Sim3")
        return n.value

    def Fuse(self, KF: Frame, pts: MapPoints, geo: MapPointGeo, skip, logScaleFactor, th=3.0):
        """Fuse(pKF, vpMapPoints, th) (ORBmatcher.cc:825-975) -> (nFused, best keypoint per point or -1)."""
        skip = np.ascontiguousarray(skip, np.uint8)
        best = np.full(max(pts.n, 1), -1, np.int32)
        f, m, g, n = KF.cstruct(), pts.cstruct(), geo.cstruct(), C.c_int()
        check(self._L.ORBmatcher_Fuse(self._h, C.byref(f), C.byref(m), C.byref(g), ptr(skip), float(logScaleFactor),
                                      float(th), ptr(best), C.byref(n)), "Fuse")
        return n.value, best[:pts.n]

    def Fuse_Sim3(self, KF: Frame, Scw, pts: MapPoints, geo: MapPointGeo, skip, logScaleFactor, th=4.0):
        """Fuse(pKF, Scw, vpPoints, th, vpReplacePoint) (ORBmatcher.cc:977-1100) -> (nFused, best)."""
        S = np.ascontiguousarray(Scw, np.float32).reshape(16)
        skip = np.ascontiguousarray(skip, np.uint8)
        best = np.full(max(pts.n, 1), -1, np.int32)
        f, m, g, n = KF.cstruct(), pts.cstruct(), geo.cstruct(), C.c_int()
        check(self._L.ORBmatcher_Fuse_Sim3(self._h, C.byref(f), ptr(S), C.byref(m), C.byref(g), ptr(skip),
                                           float(logScaleFactor), float(th), ptr(best), C.byref(n)), "Fuse_Sim3")
        return n.value, best[:pts.n]

    def SearchBySim3(self, KF1: Frame, mp1, KF2: Frame, mp2, pts: MapPoints, geo: MapPointGeo, bad, matches12, s12,
                     R12, t12, logScaleFactor, th=7.5):
        """SearchBySim3(pKF1, pKF2, vpMatches12, s12, R12, t12, th) (ORBmatcher.cc:1102-1326).
        matches12 (KF1.N int32: -1 / KF2 keypoint / -2) is updated in place; returns nFound."""
        assert matches12.dtype == np.int32 and matches12.flags.c_contiguous and len(matches12) == KF1.N
        mp1, mp2 = np.ascontiguousarray(mp1, np.int32), np.ascontiguousarray(mp2, np.int32)
        bad = np.ascontiguousarray(bad, np.uint8)
        R = np.ascontiguousarray(R12, np.float32).reshape(9)
        t = np.ascontiguousarray(t12, np.float32).reshape(3)
        f1, f2, m, g, n = KF1.cstruct(), KF2.cstruct(), pts.cstruct(), geo.cstruct(), C.c_int()
        check(self._L.ORBmatcher_SearchBySim3(self._h, C.byref(f1), ptr(mp1), C.byref(f2), ptr(mp2), C.byref(m),
                                              C.byref(g), ptr(bad), float(s12), ptr(R), ptr(t), float(logScaleFactor),
                                              float(th), ptr(matches12), C.byref(n)), "SearchBySim3")
        return n.value

    def SearchForInitialization(self, F1: Frame, F2: Frame, prev_matched, windowSize=10):
        """SearchForInitialization(F1, F2, vbPrevMatched, vnMatches12, windowSize) (ORBmatcher.cc:405).
        prev_matched (N1 x 2 float32) is updated in place; returns (nmatches, vnMatches12)."""
        assert prev_matched.dtype == np.float32 and prev_matched.flags.c_contiguous
        m12 = np.full(max(F1.N, 1), -1, np.int32)
        f1, f2, n = F1.cstruct(), F2.cstruct(), C.c_int()
        check(self._L.ORBmatcher_SearchForInitialization(self._h, C.byref(f1), C.byref(f2), ptr(prev_matched),
                                                         ptr(m12), int(windowSize), C.byref(n)),
              "SearchForInitialization")
        return n.value, m12[:F1.N]

    def SearchByBoW_Frame(self, kf_desc, kf_angle, kf_mp, kf_mp_bad, fvKF: FeatureVector, f_desc, f_angle,
                          fvF: FeatureVector):
        """SearchByBoW(pKF, F, vpMapPointMatches) (ORBmatcher.cc:159) -> (nmatches, matches[NF])."""
        kd = np.ascontiguousarray(kf_desc, np.uint8).reshape(-1, 32)
        fd = np.ascontiguousarray(f_desc, np.uint8).reshape(-1, 32)
        ka = np.ascontiguousarray(kf_angle, np.float32)
        fa = np.ascontiguousarray(f_angle, np.float32)
        km = np.ascontiguousarray(kf_mp, np.int32)
        kb = np.ascontiguousarray(kf_mp_bad, np.uint8)
        out = np.full(max(len(fd), 1), -1, np.int32)
        v1, v2, n = fvKF.cstruct(), fvF.cstruct(), C.c_int()
        check(self._L.ORBmatcher_SearchByBoW_Frame(self._h, len(kd), ptr(kd), ptr(ka), ptr(km), ptr(kb), C.byref(v1),
                                                   len(fd), ptr(fd), ptr(fa), C.byref(v2), ptr(out), C.byref(n)),
              "SearchByBoW_Frame")
        return n.value, out[:len(fd)]

    def SearchByBoW_KeyFrames(self, desc1, angle1, mp1, bad1, fv1: FeatureVector, desc2, angle2, mp2, bad2,
                              fv2: FeatureVector):
        """SearchByBoW(pKF1, pKF2, vpMatches12) (ORBmatcher.cc:522) -> (nmatches, matches12[n1])."""
        d1 = np.ascontiguousarray(desc1, np.uint8).reshape(-1, 32)
        d2 = np.ascontiguousarray(desc2, np.uint8).reshape(-1, 32)
        a1, a2 = np.ascontiguousarray(angle1, np.float32), np.ascontiguousarray(angle2, np.float32)
        m1, m2 = np.ascontiguousarray(mp1, np.int32), np.ascontiguousarray(mp2, np.int32)
        b1, b2 = np.ascontiguousarray(bad1, np.uint8), np.ascontiguousarray(bad2, np.uint8)
        out = np.full(max(len(d1), 1), -1, np.int32)
        v1, v2, n = fv1.cstruct(), fv2.cstruct(), C.c_int()
        check(self._L.ORBmatcher_SearchByBoW_KeyFrames(self._h, len(d1), ptr(d1), ptr(a1), ptr(m1), ptr(b1),
                                                       C.byref(v1), len(d2), ptr(d2), ptr(a2), ptr(m2), ptr(b2),
                                                       C.byref(v2), ptr(out), C.byref(n)), "SearchByBoW_KeyFrames")
        return n.value, out[:len(d1)]

    def SearchForTriangulation(self, KF1: Frame, has_mp1, fv1: FeatureVector, KF2: Frame, has_mp2,
                               fv2: FeatureVector, levelSigma2_2, F12, bOnlyStereo=False):
        """SearchForTriangulation(pKF1, pKF2, F12, vMatchedPairs, bOnlyStereo) (ORBmatcher.cc:657)
        -> array (n, 2) of (idx1, idx2)."""
        h1 = np.ascontiguousarray(has_mp1, np.uint8)
        h2 = np.ascontiguousarray(has_mp2, np.uint8)
        s2 = np.ascontiguousarray(levelSigma2_2, np.float32)
        F = np.ascontiguousarray(F12, np.float32).reshape(3, 3)
        cap = max(KF1.N, 1)
        pairs = np.zeros((cap, 2), np.int32)
        k1, k2, v1, v2, n = KF1.cstruct(), KF2.cstruct(), fv1.cstruct(), fv2.cstruct(), C.c_int()
        check(self._L.ORBmatcher_SearchForTriangulation(self._h, C.byref(k1), ptr(h1), C.byref(v1), C.byref(k2),
                                                        ptr(h2), C.byref(v2), ptr(s2), ptr(F), int(bool(bOnlyStereo)),
                                                        ptr(pairs), cap, C.byref(n)), "SearchForTriangulation")
        return pairs[:n.value].copy()

    def SearchCandidates(self, qdesc, tdesc, offsets, cand):
        q = np.ascontiguousarray(qdesc, np.uint8).reshape(-1, 32)
        t = np.ascontiguousarray(tdesc, np.uint8).reshape(-1, 32)
        off = np.ascontiguousarray(offsets, np.int32)
        c = np.ascontiguousarray(cand, np.int32)
        nq = len(q)
        dist = np.zeros(max(len(c), 1), np.int32)
        bi, bd, sd = (np.zeros(max(nq, 1), np.int32) for _ in range(3))
        check(self._L.ORBmatcher_SearchCandidates(self._h, ptr(q), nq, ptr(t), len(t), ptr(off), ptr(c), ptr(dist),
                                                  ptr(bi), ptr(bd), ptr(sd)), "SearchCandidates")
        return dist[:len(c)], bi[:nq], bd[:nq], sd[:nq]
