"""ctypes binding of liborbslam_gpu.so (the C ABI in include/orbslam_gpu.h).

The product path is the HIP library: if it is missing or no GPU is usable the
calls fail loudly (ORB_E_NODEVICE / ImportError) -- there is no CPU fallback.
"""
import ctypes as C
import os
import re
from pathlib import Path

import numpy as np

PKG = Path(__file__).resolve().parent
ROOT = PKG.parent
# ORBGPU_LIB: an instrumented build (make -C c_orb_slam_amd/csrc prof) for tools/ only
LIB_PATH = Path(os.environ["ORBGPU_LIB"]) if os.environ.get("ORBGPU_LIB") else PKG / "liborbslam_gpu.so"
HEADER = ROOT / "include" / "orbslam_gpu.h"

ORB_OK, ORB_E_INVALID, ORB_E_HIP, ORB_E_CAPACITY, ORB_E_NODEVICE = 0, -1, -2, -3, -4
_ERR = {ORB_E_INVALID: "ORB_E_INVALID", ORB_E_HIP: "ORB_E_HIP", ORB_E_CAPACITY: "ORB_E_CAPACITY",
        ORB_E_NODEVICE: "ORB_E_NODEVICE"}

KP_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
                     ("response", "<f4"), ("octave", "<i4"), ("class_id", "<i4")])
assert KP_DTYPE.itemsize == 28


class OrbGpuError(RuntimeError):
    def __init__(self, code, what=""):
        super().__init__(f"{what}: {_ERR.get(code, code)}")
        self.code = code


def check(rc, what=""):
    if rc != ORB_OK:
        raise OrbGpuError(rc, what)
    return rc


class orb_frame(C.Structure):
    _fields_ = [("N", C.c_int), ("keysUn", C.c_void_p), ("desc", C.c_void_p), ("uRight", C.c_void_p),
                ("minX", C.c_float), ("maxX", C.c_float), ("minY", C.c_float), ("maxY", C.c_float),
                ("gridWInv", C.c_float), ("gridHInv", C.c_float), ("scaleFactors", C.c_void_p),
                ("nlevels", C.c_int), ("fx", C.c_float), ("fy", C.c_float), ("cx", C.c_float),
                ("cy", C.c_float), ("bf", C.c_float), ("b", C.c_float), ("Tcw", C.c_void_p)]


class orb_featvec(C.Structure):
    _fields_ = [("n_nodes", C.c_int), ("node_id", C.c_void_p), ("start", C.c_void_p), ("feat", C.c_void_p)]


class orb_mappoint_geo(C.Structure):
    _fields_ = [("max_dist", C.c_void_p), ("min_dist", C.c_void_p), ("normal", C.c_void_p)]


class orb_mappoints(C.Structure):
    _fields_ = [("n", C.c_int), ("pos", C.c_void_p), ("desc", C.c_void_p), ("observations", C.c_void_p)]


class orb_newpoints(C.Structure):
    _fields_ = [("N", C.c_int), ("keysUn", C.c_void_p), ("depth", C.c_void_p), ("Twc", C.c_void_p),
                ("fx", C.c_float), ("fy", C.c_float), ("cx", C.c_float), ("cy", C.c_float),
                ("scaleFactors", C.c_void_p), ("nlevels", C.c_int), ("row_base", C.c_int32), ("x3D", C.c_void_p),
                ("row", C.c_void_p), ("normal", C.c_void_p), ("max_dist", C.c_void_p), ("min_dist", C.c_void_p)]


class orb_localprep(C.Structure):
    _fields_ = [("N", C.c_int), ("cur_mp", C.c_void_p), ("outlier", C.c_void_p), ("n", C.c_int),
                ("row", C.c_void_p), ("skip", C.c_void_p)]


class orb_localmap(C.Structure):
    _fields_ = [("n", C.c_int), ("pos", C.c_void_p), ("desc", C.c_void_p), ("observations", C.c_void_p),
                ("max_dist", C.c_void_p), ("min_dist", C.c_void_p), ("normal", C.c_void_p), ("skip", C.c_void_p)]


def header_functions(path=HEADER):
    """Names of every function the public header declares."""
    txt = re.sub(r"/\*.*?\*/", "", Path(path).read_text(), flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[A-Za-z_][\w\s\*]*?\b([A-Za-z_]\w*)\s*\(", txt, flags=re.M))
                  - {"if", "while", "for", "return", "sizeof"})


_lib = None


class _MissingSymbol:
    """A symbol an older tools build (ORBGPU_LIB) does not export: binding it is a no-op, calling it fails."""

    def __init__(self, name):
        self.__dict__["name"] = name

    def __setattr__(self, k, v):
        pass

    def __call__(self, *a):
        raise AttributeError(f"{LIB_PATH} does not export {self.name}")


class _ToolsCDLL(C.CDLL):
    def __getattr__(self, name):
        try:
            return super().__getattr__(name)
        except AttributeError:
            if name.startswith("__"):
                raise
            return _MissingSymbol(name)


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not LIB_PATH.exists():
        raise ImportError(f"{LIB_PATH} not built: run `python -c 'import __graft_entry__ as g; g.build()'`")
    # the product library must export every binding below; a tools build given by ORBGPU_LIB (an
    # instrumented or older build for A/B timing) may lack newer entry points
    L = (_ToolsCDLL if os.environ.get("ORBGPU_LIB") else C.CDLL)(str(LIB_PATH))
    vp, i32, f32, sz = C.c_void_p, C.c_int, C.c_float, C.c_size_t
    P = C.POINTER
    L.orbgpu_version.restype = C.c_char_p
    L.ORBextractor_create.argtypes = [i32, f32, i32, i32, i32, i32, i32, i32, P(vp)]
    L.ORBextractor_destroy.argtypes = [vp]
    L.ORBextractor_extract.argtypes = [vp, vp, i32, i32, i32, vp, vp, i32, P(i32)]
    L.ORBextractor_extract_batch.argtypes = [vp, vp, i32, i32, i32, i32, sz, i32, vp, vp, i32, i32, vp]
    L.ORBextractor_extract_images.argtypes = [vp, vp, i32, i32, i32, i32, vp, vp, i32, i32, vp]
    L.ORBextractor_get_level.argtypes = [vp, i32, i32, vp, i32, P(i32), P(i32)]
    L.ORBextractor_get_blurred_level.argtypes = [vp, i32, i32, vp, i32, P(i32), P(i32)]
    L.ORBextractor_get_levels.argtypes = [vp, P(i32), P(f32)]
    L.ORBextractor_get_scale_tables.argtypes = [vp, vp, vp, vp, vp, vp]
    L.ORBextractor_reserve_cus.argtypes = [vp, i32]
    L.ORBextractor_share_stream.argtypes = [vp, vp]
    L.ORBextractor_stream.restype = vp
    L.ORBextractor_stream.argtypes = [vp]
    L.ORBextractor_last_timings.argtypes = [vp, vp]
    L.ORBextractor_last_corner_count.argtypes = [vp, vp]
    L.ORBmatcher_create.argtypes = [f32, i32, P(vp)]
    L.ORBmatcher_set_deferred.argtypes = [vp, i32]
    L.ORBmatcher_finish.argtypes = [vp]
    L.ORBmatcher_chain_close.argtypes = [vp, P(C.c_longlong)]
    L.ORBmatcher_chain_wait.argtypes = [vp, C.c_longlong]
    L.ORBmatcher_chain_finish.argtypes = [vp, C.c_longlong]
    L.Optimizer_PoseOptimization_frames_device_deferred.argtypes = [vp, i32, vp, vp, vp, vp]
    L.ORBmatcher_destroy.argtypes = [vp]
    L.ORBmatcher_set_device_pointers.argtypes = [vp, i32]
    L.ORBmatcher_stream.restype = vp
    L.ORBmatcher_stream.argtypes = [vp]
    L.ORBmatcher_DescriptorDistance.argtypes = [vp, vp]
    L.ORBmatcher_SearchByProjection_LastFrame.argtypes = [vp, P(orb_frame), vp, P(orb_frame), vp, vp, vp,
                                                          P(orb_mappoints), f32, i32, P(i32)]
    L.ORBmatcher_SearchByProjection_LastFrame_batch.argtypes = [vp, i32, vp, vp, vp, vp, vp, vp, vp, f32, i32, vp]
    L.ORBmatcher_SearchByProjection_MapPoints.argtypes = [vp, P(orb_frame), vp, i32, vp, vp, vp, vp, vp, vp, vp,
                                                          P(orb_mappoints), f32, P(i32)]
    L.ORBmatcher_ComputeStereoMatches.argtypes = [vp, vp, vp, i32, i32, vp, vp, i32, vp, vp, f32, f32, vp, vp,
                                                  P(i32)]
    L.ORBmatcher_ComputeStereoMatches_batch.argtypes = [vp, vp, vp, i32, vp, vp, vp, vp, vp, vp, f32, f32, vp, vp,
                                                        vp]
    L.ORBmatcher_ComputeStereoMatches_batch_at.argtypes = [vp, vp, i32, vp, i32, i32, vp, vp, vp, vp, vp, vp, f32, f32,
                                                           vp, vp, vp]
    L.ORBmatcher_SearchByProjection_KeyFrame.argtypes = [vp, P(orb_frame), vp, i32, vp, vp, vp, P(orb_mappoints), vp,
                                                         vp, f32, f32, i32, P(i32)]
    L.ORBmatcher_SearchForInitialization.argtypes = [vp, P(orb_frame), P(orb_frame), vp, vp, i32, P(i32)]
    L.ORBmatcher_SearchByBoW_Frame.argtypes = [vp, i32, vp, vp, vp, vp, P(orb_featvec), i32, vp, vp, P(orb_featvec),
                                               vp, P(i32)]
    L.ORBmatcher_SearchByBoW_KeyFrames.argtypes = [vp, i32, vp, vp, vp, vp, P(orb_featvec), i32, vp, vp, vp, vp,
                                                   P(orb_featvec), vp, P(i32)]
    L.ORBmatcher_SearchForTriangulation.argtypes = [vp, P(orb_frame), vp, P(orb_featvec), P(orb_frame), vp,
                                                    P(orb_featvec), vp, vp, i32, vp, i32, P(i32)]
    L.ORBmatcher_SearchByProjection_Sim3.argtypes = [vp, P(orb_frame), vp, P(orb_mappoints), P(orb_mappoint_geo), vp,
                                                     f32, i32, vp, P(i32)]
    L.ORBmatcher_Fuse.argtypes = [vp, P(orb_frame), P(orb_mappoints), P(orb_mappoint_geo), vp, f32, f32, vp, P(i32)]
    L.ORBmatcher_Fuse_Sim3.argtypes = [vp, P(orb_frame), vp, P(orb_mappoints), P(orb_mappoint_geo), vp, f32, f32, vp,
                                       P(i32)]
    L.ORBmatcher_SearchBySim3.argtypes = [vp, P(orb_frame), vp, P(orb_frame), vp, P(orb_mappoints),
                                          P(orb_mappoint_geo), vp, f32, vp, vp, f32, f32, vp, P(i32)]
    L.ORBmatcher_SearchCandidates.argtypes = [vp, vp, i32, vp, i32, vp, vp, vp, vp, vp, vp]
    L.orb_rng_seed.argtypes = [vp, C.c_uint]
    L.orb_rng_rand.argtypes = [vp]
    L.PnPsolver_create.argtypes = [i32, vp, vp, vp, vp, i32, f32, f32, f32, f32, P(vp)]
    L.PnPsolver_destroy.argtypes = [vp]
    L.PnPsolver_set_ransac.argtypes = [vp, C.c_double, i32, i32, i32, f32, f32]
    L.PnPsolver_iterate.argtypes = [vp, i32, vp, P(i32), vp, P(i32), vp, P(i32)]
    L.PnPsolver_iterate_batch.argtypes = [i32, vp, i32, vp, vp, vp, vp, vp, vp]
    L.PnPsolver_get_state.argtypes = [vp, P(i32), P(i32), P(i32)]
    L.PnPsolver_enable_timing.argtypes = [i32]
    L.PnPsolver_last_timings.argtypes = [vp, vp]
    L.Optimizer_LocalBundleAdjustment.argtypes = [vp, vp, vp]
    L.Optimizer_BundleAdjustment.argtypes = [vp, i32, i32, vp, vp]
    L.Optimizer_LocalBundleAdjustment_sharded.argtypes = [vp, vp, vp, vp]
    L.Optimizer_BundleAdjustment_sharded.argtypes = [vp, vp, i32, i32, vp, vp]
    L.Optimizer_partition_points.argtypes = [vp, i32, vp]
    L.Optimizer_partition_points_nd.argtypes = [vp, i32, vp, vp]
    L.Optimizer_last_sharding.argtypes = [vp]
    L.Optimizer_last_lm_path.argtypes = [vp]
    L.orbgpu_comm_unique_id.argtypes = [vp]
    L.orbgpu_comm_init_rccl.argtypes = [i32, i32, vp, P(vp)]
    L.orbgpu_comm_init_local.argtypes = [i32, vp]
    L.orbgpu_comm_init_shm.argtypes = [C.c_char_p, i32, i32, C.c_size_t, P(vp)]
    L.orbgpu_comm_rank.argtypes = [vp, P(i32), P(i32)]
    L.orbgpu_comm_destroy.argtypes = [vp]
    L.Optimizer_last_trace.argtypes = [vp, vp, i32, P(i32), vp, vp, i32, P(i32)]
    L.Optimizer_last_timings.argtypes = [vp]
    L.Optimizer_PoseOptimization.argtypes = [P(pose_problem), vp, vp, P(i32)]
    L.Optimizer_PoseOptimization_batch.argtypes = [i32, vp, vp, vp, vp]
    L.Optimizer_PoseOptimization_batch_device.argtypes = [i32, vp, vp, vp, vp]
    L.Optimizer_OptimizeSim3.argtypes = [vp, vp, vp, P(i32)]
    L.Optimizer_OptimizeSim3_batch.argtypes = [i32, vp, vp, vp, vp]
    L.Optimizer_PoseOptimization_frames_device.argtypes = [i32, vp, vp, vp, vp]
    L.Optimizer_pose_timing.argtypes = [i32, vp]
    L.orbgpu_unit_ba_struct.argtypes = [i32, i32, i32, vp, vp, vp, vp, vp, vp, i32, vp, C.c_longlong]
    L.Frame_UnprojectStereo_batch_device.argtypes = [vp, i32, vp]
    L.Frame_UndistortKeyPoints.argtypes = [vp, vp]
    L.Frame_UndistortKeyPoints_batch.argtypes = [vp, i32, vp]
    L.Frame_ComputeImageBounds.argtypes = [vp, i32, i32, vp, vp, i32, vp]
    L.ORBvocabulary_create.argtypes = [P(vp)]
    L.ORBvocabulary_destroy.argtypes = [vp]
    L.ORBvocabulary_loadFromTextFile.argtypes = [vp, C.c_char_p]
    L.ORBvocabulary_info.argtypes = [vp, vp, vp, vp, vp, vp, vp]
    L.ORBvocabulary_transform.argtypes = [vp, vp, i32, i32, vp]
    L.ORBvocabulary_transform_batch.argtypes = [vp, i32, vp, vp, i32, vp]
    L.ORBvocabulary_transform_features.argtypes = [vp, vp, i32, i32, vp, vp, vp]
    L.ORBvocabulary_score.argtypes = [vp, vp, vp, i32, i32, vp, vp, vp, vp]
    L.orbgpu_unit_ldlt_solve.argtypes = [i32, vp, vp, vp, i32, P(i32)]
    L.orbgpu_unit_csum.argtypes = [vp, i32, vp]
    L.orbgpu_unit_pnp_layout.argtypes = [i32, vp, vp, vp, vp]
    L.MapPoint_CreateStereo_batch_device.argtypes = [vp, i32, vp]
    L.Tracking_PrepareLocalSearch_batch_device.argtypes = [vp, i32, vp]
    L.ORBmatcher_SearchDense_batch.argtypes = [vp, i32, vp, vp, vp, vp, vp, vp, vp]
    L.ORBmatcher_last_dense_timing.argtypes = [vp, vp, vp]
    L.ORBmatcher_SearchLocalPoints_batch.argtypes = [vp, i32, vp, vp, vp, f32, f32, f32, vp, vp]
    L.Frame_isInFrustum_batch.argtypes = [vp, i32, vp, vp, f32, f32, vp, vp, vp, vp, vp, vp, vp]
    L.ORBmatcher_enable_timing.argtypes = [vp, i32]
    L.ORBmatcher_last_timings.argtypes = [vp, vp, vp]
    L.orbgpu_unit_ldlt_factor.argtypes = [i32, vp, vp]
    L.orbgpu_unit_wave_tree.argtypes = [vp, vp]
    L.orbgpu_unit_shared_div.argtypes = [vp, vp, i32, vp]
    L.orbgpu_unit_set_csum_lds_max.argtypes = [i32]
    L.orbgpu_unit_set_scale_small_max.argtypes = [i32]
    L.orbgpu_unit_set_struct_gpu_min_edges.argtypes = [i32]
    L.orbgpu_unit_set_posegraph_check.argtypes = [i32]
    L.orbgpu_unit_ba_struct_all.argtypes = [i32, i32, i32, vp, vp, vp, vp, vp, vp, i32, i32, vp, C.c_longlong, vp]
    L.orbgpu_unit_nd_order.argtypes = [i32, vp, vp, i32, vp, vp, vp]
    L.orbgpu_debug_prof.argtypes = [vp]
    L.orbgpu_debug_prof_match.argtypes = [vp]
    L.orbgpu_debug_prof_extract.argtypes = [vp]
    L.Sim3Solver_create.argtypes = [i32, vp, vp, vp, vp, vp, i32, vp, vp, i32, P(vp)]
    L.Sim3Solver_destroy.argtypes = [vp]
    L.Sim3Solver_set_ransac.argtypes = [vp, C.c_double, i32, i32]
    L.Sim3Solver_iterate.argtypes = [vp, i32, vp, P(i32), vp, P(i32), vp, P(i32)]
    L.Sim3Solver_iterate_batch.argtypes = [i32, vp, i32, vp, vp, vp, vp, vp, vp]
    L.Sim3Solver_get_estimate.argtypes = [vp, vp, vp, vp]
    L.Sim3Solver_get_state.argtypes = [vp, P(i32), P(i32), P(i32)]
    L.Sim3Solver_enable_timing.argtypes = [i32]
    L.Sim3Solver_last_timings.argtypes = [vp, vp]
    _lib = L
    return L


class orb_rng(C.Structure):
    _fields_ = [("tbl", C.c_int32 * 31), ("f", C.c_int32), ("r", C.c_int32)]


def ptr(a):
    return None if a is None else C.c_void_p(a.ctypes.data)


def device_available():
    return bool(lib().orbgpu_device_available())


class ba_problem(C.Structure):
    _fields_ = [("n_kf", C.c_int), ("kf_id", C.c_void_p), ("kf_Tcw", C.c_void_p), ("kf_local", C.c_void_p),
                ("kf_cam", C.c_void_p), ("n_pt", C.c_int), ("pt_id", C.c_void_p), ("pt_pos", C.c_void_p),
                ("n_edge", C.c_int), ("edge_pt", C.c_void_p), ("edge_kf", C.c_void_p), ("edge_obs", C.c_void_p),
                ("edge_inv_sigma2", C.c_void_p)]


class orb_unproject(C.Structure):
    _fields_ = [("N", C.c_int), ("keysUn", C.c_void_p), ("depth", C.c_void_p), ("Twc", C.c_void_p),
                ("fx", C.c_float), ("fy", C.c_float), ("cx", C.c_float), ("cy", C.c_float),
                ("x3D", C.c_void_p), ("mp", C.c_void_p)]


class orb_undistort(C.Structure):
    _fields_ = [("N", C.c_int), ("keys", C.c_void_p), ("keysUn", C.c_void_p), ("K", C.c_float * 9),
                ("dist", C.c_float * 8), ("ndist", C.c_int)]


class orb_bow(C.Structure):
    _fields_ = [("cap", C.c_int), ("word", C.c_void_p), ("value", C.c_void_p), ("n_words", C.c_int),
                ("fv_node", C.c_void_p), ("fv_start", C.c_void_p), ("fv_feat", C.c_void_p), ("n_nodes", C.c_int)]


class pose_frame(C.Structure):
    _fields_ = [("N", C.c_int), ("Tcw", C.c_void_p), ("mp", C.c_void_p), ("mp_pos", C.c_void_p),
                ("keysUn", C.c_void_p), ("uRight", C.c_void_p), ("invLevelSigma2", C.c_void_p),
                ("nlevels", C.c_int), ("fx", C.c_float), ("fy", C.c_float), ("cx", C.c_float),
                ("cy", C.c_float), ("bf", C.c_float)]


class pose_problem(C.Structure):
    _fields_ = [("N", C.c_int), ("Tcw", C.c_void_p), ("has_mp", C.c_void_p), ("Xw", C.c_void_p),
                ("obs", C.c_void_p), ("inv_sigma2", C.c_void_p), ("fx", C.c_float), ("fy", C.c_float),
                ("cx", C.c_float), ("cy", C.c_float), ("bf", C.c_float)]


class sim3opt_problem(C.Structure):
    _fields_ = [("N", C.c_int), ("valid", C.c_void_p), ("X1c", C.c_void_p), ("X2c", C.c_void_p),
                ("obs1", C.c_void_p), ("obs2", C.c_void_p), ("inv_sigma2_1", C.c_void_p),
                ("inv_sigma2_2", C.c_void_p), ("K1", C.c_float * 4), ("K2", C.c_float * 4), ("th2", C.c_float),
                ("bFixScale", C.c_int)]


class ba_result(C.Structure):
    _fields_ = [("kf_Tcw", C.c_void_p), ("pt_pos", C.c_void_p), ("edge_erase", C.c_void_p),
                ("iterations", C.c_int32 * 2), ("n_erased", C.c_int32), ("aborted", C.c_int32)]
