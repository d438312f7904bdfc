"""c_orb_slam_amd -- MI355X-native ORB-SLAM2 per-frame hot path.

Host mirror (Python, over the C ABI of include/orbslam_gpu.h) of the reference
junejunejune/c_orb_slam classes on the hot path.  All compute runs in the HIP
library liborbslam_gpu.so (gfx950); there is no CPU fallback.
"""
from ._lib import KP_DTYPE, OrbGpuError, device_available, lib  # noqa: F401
from .orb import FeatureVector, Frame, MapPoints, ORBextractor, ORBmatcher  # noqa: F401
from .optimizer import (BundleAdjustment, LocalBundleAdjustment, OptimizeSim3, OptimizeSim3Batch,  # noqa: F401
                        PoseOptimization, PoseOptimizationBatch)

__all__ = ["ORBextractor", "ORBmatcher", "Frame", "MapPoints", "KP_DTYPE", "OrbGpuError",
           "device_available", "lib"]
from .vocabulary import BowVector, ORBVocabulary  # noqa: F401
