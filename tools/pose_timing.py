"""Time Optimizer_PoseOptimization_batch: F KITTI-shaped frames (~N*mp_frac edges) per launch."""
import sys
import time

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
import numpy as np  # noqa: E402

from c_orb_slam_amd import PoseOptimizationBatch  # noqa: E402
from pose_cases import pose_problem  # noqa: E402

Fs = [int(a) for a in sys.argv[1:]] or [1, 64, 256]
for F in Fs:
    frames = [pose_problem(s, N=2000) for s in range(F)]
    PoseOptimizationBatch(frames)
    t = time.perf_counter()
    reps = 5
    for _ in range(reps):
        PoseOptimizationBatch(frames)
    dt = (time.perf_counter() - t) / reps
    print(f"F={F}: {dt*1e3:.2f} ms/launch  {F/dt:.0f} frames/s", flush=True)
