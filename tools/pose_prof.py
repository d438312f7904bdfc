"""Section timers of k_pose_opt (workgroup 0) from the instrumented build:
   make -C c_orb_slam_amd/csrc prof && ORBGPU_LIB=build/liborbslam_gpu_prof.so python tools/pose_prof.py"""
import ctypes as C
import sys

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
from c_orb_slam_amd import PoseOptimizationBatch  # noqa: E402
from c_orb_slam_amd._lib import lib  # noqa: E402
from pose_cases import pose_problem  # noqa: E402

# argv: keypoints per frame, fraction with a map point (the bench's batch: ~1200 and ~0.45)
N = int(sys.argv[1]) if len(sys.argv) > 1 else 1500
mp = float(sys.argv[2]) if len(sys.argv) > 2 else 0.7
frames = [pose_problem(s, N=N, mp_frac=mp) for s in range(64)]
PoseOptimizationBatch(frames)
out = (C.c_ulonglong * 32)()
lib().orbgpu_debug_prof(out)
PoseOptimizationBatch(frames)
lib().orbgpu_debug_prof(out)
names = ["iter_top", "fused28", "solve_tail_sync", "cand_pass", "decide", "to_solve_done", "unused6", "unused7"]
v = [out[i] for i in range(len(names))]
tot = sum(v)
print("cycles (frame 0, one call):", dict(zip(names, v)), "total", tot)
print({n: round(x / tot, 3) for n, x in zip(names, v)})
print("28-sum passes", out[8], "rounds (solve + candidate pass)", out[9], "round start", out[10])
