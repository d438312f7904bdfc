#!/usr/bin/env python3
"""Section timers of k_ldlt_sparse (prof build) on one global-BA call:
   make -C c_orb_slam_amd/csrc prof && ORBGPU_LIB=build/liborbslam_gpu_prof.so python tools/ldlt_prof.py [n_kf]"""
import ctypes as C
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
from ba_cases import global_ba_problem  # noqa: E402
from c_orb_slam_amd._lib import lib  # noqa: E402
from c_orb_slam_amd.optimizer import BundleAdjustment  # noqa: E402

nkf = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
pr = global_ba_problem(0, n_kf=nkf, pts_per_kf=150)
BundleAdjustment(pr, 1, False)
out = (C.c_ulonglong * 32)()
lib().orbgpu_debug_prof(out)
r = BundleAdjustment(pr, 1, False, trace=True)
lib().orbgpu_debug_prof(out)
ntr = len(r["trial_chi2"])
nt = (6 * (nkf - 1) + 63) // 64
names = ["diag", "chunks", "trail"]
v = [out[16 + i] for i in range(3)]
print(f"n_kf {nkf}: {ntr} factorisations x {nt} panels; cycles per panel:",
      {k: round(x / max(ntr * nt, 1)) for k, x in zip(names, v)})
