#!/usr/bin/env python3
"""Section timers of k_schur's block 0 (the first diagonal block) over local-BA calls (or global-BA
calls: second argument "gba"), from an instrumented build:
ORBGPU_LIB=build/liborbslam_gpu_prof.so python tools/schur_prof.py [calls] [gba]."""
import ctypes as C
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))

from ba_cases import ba_problem  # noqa: E402
from c_orb_slam_amd._lib import lib  # noqa: E402

KEYS = ("kf_id", "kf_Tcw", "kf_local", "kf_cam", "pt_id", "pt_pos", "edge_pt", "edge_kf", "edge_obs",
        "edge_inv_sigma2")


def main():
    from c_orb_slam_amd.optimizer import LocalBundleAdjustment, BundleAdjustment
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    gba = len(sys.argv) > 2 and sys.argv[2] == "gba"   # config 5 (2000 keyframes, 4 laps) instead
    if gba:
        from ba_cases import global_ba_problem
        pr = global_ba_problem(0, n_kf=2000, pts_per_kf=150, laps=4)
        run = lambda: BundleAdjustment(pr, 10, False)  # noqa: E731
    else:
        pr = ba_problem(0)
        args = [pr[k] for k in KEYS]
        run = lambda: LocalBundleAdjustment(*args)  # noqa: E731
    run()
    out = (C.c_ulonglong * 32)()
    lib().orbgpu_debug_prof(out)
    for _ in range(reps):
        run()
    lib().orbgpu_debug_prof(out)
    if gba:   # the many-block launch: per-wave chunk-phase durations (log2 buckets from 1 k cycles)
        print("waves by chunk-phase cycles:", {f">={1 << (10 + b)}": out[b] for b in range(10)})
        print(f"chunk-phase cycles summed: diagonal-block waves {out[10]:.3g}, off-diagonal waves {out[14]:.3g}")
    n = max(out[15], 1)
    print(f"k_schur block 0 over {out[15]} launches, cycles per launch: terms+trees (wave 0) {out[11] / n:.0f} | "
          f"barrier wait {out[12] / n:.0f} | final sums {out[13] / n:.0f}")


if __name__ == "__main__":
    main()
