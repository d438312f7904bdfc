#!/usr/bin/env python3
"""Time GPU local BA on SURVEY config 4 (EuRoC-shaped, 15+15 KFs, 3000 points) and the oracle."""
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))

from ba_cases import ba_problem  # noqa: E402

KEYS = ("kf_id", "kf_Tcw", "kf_local", "kf_cam", "pt_id", "pt_pos", "edge_pt", "edge_kf", "edge_obs",
        "edge_inv_sigma2")


def main():
    from c_orb_slam_amd.optimizer import LocalBundleAdjustment, last_timings
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    pr = ba_problem(0)
    args = [pr[k] for k in KEYS]
    for _ in range(3):
        g = LocalBundleAdjustment(*args)
    t0 = time.perf_counter()
    its = 0
    for _ in range(reps):
        g = LocalBundleAdjustment(*args, trace=True)
        its += sum(g["iterations"])
    dt = time.perf_counter() - t0
    ms = last_timings()
    print(f"gpu: {reps} LBA calls, {its} solves, {dt / reps * 1e3:.2f} ms/call, {its / dt:.1f} iter/s, "
          f"trials/call {len(g['trial_chi2'])}, struct {ms[1]:.2f} ms, total(host clock) {ms[0]:.2f} ms")
    import oracle_lib
    t0 = time.perf_counter()
    o = oracle_lib.oracle_local_ba(pr)
    dt = time.perf_counter() - t0
    print(f"oracle: {dt * 1e3:.1f} ms/call, {sum(o['iterations']) / dt:.1f} iter/s")


if __name__ == "__main__":
    main()
