#!/usr/bin/env python3
"""Local BA throughput over S concurrent streams (bench.py's local_ba.value shape) and one stream."""
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))

from ba_cases import ba_problem  # noqa: E402

KEYS = ("kf_id", "kf_Tcw", "kf_local", "kf_cam", "pt_id", "pt_pos", "edge_pt", "edge_kf", "edge_obs",
        "edge_inv_sigma2")


def main():
    from c_orb_slam_amd.optimizer import LocalBundleAdjustment
    S = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 60
    pr = ba_problem(0)
    a = [pr[k] for k in KEYS]

    def stream(_):
        return sum(sum(LocalBundleAdjustment(*a)["iterations"]) for _ in range(reps))
    with ThreadPoolExecutor(S) as ex:
        list(ex.map(lambda i: LocalBundleAdjustment(*a), range(S)))
        t0 = time.perf_counter()
        its = sum(ex.map(stream, range(S)))
        dt = time.perf_counter() - t0
    t0 = time.perf_counter()
    its1 = stream(0)
    dt1 = time.perf_counter() - t0
    print(f"streams {S}: {its / dt:.1f} iter/s; single: {its1 / dt1:.1f} iter/s "
          f"(ORBGPU_STRUCT_SMALL={os.environ.get('ORBGPU_STRUCT_SMALL', '')})")


if __name__ == "__main__":
    main()
