#!/usr/bin/env python3
"""Time GPU global BA (Optimizer::BundleAdjustment, 10 its) on config-5-shaped problems of growing size."""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))

from ba_cases import global_ba_problem  # noqa: E402


def main():
    from c_orb_slam_amd.optimizer import BundleAdjustment, last_timings
    # arguments: sizes, each optionally "<kf>:<laps>" (laps -1 / omitted: one lap per 500 keyframes)
    sizes = sys.argv[1:] or ["128", "512", "1024", "2000"]
    for arg in sizes:
        nkf, _, lp = arg.partition(":")
        nkf = int(nkf)
        laps = nkf // 500 if lp in ("", "-1") else int(lp)
        t0 = time.perf_counter()
        pr = global_ba_problem(0, n_kf=nkf, pts_per_kf=150, laps=laps)
        tg = time.perf_counter() - t0
        BundleAdjustment(pr, 10, False)
        t0 = time.perf_counter()
        r = BundleAdjustment(pr, 10, False, trace=True)
        dt = time.perf_counter() - t0
        ms = last_timings()
        print(f"nkf {nkf} laps {laps}: pts {len(pr['pt_id'])} edges {len(pr['edge_pt'])} gen {tg:.1f}s | "
              f"{dt * 1e3:.1f} ms/call, its {r['iterations'][0]}, trials {len(r['trial_chi2'])}, "
              f"{r['iterations'][0] / dt:.1f} iter/s, struct {ms[1]:.1f} ms", flush=True)


if __name__ == "__main__":
    main()
