#!/usr/bin/env python3
"""Config-5 global BA over R in-process ranks on ONE device (the RCCL protocol through the
in-process transport): wall time per BundleAdjustment(10) call with the keyframe-block
partition (replicated factorisation: every rank factors the whole pose system) and with the
separator-tree partition (sharded factorisation).  The ranks share the GPU, so the wall time
tracks the TOTAL device work of all ranks: what the sharded factorisation removes is the
(R - 1) extra copies of the subtree factorisation.  usage: gba_sharded_timing.py [nkf:laps] [R...]"""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))

from ba_cases import global_ba_problem  # noqa: E402


def main():
    from c_orb_slam_amd.optimizer import partition_points_nd, run_sharded_local
    spec = sys.argv[1] if len(sys.argv) > 1 else "2000:4"
    nkf, _, lp = spec.partition(":")
    nkf, laps = int(nkf), int(lp or 0)
    ranks = [int(a) for a in sys.argv[2:]] or [2, 4, 8]
    pr = global_ba_problem(0, n_kf=nkf, pts_per_kf=150, laps=laps)
    for R in ranks:
        _, kfo = partition_points_nd(pr, R, with_kf_owner=True)
        for part in ("block", "nd"):
            run_sharded_local(pr, R, "global", 10, False, partition=part)   # warm-up
            t0 = time.perf_counter()
            reps = 2
            for _ in range(reps):
                s, per = run_sharded_local(pr, R, "global", 10, False, partition=part)
            dt = (time.perf_counter() - t0) / reps
            sh = per[0]["sharding"]
            print(f"nkf {nkf} laps {laps} R {R} partition {part}: {dt * 1e3:.1f} ms/call (all ranks on one GPU), "
                  f"its {s['iterations'][0]}, sharded factorisation {sh[0]}, separator tiles {sh[1]} / pattern tiles "
                  f"{sh[3]}, separator rows {sh[2]}; separator poses {(kfo == -1).sum()}, rank poses "
                  f"{[int((kfo == q).sum()) for q in range(R)]}", flush=True)


if __name__ == "__main__":
    main()
