#!/usr/bin/env python3
"""One config-5 sharded global BA run for tools/gba_rank_model.py: R in-process ranks with the
separator-tree partition, a warm-up call then one measured call (each call on fresh rank
threads); prints the exchange volume per trial and the LM trial count of the measured call.
With mode "local": SURVEY config 4 (Optimizer::LocalBundleAdjustment, 15 local + 15 fixed
keyframes, 3,000 points) keyframe-block sharded over R ranks instead.
usage: gba_rank_run.py <R> [nkf:laps] [global|local]"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
from ba_cases import ba_problem, global_ba_problem  # noqa: E402


def main():
    from c_orb_slam_amd.optimizer import partition_points_nd, run_sharded_local
    R = int(sys.argv[1])
    spec = sys.argv[2] if len(sys.argv) > 2 else "2000:4"
    if len(sys.argv) > 3 and sys.argv[3] == "local":
        pr = ba_problem(0)
        run_sharded_local(pr, R, "local", partition="block")   # warm-up
        s, per = run_sharded_local(pr, R, "local", partition="block", trace=True)
        n = 6 * int((pr["kf_local"] != 0).sum())
        nt = (n + 63) // 64
        # per trial: the union-pattern 64 x 64 tiles of the dense S + b_s; per iteration
        # {Hpp, b_p, chi2} and the trial scalars (about n * 4.5 + 8 doubles, folded in)
        xd = nt * (nt + 1) // 2 * 4096 + n + (n * 9) // 2 + 8 if R > 1 else 0
        its = s["iterations"]
        print(f"R {R} iterations {its[0] + its[1]} trials {len(s['trial_chi2'])} exchange_doubles_per_trial {xd} "
              f"sharded_factorisation 0 separator_tiles 0 pattern_tiles {nt * (nt + 1) // 2}", flush=True)
        return
    nkf, _, lp = spec.partition(":")
    pr = global_ba_problem(0, n_kf=int(nkf), pts_per_kf=150, laps=int(lp or 0))
    part = "nd" if R > 1 else "block"
    run_sharded_local(pr, R, "global", 10, False, partition=part)   # warm-up
    s, per = run_sharded_local(pr, R, "global", 10, False, partition=part, trace=True)
    used, tiles, rows, pattern = per[0]["sharding"]
    _, kfo = partition_points_nd(pr, R, with_kf_owner=True)
    poses = int((kfo >= -1).sum())
    xd = (tiles * 4096 + rows + 6 * poses) if used else (pattern * 4096 + 6 * poses)
    print(f"R {R} iterations {s['iterations'][0]} trials {len(s['trial_chi2'])} exchange_doubles_per_trial {xd} "
          f"sharded_factorisation {used} separator_tiles {tiles} pattern_tiles {pattern}", flush=True)


if __name__ == "__main__":
    main()
