#!/usr/bin/env python3
"""Multi-GPU cost model of the sharded global BA (SURVEY config 5) from rocprofv3
kernel traces of in-process ranks on ONE device.

Each in-process rank launches from its own host thread on its own stream, so a kernel's rank is
its Thread_Id.  Per rank and per BundleAdjustment(10) call this reports the device time (sum of
its kernel durations), split into
  - factorisation (k_ldlt_*: subtrees + replicated separators),
  - exchange packing (k_tile_*, k_slot_*, k_b_unpack, k_x_zero_rows),
  - the rest (linearisation, Schur assembly, update, chi2, structure),
and the projection of the 1 -> 2 -> 4 -> 8 strong-scaling curve: per call
  T(R) = max over ranks of the rank's device time + the all-reduce time of the exchanged
         volume, 2 (R-1)/R * bytes / 153 GB/s per link (ring over xGMI).
The ranks share one GPU in the measurement, so a rank's kernels may run slower than alone; the
BA kernels are small latency-bound grids (a few CUs each), so the sum is an upper bound close to
the one-rank-per-GPU time.

usage: gba_rank_model.py 1 <R>:<kernel_trace.csv>[:<exchange doubles per trial>:<trials>] ...
(the trace's last call is the measured one: one call per rank thread)
"""
import csv
import sys
from collections import defaultdict

XGMI_GBS = 153.0


def kind(name):
    n = name.split("(")[0].replace("void ", "").replace("orbgpu::", "")
    if n.startswith("k_ldlt"):
        return "factorisation"
    if n.startswith(("k_tile_", "k_slot_", "k_b_unpack", "k_x_zero_rows", "k_fail_pub", "k_scal_pub")):
        return "exchange_pack"
    if n.startswith(("k_gs_", "k_align")):
        return "structure"
    if n.startswith("__amd_rocclr"):
        return "copies"
    return "system"


def rank_times(path):
    per = defaultdict(lambda: defaultdict(float))
    first = {}
    for r in csv.DictReader(open(path)):
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        t = r["Thread_Id"]
        first[t] = min(first.get(t, s), s)
        per[t][kind(r["Kernel_Name"])] += (e - s) * 1e-6   # ms
    return per, first


def main():
    calls = int(sys.argv[1])
    rows = []
    for spec in sys.argv[2:]:
        parts = spec.split(":")
        R, path = int(parts[0]), parts[1]
        xd = float(parts[2]) if len(parts) > 2 else 0.0
        trials = float(parts[3]) if len(parts) > 3 else 10.0
        per, first = rank_times(path)
        # every call runs its ranks on fresh host threads: the last call's ranks are the R
        # threads that started last (earlier threads: warm-up calls)
        # (helper threads -- the structure's nested dissection, the early pose graph -- launch a
        # few copies and fills of their own: only threads with a rank's share of the work count)
        big = max(sum(v.values()) for v in per.values())
        cand = [t for t in first if sum(per[t].values()) >= 0.05 * big]
        last = sorted(cand, key=lambda t: first[t])[-R:]
        ranks = sorted(((t, per[t]) for t in last), key=lambda kv: -sum(kv[1].values()))
        tot = [sum(v.values()) / calls for _, v in ranks]
        fac = [v["factorisation"] / calls for _, v in ranks]
        xbytes = xd * 8 * trials
        ar_ms = 0.0 if R == 1 else 2 * (R - 1) / R * xbytes / (XGMI_GBS * 1e9) * 1e3
        rows.append((R, max(tot), min(tot), max(fac), ar_ms))
        print(f"R={R}: per-rank device ms per call max {max(tot):.2f} min {min(tot):.2f} "
              f"(factorisation max {max(fac):.2f}); categories of the busiest rank: "
              + ", ".join(f"{k} {v / calls:.2f}" for k, v in sorted(ranks[0][1].items(), key=lambda kv: -kv[1])))
        print(f"      all-reduce volume per call {xbytes / 1e6:.2f} MB -> {ar_ms:.3f} ms at {XGMI_GBS:.0f} GB/s per link")
    if rows and rows[0][0] == 1:
        t1 = rows[0][1]
        print("projected strong scaling (T1 / T_R, T_R = busiest rank + all-reduce):")
        for R, mx, mn, fac, ar in rows:
            print(f"  R={R}: T_R = {mx + ar:.2f} ms  speed-up {t1 / (mx + ar):.2f}x  "
                  f"(imbalance max/min {mx / max(mn, 1e-9):.2f})")


if __name__ == "__main__":
    main()
