#!/usr/bin/env python3
"""Per-step timeline of a bench rocprofv3 kernel trace: kernels of one pipeline step (between two
k_pose_opt launches), grouped per stream, with start/end relative to the step start (us).
usage: timeline.py kernel_trace.csv [step_index] [pose launches per step (2: TrackLocalMap's second one)]"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
k = int(sys.argv[2]) if len(sys.argv) > 2 else 8
per = int(sys.argv[3]) if len(sys.argv) > 3 else 2
po = [r for r in rows if "k_pose_opt" in r["Kernel_Name"]][per - 1::per]
t0, t1 = int(po[k - 1]["End_Timestamp"]), int(po[k]["End_Timestamp"])
print(f"step {k}: {(t1 - t0) / 1e3:.1f} us")
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if e <= t0 or s >= t1:
        continue
    name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("orbgpu::", "")[:40]
    print(f"  q{r['Queue_Id']:>2s} s{r['Stream_Id']:>2s} {(s - t0) / 1e3:8.1f} {(e - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f}  {name}")
