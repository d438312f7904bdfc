#!/usr/bin/env python3
"""Per-step timeline of a bench rocprofv3 kernel trace: the kernels of one pipeline step, grouped
per stream, with start/end relative to the step start (us).  A step runs from the start of one
extraction's first pyramid launch (k_pyr_level0) to the start of the next extraction's, so the
window stays one step when the lanes' tracking chains run on streams of their own
(--lane-matchers 1) and overlap.
usage: timeline.py kernel_trace.csv [step_index] [k_pyr_level0 launches per step (2: --stereo-batch 0)]"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
k = int(sys.argv[2]) if len(sys.argv) > 2 else 8
per = int(sys.argv[3]) if len(sys.argv) > 3 else 1
pyr = [r for r in rows if "k_pyr_level0" in r["Kernel_Name"]][::per]
t0, t1 = int(pyr[k - 1]["Start_Timestamp"]), int(pyr[k]["Start_Timestamp"])
print(f"step {k}: {(t1 - t0) / 1e3:.1f} us")
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if e <= t0 or s >= t1:
        continue
    name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("orbgpu::", "")[:40]
    print(f"  q{r['Queue_Id']:>2s} s{r['Stream_Id']:>2s} {(s - t0) / 1e3:8.1f} {(e - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f}  {name}")
