#!/usr/bin/env python3
"""Timeline of one LocalBundleAdjustment call from a rocprofv3 kernel trace of tools/ba_timing.py:
the kernels of the last call (from its first k_linearize after the preceding k_gate pair) with
start/end/duration and the idle gap before each, then the totals: busy time, idle time, launches.
usage: lba_timeline.py kernel_trace.csv [memory_copy_trace.csv]"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
       r["Kernel_Name"].split("(")[0].replace("void ", "").replace("orbgpu::", "")[:34]) for r in rows]
if len(sys.argv) > 2:
    for r in csv.DictReader(open(sys.argv[2])):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "copy " + r.get("Direction", "")[:20]))
ev.sort()
gates = [i for i, e in enumerate(ev) if e[2].startswith("k_gate")]
# a call ends with its final gate (the second k_gate of the call); the previous call's final gate
# precedes the last call's first kernel
if len(gates) < 4:
    sys.exit("need two calls in the trace")
a, b = gates[-3] + 1, gates[-1] + 1
t0 = ev[a][0]
busy = idle = 0
prev = t0
n = 0
for s, e, name in ev[a:b]:
    gap = max(0, s - prev)
    idle += gap
    busy += e - s
    if not name.startswith("copy"):
        n += 1
    print(f"{(s - t0) / 1e3:9.1f} {(e - t0) / 1e3:9.1f} {(e - s) / 1e3:7.1f}  gap {gap / 1e3:6.1f}  {name}")
    prev = max(prev, e)
print(f"call: {(prev - t0) / 1e3:.1f} us, busy {busy / 1e3:.1f} us, idle {idle / 1e3:.1f} us, kernels {n}")
