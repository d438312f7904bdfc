#!/usr/bin/env python3
"""Timeline of the structure phase of the last BundleAdjustment call in a rocprofv3 trace of
tools/gba_timing.py: from the call's upload copy and unpack kernel to its first
k_linearize, with the idle gap before each entry (host work between launches shows as gaps).
usage: gba_struct_timeline.py kernel_trace.csv [memory_copy_trace.csv]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
       r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")
       .replace("orbgpu::", "")[:40]) for r in rows]
if len(sys.argv) > 2:
    for r in csv.DictReader(open(sys.argv[2])):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "copy " + r.get("Direction", "")[:24]))
ev.sort()
exp = [i for i, e in enumerate(ev) if e[2].startswith(("k_unpack_upload", "k_expand_edges"))]
if not exp:
    sys.exit("no upload kernel in the trace")
a = exp[-1]
while a > 0 and ev[a - 1][2].startswith("copy"):   # the call's uploads
    a -= 1
b = next((i for i in range(a, len(ev)) if ev[i][2].startswith("k_linearize")), len(ev))
t0 = ev[a][0]
prev = t0
busy = idle = 0
for s, e, name in ev[a:b + 1]:
    gap = max(0, s - prev)
    idle += gap
    busy += e - s
    print(f"{(s - t0) / 1e3:9.1f} {(e - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f}  gap {gap / 1e3:7.1f}  {name}")
    prev = max(prev, e)
print(f"structure phase: {(prev - t0) / 1e3:.1f} us, busy {busy / 1e3:.1f} us, idle {idle / 1e3:.1f} us")
