#!/usr/bin/env python3
"""Launches of the last sparse LDL^T solve in a rocprofv3 kernel trace (k_ldlt_update, the panel
steps k_ldlt_pdiag / prow / ptrail, k_ldlt_pfwd, k_ldlt_backward; in launch order) with their
durations and grid sizes.
usage: ldlt_levels.py kernel_trace.csv"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
ld = [r for r in rows if "k_ldlt_" in r["Kernel_Name"] and "k_ldlt_reg" not in r["Kernel_Name"]]
# a solve starts at the first update/factor after a backward run
def bwd(r):
    n = r["Kernel_Name"]
    return "backward" in n or "bwdn" in n or "k_ldlt_bin" in n or "bpush" in n


starts = [i for i in range(len(ld)) if not bwd(ld[i]) and (i == 0 or bwd(ld[i - 1]))]
seg = ld[starts[-1]:]
t0 = int(seg[0]["Start_Timestamp"])
tot = {}
for r in seg:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = r["Kernel_Name"].split("(")[0].replace("orbgpu::", "")
    g = r.get("Grid_Size_X") or r.get("Grid_Size") or ""
    wg = r.get("Workgroup_Size_X") or r.get("Workgroup_Size") or ""
    print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:9.1f} us  {name:18s} grid {g} wg {wg}")
    tot[name] = tot.get(name, 0) + (e - s)
print({k: round(v / 1e3, 1) for k, v in tot.items()}, "us; span", (int(seg[-1]["End_Timestamp"]) - t0) / 1e3, "us")
