#!/usr/bin/env python3
"""Print a rocprofv3 *_kernel_stats.csv as a short table (name, calls, total ms, avg us, pct)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 25
print(f"{'kernel':48s} {'calls':>7s} {'total_ms':>10s} {'avg_us':>10s} {'pct':>6s}")
for r in rows[:n]:
    name = r['Name'].replace('(anonymous namespace)::', '')
    print(f"{name.split('(')[0][:48]:48s} {int(r['Calls']):7d} {float(r['TotalDurationNs']) / 1e6:10.2f} "
          f"{float(r['AverageNs']) / 1e3:10.2f} {float(r['Percentage']):6.2f}")
