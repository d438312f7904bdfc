#!/usr/bin/env python3
"""Print the top-kernels table of a rocprofv3 rocpd database (name, calls, total us, avg us, %)."""
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
rows = list(c.execute("select name, total_calls, total_duration, average, percentage from top_kernels"))
print(f"{'kernel':60s} {'calls':>6s} {'total_us':>10s} {'avg_us':>9s} {'pct':>6s}")
for name, calls, tot, avg, pct in rows:
    short = name.split("(")[0]
    print(f"{short[:60]:60s} {calls:6d} {tot / 1e3:10.1f} {avg / 1e3:9.2f} {pct:6.2f}")
