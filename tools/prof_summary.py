#!/usr/bin/env python3
"""Print the top-kernels table of a rocprofv3 rocpd database (durations in the db are us)."""
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
rows = list(c.execute("select name, total_calls, total_duration, average, percentage from top_kernels"))
print(f"{'kernel':60s} {'calls':>6s} {'total_ms':>10s} {'avg_us':>9s} {'pct':>6s}")
for name, calls, tot, avg, pct in rows:
    short = name.split("(")[0]
    print(f"{short[:60]:60s} {calls:6d} {tot / 1e3:10.2f} {avg:9.2f} {pct:6.2f}")
