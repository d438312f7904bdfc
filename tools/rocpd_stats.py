#!/usr/bin/env python3
"""Kernel stats (count, total / average / min / max ns, percentage) from a rocprofv3 SQLite
output (rocpd schema, the default -f of rocprofv3 7.x), in the layout of its --stats CSV.
usage: tools/rocpd_stats.py <results.db> [out.csv]"""
import csv
import sqlite3
import sys


def main():
    c = sqlite3.connect(sys.argv[1])
    rows = c.execute("select s.kernel_name, d.start, d.end from rocpd_kernel_dispatch d "
                     "join rocpd_info_kernel_symbol s on d.kernel_id = s.id").fetchall()
    agg = {}
    for name, a, b in rows:
        e = agg.setdefault(name, [])
        e.append(b - a)
    tot = sum(sum(v) for v in agg.values()) or 1
    out = [("Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs")]
    for name, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        out.append((name, len(v), sum(v), sum(v) / len(v), 100.0 * sum(v) / tot, min(v), max(v)))
    w = csv.writer(open(sys.argv[2], "w") if len(sys.argv) > 2 else sys.stdout)
    w.writerows(out)


if __name__ == "__main__":
    main()
