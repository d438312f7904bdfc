#!/usr/bin/env python3
"""Check bench.py's roofline duration against rocprofv3: the bench's roofline pass is the last
ROOFLINE_REPS launches of the kernel in the run; average their kernel-trace durations.

usage: roofline_check.py kernel_trace.csv bench.json
"""
import csv
import json
import sys

trace, bench = sys.argv[1], json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
roof = bench["roofline"]
k, reps = roof["kernel"], roof.get("launches", 5)
rows = sorted((r for r in csv.DictReader(open(trace)) if k in r["Kernel_Name"]), key=lambda r: int(r["Start_Timestamp"]))
# the roofline pass runs full batches; later legs (the batch-1 latency leg) launch the same kernel
# on one image: keep the full-batch launches only
gsz = lambda r: int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
gmax = max(gsz(r) for r in rows)
rows = [r for r in rows if gsz(r) == gmax]
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows]
iso = d[-reps:]
pipe = d[:-reps]
out = {"kernel": k, "rocprof_avg_ms_roofline_pass": round(sum(iso) / len(iso), 4),
       "bench_avg_launch_ms": roof["avg_launch_ms"],
       "rocprof_avg_ms_pipeline": round(sum(pipe) / max(len(pipe), 1), 4), "launches_total": len(d)}
out["ratio"] = round(out["rocprof_avg_ms_roofline_pass"] / roof["avg_launch_ms"], 3)
print(json.dumps(out))
