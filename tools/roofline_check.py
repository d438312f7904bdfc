#!/usr/bin/env python3
"""Check bench.py's roofline durations against rocprofv3: each roofline pass (k_pose_opt, the
headline; k_fast_cells, its `secondary`) is the last `launches` full-size launches of its kernel
in the run; average their kernel-trace durations and compare with the bench's HIP-event figure.

usage: roofline_check.py kernel_trace.csv bench.json
"""
import csv
import json
import sys

trace, bench = sys.argv[1], json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
rows_all = list(csv.DictReader(open(trace)))
gsz = lambda r: int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
res = []
for roof in (bench["roofline"], bench["roofline"].get("secondary")):
    if not roof:
        continue
    k, reps = roof["kernel"], roof.get("launches", 5)
    rows = sorted((r for r in rows_all if k in r["Kernel_Name"]), key=lambda r: int(r["Start_Timestamp"]))
    # the roofline passes run full batches; later legs (the batch-1 latency legs) launch the same
    # kernels on one frame: keep the full-batch launches only
    gmax = max(gsz(r) for r in rows)
    rows = [r for r in rows if gsz(r) == gmax]
    d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows]
    iso, pipe = d[-reps:], d[:-reps]
    out = {"kernel": k, "rocprof_avg_ms_roofline_pass": round(sum(iso) / len(iso), 4),
           "bench_avg_launch_ms": roof["avg_launch_ms"],
           "rocprof_avg_ms_pipeline": round(sum(pipe) / max(len(pipe), 1), 4), "launches_total": len(d)}
    out["ratio"] = round(out["rocprof_avg_ms_roofline_pass"] / roof["avg_launch_ms"], 3)
    res.append(out)
print(json.dumps(res))
