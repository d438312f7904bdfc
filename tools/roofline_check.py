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
    # kernels on one frame.  With --stereo-batch the pipeline extracts 2B images per launch and the
    # k_fast_cells roofline pass B: a launch shape that occurs exactly `reps` times is the pass;
    # otherwise the pass is the last `reps` launches of the largest shape
    import collections
    shapes = collections.Counter(gsz(r) for r in rows)
    exact = [g for g, c in shapes.items() if c == reps]
    gmax = max(shapes)
    if exact and len(shapes) > 1:
        g = exact[0]
        iso_rows = [r for r in rows if gsz(r) == g]
        pipe_rows = [r for r in rows if gsz(r) == gmax and g != gmax]
    else:
        full = [r for r in rows if gsz(r) == gmax]
        iso_rows, pipe_rows = full[-reps:], full[:-reps]
    dur = lambda rs: [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rs]
    iso, pipe = dur(iso_rows), dur(pipe_rows)
    d = iso + pipe
    out = {"kernel": k, "rocprof_avg_ms_roofline_pass": round(sum(iso) / len(iso), 4),
           "bench_avg_launch_ms": roof["avg_launch_ms"],
           "rocprof_avg_ms_pipeline": round(sum(pipe) / max(len(pipe), 1), 4), "launches_total": len(d)}
    out["ratio"] = round(out["rocprof_avg_ms_roofline_pass"] / roof["avg_launch_ms"], 3)
    res.append(out)
print(json.dumps(res))
