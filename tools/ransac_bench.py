"""The bench's RANSAC leg alone (SURVEY config 3): python tools/ransac_bench.py [--no-cpu]"""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import bench  # noqa: E402

r = bench.bench_ransac(cpu="--no-cpu" not in sys.argv, cpu_budget_s=4.0)
r.pop("_cpu_args", None)   # the CPU leg's inputs (arrays), not part of the report
print(json.dumps(r, indent=1), flush=True)
