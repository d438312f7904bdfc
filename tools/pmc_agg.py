"""Per-kernel averages of a rocprofv3 --pmc counter_collection.csv: python tools/pmc_agg.py file [substr]"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
flt = sys.argv[2] if len(sys.argv) > 2 else ""
agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.Counter()
for r in rows:
    k = r["Kernel_Name"].split("(")[0]
    if flt not in k:
        continue
    agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    cnt[(k, r["Counter_Name"])] += 1
for k, d in agg.items():
    n = max(cnt[(k, c)] for c in d)
    waves = d.get("SQ_WAVES", 0) / n
    out = {c: round(v / n) for c, v in d.items()}
    if waves:
        out["VALU_per_wave"] = round(d.get("SQ_INSTS_VALU", 0) / n / waves, 1)
        out["LDS_per_wave"] = round(d.get("SQ_INSTS_LDS", 0) / n / waves, 1)
    print(k, out)
