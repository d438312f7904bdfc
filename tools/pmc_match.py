#!/usr/bin/env python3
"""Per-launch HBM traffic and VALU issue of every kernel, from three rocprofv3 --pmc passes
(FETCH_SIZE, WRITE_SIZE, SQ_INSTS_VALU; one counter set per run, MI355X_MICROARCH.md HBM
section): bytes = 2 x FETCH_SIZE (KiB, the gfx950 correction, calibrated for 16/4/1-B loads in
profiles/fetch_calib_r01.txt) + WRITE_SIZE (KiB).  Template arguments are dropped from kernel
names (k_candidates<true> -> k_candidates).

usage: pmc_match.py FETCH.csv WRITE.csv VALU.csv out.json [workload note]
"""
import collections
import csv
import json
import re
import sys


def per_launch(path, counter):
    tot = collections.defaultdict(float)
    n = collections.defaultdict(set)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        k = r["Kernel_Name"].split("(")[0].replace("orbgpu::", "").replace("void ", "")
        k = re.sub(r"<.*>", "", k).strip()
        tot[k] += float(r["Counter_Value"])
        n[k].add(r.get("Dispatch_Id") or r.get("Correlation_Id"))
    return {k: (tot[k] / max(len(n[k]), 1), len(n[k])) for k in tot}


def main():
    fetch = per_launch(sys.argv[1], "FETCH_SIZE")
    write = per_launch(sys.argv[2], "WRITE_SIZE")
    valu = per_launch(sys.argv[3], "SQ_INSTS_VALU")
    out = {"_note": "per launch (mean over the run's launches); hbm = 2 x FETCH_SIZE + WRITE_SIZE (KiB -> B); "
                    "SQ_INSTS_VALU = wave-level VALU instructions; separate --pmc passes; "
                    + (sys.argv[5] if len(sys.argv) > 5 else "")}
    for k in sorted(set(fetch) | set(write) | set(valu)):
        if not k.startswith("k_"):
            continue
        f, w = fetch.get(k, (0.0, 0))[0], write.get(k, (0.0, 0))[0]
        out[k] = {"fetch_kib": round(f, 1), "write_kib": round(w, 1), "hbm_bytes_per_launch": int(round((2 * f + w) * 1024)),
                  "valu_insts_per_launch": round(valu.get(k, (0.0, 0))[0]), "launches": fetch.get(k, (0, 0))[1]}
    json.dump(out, open(sys.argv[4], "w"), indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
