"""Golden fixture for config 5 at its stated sizes (N_kf in {2k, 8k, 16k}):
the oracle's BundleAdjustment (oracle/ba.c, the restatement of Optimizer.cc:49-237 + g2o) on
  - 8,000 keyframes, 4 laps, nIterations = 10 (LoopClosing.cc:650's call),
  - 16,000 keyframes, 4 laps, nIterations = 1,
too slow for the single-thread oracle inside a GPU test (minutes per iteration), so run here
once.  Stored: the LM trace and SHA-256 digests of the float32 results (the poses and points
themselves would be 13-26 MB), plus a digest of the generated inputs so the test knows it feeds
the GPU the same problem.  TEST INFRASTRUCTURE ONLY.

usage: python tests/golden/make_gba_large.py   (writes tests/golden/gba_large.json)
"""
import hashlib
import json
import sys
import time
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parent))
import oracle_lib  # noqa: E402
from ba_cases import global_ba_problem  # noqa: E402

CASES = [dict(name="kf8000_its10", seed=6, n_kf=8000, pts_per_kf=150, laps=4, its=10),
         dict(name="kf16000_its1", seed=7, n_kf=16000, pts_per_kf=150, laps=4, its=1)]
KEYS = ("kf_id", "kf_Tcw", "kf_local", "kf_cam", "pt_id", "pt_pos", "edge_pt", "edge_kf", "edge_obs", "edge_inv_sigma2")


def digest(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def input_digest(pr):
    h = hashlib.sha256()
    for k in KEYS:
        h.update(np.ascontiguousarray(pr[k]).tobytes())
    return h.hexdigest()


def main():
    out = {}
    want = sys.argv[1:]
    for c in CASES:
        if want and c["name"] not in want:
            continue
        pr = global_ba_problem(c["seed"], n_kf=c["n_kf"], pts_per_kf=c["pts_per_kf"], laps=c["laps"])
        t0 = time.time()
        o = oracle_lib.oracle_global_ba(pr, c["its"], False)
        dt = time.time() - t0
        out[c["name"]] = dict(case=c, input_sha256=input_digest(pr), n_edges=int(len(pr["edge_pt"])),
                              n_points=int(len(pr["pt_id"])), iterations=list(o["iterations"]),
                              trial_chi2=[float(v) for v in o["trial_chi2"]],
                              trial_lambda=[float(v) for v in o["trial_lambda"]],
                              solve_chi2=[float(v) for v in o["solve_chi2"]],
                              kf_Tcw_sha256=digest(np.asarray(o["kf_Tcw"], np.float32)),
                              pt_pos_sha256=digest(np.asarray(o["pt_pos"], np.float32)),
                              kf_Tcw_head=[float(v) for v in np.asarray(o["kf_Tcw"], np.float32).reshape(-1)[:48]],
                              oracle_seconds=round(dt, 1))
        print(c["name"], dt, o["iterations"], len(o["trial_chi2"]), flush=True)
        p = HERE / "gba_large.json"
        cur = json.loads(p.read_text()) if p.exists() else {}
        cur.update(out)
        p.write_text(json.dumps(cur, indent=1) + "\n")


if __name__ == "__main__":
    main()
