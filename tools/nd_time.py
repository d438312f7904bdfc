#!/usr/bin/env python3
"""Time the product's nested-dissection order (orbgpu_unit_nd_order) on the config-5 pose graph
(2,000 keyframes, 4 laps) and print a digest of the order (host only)."""
import ctypes as C
import hashlib
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
from ba_cases import global_ba_problem  # noqa: E402
from c_orb_slam_amd._lib import lib, ptr  # noqa: E402


def pose_graph_csr(pr):
    free = pr["kf_id"] != 0
    pidx = -np.ones(len(free), np.int64)
    pidx[free] = np.arange(int(free.sum()))
    pe, ke = pr["edge_pt"], pidx[pr["edge_kf"]]
    o = np.argsort(pe, kind="stable")
    pe, ke = pe[o], ke[o]
    cut = np.flatnonzero(np.r_[True, pe[1:] != pe[:-1], True])
    n = int(free.sum())
    keys = set()
    for s, t in zip(cut[:-1], cut[1:]):
        ks = sorted(set(int(k) for k in ke[s:t] if k >= 0))
        for i, a in enumerate(ks):
            for b in ks[i + 1:]:
                keys.add(a * n + b)
    nb = [[] for _ in range(n)]
    for q in keys:
        a, b = divmod(q, n)
        nb[a].append(b)
        nb[b].append(a)
    as_ = np.zeros(n + 1, np.int32)
    adj = []
    for i in range(n):
        as_[i + 1] = as_[i] + len(nb[i])
        adj += sorted(nb[i])
    return n, as_, np.array(adj + [0], np.int32)


def main():
    pr = global_ba_problem(0, n_kf=2000, pts_per_kf=150, laps=4)
    n, as_, adj = pose_graph_csr(pr)
    perm = np.zeros(n, np.int32)
    nn, h = C.c_int32(), C.c_int32()
    ts = []
    for _ in range(20):
        t = time.perf_counter()
        assert lib().orbgpu_unit_nd_order(n, ptr(as_), ptr(adj), 32, ptr(perm), C.byref(nn), C.byref(h)) == 0
        ts.append(time.perf_counter() - t)
    print(f"n {n} adj {len(adj) - 1} nodes {nn.value} height {h.value} median {np.median(ts) * 1e3:.2f} ms "
          f"min {min(ts) * 1e3:.2f} ms digest {hashlib.md5(perm.tobytes()).hexdigest()}")


if __name__ == "__main__":
    main()
