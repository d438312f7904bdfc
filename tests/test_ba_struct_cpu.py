"""CPU: the host structure builder of the BA kernels (csrc/ba_struct.cpp) against a plain
restatement of what g2o builds (sparse_optimizer.cpp initializeOptimization/buildIndexMapping,
block_solver.hpp:73-216 buildStructure):

* active edges = the edges of the optimisation level, in insertion order;
* pose vertices: keyframes with an active edge that are not fixed, ascending mnId; landmark
  vertices: points with an active edge, ascending mnId (Optimizer.cc ids: poses below points);
* per landmark its edges to free poses in pose order; a second edge to the same pose is an error;
* Schur blocks: every diagonal block first (pose order), then off-diagonal blocks (i1 <= i2) in
  order of first use walking the landmarks in order and their pose pairs u <= v; each block's
  terms (pairA, pairB) in landmark order.
"""
import ctypes as C

import numpy as np
import pytest

from ba_cases import ba_problem, global_ba_problem
from c_orb_slam_amd._lib import lib, ptr


def _unit(pr, level_of_edge, fixed, level=0):
    ne = len(pr["edge_pt"])
    cap = 64 + 40 * ne + 4 * len(pr["pt_id"])
    out = np.zeros(cap, np.int32)
    args = [len(pr["kf_id"]), len(pr["pt_id"]), ne, ptr(np.ascontiguousarray(pr["edge_kf"], np.int32)),
            ptr(np.ascontiguousarray(pr["edge_pt"], np.int32)), ptr(np.ascontiguousarray(level_of_edge, np.uint8)),
            ptr(np.ascontiguousarray(fixed, np.uint8)), ptr(np.ascontiguousarray(pr["kf_id"], np.int32)),
            ptr(np.ascontiguousarray(pr["pt_id"], np.int32)), level, ptr(out), C.c_longlong(cap)]
    rc = lib().orbgpu_unit_ba_struct(*args)
    if rc:
        return rc, None
    nE, nP, nL, nBlk, nPair = (int(v) for v in out[:5])
    o = 5
    res = {}
    for name, n in (("poseKf", nP), ("landPt", nL), ("ePose", nE), ("eLand", nE), ("lpStart", nL + 1)):
        res[name] = out[o:o + n].copy()
        o += n
    nlp = int(res["lpStart"][-1])
    for name, n in (("lpList", nlp), ("blkI", nBlk), ("blkJ", nBlk), ("blkStart", nBlk + 1), ("pairA", nPair),
                    ("pairB", nPair)):
        res[name] = out[o:o + n].copy()
        o += n
    res["nE"] = nE
    return 0, res


def _expected(pr, level_of_edge, fixed, level=0):
    ekf, ept = pr["edge_kf"], pr["edge_pt"]
    aE = [i for i in range(len(ekf)) if level_of_edge[i] == level]
    kf_act = sorted({int(ekf[i]) for i in aE if not fixed[ekf[i]]}, key=lambda k: pr["kf_id"][k])
    pt_act = sorted({int(ept[i]) for i in aE}, key=lambda p: pr["pt_id"][p])
    pidx = {k: i for i, k in enumerate(kf_act)}
    lidx = {p: i for i, p in enumerate(pt_act)}
    ePose = [pidx.get(int(ekf[i]), -1) for i in aE]
    eLand = [lidx[int(ept[i])] for i in aE]
    per_land = [[] for _ in pt_act]
    for a, (p, l) in enumerate(zip(ePose, eLand)):
        if p >= 0:
            per_land[l].append((p, a))
    for lst in per_land:
        lst.sort()
        ps = [p for p, _ in lst]
        if len(set(ps)) != len(ps):
            return None
    nP = len(kf_act)
    blocks = {(i, i): i for i in range(nP)}
    order = [(i, i) for i in range(nP)]
    terms = {}
    for lst in per_land:
        for u in range(len(lst)):
            for v in range(u, len(lst)):
                key = (lst[u][0], lst[v][0])
                if key not in blocks:
                    blocks[key] = len(order)
                    order.append(key)
                terms.setdefault(key, []).append((lst[u][1], lst[v][1]))
    pairA = [a for key in order for a, _ in terms.get(key, [])]
    pairB = [b for key in order for _, b in terms.get(key, [])]
    starts = np.cumsum([0] + [len(terms.get(key, [])) for key in order])
    return dict(poseKf=kf_act, landPt=pt_act, ePose=ePose, eLand=eLand,
                lpList=[a for lst in per_land for _, a in lst],
                lpStart=np.cumsum([0] + [len(lst) for lst in per_land]),
                blkI=[k[0] for k in order], blkJ=[k[1] for k in order], blkStart=starts, pairA=pairA, pairB=pairB)


def _compare(got, exp):
    for k, v in exp.items():
        assert np.array_equal(np.asarray(got[k]), np.asarray(v, np.int64)), k


@pytest.mark.parametrize("seed", [0, 1])
def test_local_ba_structure(seed):
    pr = ba_problem(seed, n_local=6, n_fixed=4, n_pt=300)
    rng = np.random.default_rng(seed)
    fixed = (1 - pr["kf_local"]).astype(np.uint8)
    level = np.zeros(len(pr["edge_pt"]), np.uint8)
    rc, got = _unit(pr, level, fixed)
    assert rc == 0
    _compare(got, _expected(pr, level, fixed))
    # the second optimisation: gated edges moved to level 1, shuffled ids
    level = (rng.random(len(level)) < 0.15).astype(np.uint8)
    pr = dict(pr)
    pr["pt_id"] = rng.permutation(len(pr["pt_id"])).astype(np.int32) * 3 + 7
    pr["kf_id"] = rng.permutation(len(pr["kf_id"])).astype(np.int32) + 100
    rc, got = _unit(pr, level, fixed)
    assert rc == 0
    _compare(got, _expected(pr, level, fixed))
    rc, got = _unit(pr, level, fixed, level=1)
    assert rc == 0
    _compare(got, _expected(pr, level, fixed, level=1))


def test_global_ba_structure_with_loops():
    pr = global_ba_problem(2, n_kf=40, pts_per_kf=20, laps=2)
    fixed = (pr["kf_id"] == 0).astype(np.uint8)
    level = np.zeros(len(pr["edge_pt"]), np.uint8)
    rc, got = _unit(pr, level, fixed)
    assert rc == 0
    _compare(got, _expected(pr, level, fixed))


def test_duplicate_pose_landmark_edge_rejected():
    """A second edge between one free pose and one landmark would give g2o two Hpl blocks for
    one (pose, landmark) pair: the builder refuses it (the C ABI validates it away earlier)."""
    pr = dict(ba_problem(3, n_local=3, n_fixed=2, n_pt=40))
    i = int(np.flatnonzero(pr["kf_local"][pr["edge_kf"]] == 1)[0])   # an edge to a free pose
    for k in ("edge_pt", "edge_kf", "edge_obs", "edge_inv_sigma2"):
        pr[k] = np.concatenate([pr[k], pr[k][i:i + 1]])
    fixed = (1 - pr["kf_local"]).astype(np.uint8)
    level = np.zeros(len(pr["edge_pt"]), np.uint8)
    assert _expected(pr, level, fixed) is None
    rc, _ = _unit(pr, level, fixed)
    assert rc != 0
