"""Concurrency of the host entry points.

The bench's local-BA throughput leg calls LocalBundleAdjustment from 16 host threads at once, and
LocalMapping / Tracking / LoopClosing run concurrently in the reference (System.cc:93-121 starts
them as threads).  Each host thread gets its own engine (capi_ba.cpp thread_local engine() /
pose_engine(): stream, device arena and pinned staging of its own), so concurrent calls must give
exactly the results of the same calls made one at a time.  These tests run 16 threads, each with a
different problem, several rounds, and compare every output bit for bit with the sequential run;
they also exercise a thread exiting and its successor starting a fresh engine.
"""
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

from ba_cases import ba_problem
from pose_cases import pose_problem

pytestmark = pytest.mark.gpu

KEYS = ("kf_id", "kf_Tcw", "kf_local", "kf_cam", "pt_id", "pt_pos", "edge_pt", "edge_kf", "edge_obs",
        "edge_inv_sigma2")
THREADS = 16


def _lba(pr):
    from c_orb_slam_amd.optimizer import LocalBundleAdjustment
    r = LocalBundleAdjustment(*[pr[k] for k in KEYS])
    return r["kf_Tcw"].copy(), r["pt_pos"].copy(), np.asarray(r["edge_erase"]).copy(), tuple(r["iterations"])


def _same(a, b):
    assert len(a) == len(b)
    for x, y in zip(a, b):
        if isinstance(x, np.ndarray):
            assert np.array_equal(x, y)
        else:
            assert x == y


def test_local_ba_concurrent_threads_match_sequential(gpu):
    probs = [ba_problem(100 + i, n_pt=600 + 40 * i) for i in range(THREADS)]
    seq = [_lba(p) for p in probs]
    for rnd in range(3):
        # a fresh pool each round: threads exit and new ones build their engines again
        with ThreadPoolExecutor(THREADS) as ex:
            order = list(range(THREADS))[rnd::1] + list(range(THREADS))[:rnd]
            got = dict(zip(order, ex.map(lambda i: _lba(probs[i]), order)))
        for i in range(THREADS):
            _same(got[i], seq[i])


def test_pose_concurrent_threads_match_sequential(gpu):
    from c_orb_slam_amd.optimizer import PoseOptimization, PoseOptimizationBatch
    frames = [pose_problem(200 + i, N=400 + 50 * i) for i in range(THREADS)]

    def one(i):
        n, T, o = PoseOptimization(frames[i])
        return n, T.copy(), np.asarray(o).copy()
    seq = [one(i) for i in range(THREADS)]
    with ThreadPoolExecutor(THREADS) as ex:
        for _ in range(4):
            got = list(ex.map(one, range(THREADS)))
            for g, s in zip(got, seq):
                assert g[0] == s[0]
                assert np.array_equal(g[1], s[1]) and np.array_equal(g[2], s[2])
        # batches from several threads at once share nothing either
        nb, Tb, _ = PoseOptimizationBatch(frames)
        halves = list(ex.map(lambda h: PoseOptimizationBatch(frames[h::2]), (0, 1)))
    for h in (0, 1):
        assert np.array_equal(halves[h][0], nb[h::2]) and np.array_equal(halves[h][1], Tb[h::2])
    assert [int(x) for x in nb] == [s[0] for s in seq]
