"""Host side of keyframe-block sharded BA, on CPU.

- Optimizer_partition_points (host-only C entry point): every point gets exactly one
  rank, ranks own contiguous keyframe blocks (mnId order), edge weight is balanced.
- shard_problem / merge_shards round trip, edge order preserved inside a shard.
- world_size-2 gloo run of the exchange the library does at structure build: the
  union of the shards' active keyframes (sum all-reduce) equals the unsharded set,
  and the gathered shards reassemble the problem.
- the sharded/global C entry points validate arguments and refuse without a device.
"""
import ctypes as C
import os
import socket

import numpy as np
import pytest

from ba_cases import ba_problem, global_ba_problem


def _lib():
    from c_orb_slam_amd._lib import lib
    return lib()


@pytest.mark.parametrize("nranks", [1, 2, 3, 8])
def test_partition_contiguous_blocks_and_balance(nranks):
    from c_orb_slam_amd.optimizer import partition_points
    pr = global_ba_problem(0, n_kf=80, pts_per_kf=50)
    r = partition_points(pr, nranks)
    assert r.shape == (len(pr["pt_id"]),) and r.min() >= 0 and r.max() < nranks
    # reference keyframe = first observation; its rank is monotone in mnId
    first = np.full(len(pr["pt_id"]), -1)
    for i in range(len(pr["edge_pt"]) - 1, -1, -1):
        first[pr["edge_pt"][i]] = pr["edge_kf"][i]
    kf_rank = {}
    for p, k in enumerate(first):
        kf_rank.setdefault(int(k), set()).add(int(r[p]))
    assert all(len(v) == 1 for v in kf_rank.values()), "a keyframe block is split across ranks"
    ks = sorted(kf_rank, key=lambda k: pr["kf_id"][k])
    seq = [next(iter(kf_rank[k])) for k in ks]
    assert seq == sorted(seq), "blocks are not contiguous in mnId order"
    w = np.bincount(r[pr["edge_pt"]], minlength=nranks)
    if nranks > 1:
        assert w.min() > 0.5 * w.mean() and w.max() < 1.5 * w.mean(), w


@pytest.mark.parametrize("nranks,laps,n_kf", [(2, 0, 400), (4, 4, 400), (8, 4, 400), (8, 4, 2000)])
def test_partition_nd_subtrees(nranks, laps, n_kf):
    """Optimizer_partition_points_nd (host only): every point one rank, deterministic, and a
    keyframe observed by points of two ranks must be a separator pose, so few keyframes are:
    each rank's Schur terms stay inside its own subtrees and the separators."""
    from c_orb_slam_amd.optimizer import partition_points_nd
    pr = global_ba_problem(3, n_kf=n_kf, pts_per_kf=40, laps=laps)
    r, kfo = partition_points_nd(pr, nranks, with_kf_owner=True)
    assert r.shape == (len(pr["pt_id"]),) and r.min() >= 0 and r.max() < nranks
    assert np.array_equal(r, partition_points_nd(pr, nranks))
    assert (kfo[pr["kf_id"] == 0] == -2).all()          # the fixed keyframe is no pose
    assert set(np.unique(kfo[pr["kf_id"] != 0])) <= set(range(-1, nranks))
    # the invariant the sharded factorisation relies on: a point observes only poses of its
    # rank's subtrees or separators
    own = kfo[pr["edge_kf"]]
    assert ((own == -1) | (own == -2) | (own == r[pr["edge_pt"]])).all()
    sizes = [(kfo == q).sum() for q in range(nranks)]
    if n_kf >= 2000:   # config-5 size: every rank a subtree, separators a small share
        assert min(sizes) > 0 and max(sizes) < 2 * np.mean(sizes), sizes
        assert (kfo == -1).sum() < 0.2 * n_kf
    else:              # a small loop-closed map may leave ranks without a subtree (separators only)
        assert sum(sizes) > 0


def test_partition_nd_small_or_single_rank_is_block():
    """Below the block-sparse size (24 free poses) or at one rank: the keyframe-block partition."""
    from c_orb_slam_amd.optimizer import partition_points, partition_points_nd
    pr = global_ba_problem(1, n_kf=20, pts_per_kf=30)
    assert np.array_equal(partition_points_nd(pr, 3), partition_points(pr, 3))
    # the fallback still names an owner for every free pose: its keyframe's block,
    # the block of the points whose first observation it is
    r, kfo = partition_points_nd(pr, 3, with_kf_owner=True)
    assert (kfo[pr["kf_id"] == 0] == -2).all() and (kfo[pr["kf_id"] != 0] >= 0).all()
    first = {}
    for e, (p, k) in enumerate(zip(pr["edge_pt"], pr["edge_kf"])):
        first.setdefault(int(p), int(k))
    for p, k in first.items():
        if pr["kf_id"][k] != 0:
            assert r[p] == kfo[k]
    pr = global_ba_problem(1, n_kf=60, pts_per_kf=30)
    assert (partition_points_nd(pr, 1) == 0).all()


def test_partition_validates():
    from c_orb_slam_amd._lib import ba_problem as BP
    L = _lib()
    P = BP()
    P.n_kf = -1
    out = np.zeros(4, np.int32)
    assert L.Optimizer_partition_points(C.byref(P), 2, out.ctypes.data) == -1
    P.n_kf = 0
    assert L.Optimizer_partition_points(C.byref(P), 0, out.ctypes.data) == -1


def test_shard_merge_round_trip():
    from c_orb_slam_amd.optimizer import merge_shards, partition_points, shard_problem
    pr = ba_problem(0, n_local=8, n_fixed=4, n_pt=600)
    r = partition_points(pr, 3)
    shards = [shard_problem(pr, r, k) for k in range(3)]
    assert sum(len(s["pt_id"]) for s in shards) == len(pr["pt_id"])
    assert sum(len(s["edge_pt"]) for s in shards) == len(pr["edge_pt"])
    for s in shards:
        assert np.all(np.diff(s["edge_index"]) > 0), "edge order (g2o creation order) must be kept"
        assert np.array_equal(pr["edge_pt"][s["edge_index"]], s["pt_index"][s["edge_pt"]])
        assert np.array_equal(s["kf_Tcw"], pr["kf_Tcw"])
    fake = [dict(kf_Tcw=pr["kf_Tcw"], pt_pos=s["pt_pos"], edge_erase=np.zeros(len(s["edge_pt"]), bool),
                 iterations=(5, 10), aborted=False) for s in shards]
    m = merge_shards(pr, shards, fake)
    assert np.array_equal(m["pt_pos"], pr["pt_pos"])


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _gloo_worker(rank, world, port, q):
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parents[1]
    sys.path.insert(0, str(root))
    sys.path.insert(0, str(root / "tests"))
    import torch
    import torch.distributed as dist
    from c_orb_slam_amd.optimizer import merge_shards, partition_points, shard_problem
    from ba_cases import global_ba_problem as gbp
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        pr = gbp(11, n_kf=30, pts_per_kf=40)
        r = partition_points(pr, world)
        sh = shard_problem(pr, r, rank)
        # the structure-build exchange: union of active keyframes + global counts
        act = np.zeros(len(pr["kf_id"]) + 2)
        act[np.unique(sh["edge_kf"])] = 1
        act[-2] = len(sh["edge_pt"])
        act[-1] = len(sh["pt_id"])
        t = torch.from_numpy(act)
        dist.all_reduce(t)
        full = np.zeros(len(pr["kf_id"]))
        full[np.unique(pr["edge_kf"])] = 1
        ok_union = np.array_equal((t[:-2] > 0).numpy().astype(float), full)
        ok_counts = int(t[-2]) == len(pr["edge_pt"]) and int(t[-1]) == len(pr["pt_id"])
        # gather the shards' results (here: their inputs) and merge on rank 0
        mine = dict(pt_index=sh["pt_index"], edge_index=sh["edge_index"], pt_pos=sh["pt_pos"],
                    edge_pt=sh["edge_pt"])
        allv = [None] * world
        dist.all_gather_object(allv, mine)
        ok_merge = True
        if rank == 0:
            res = [dict(kf_Tcw=pr["kf_Tcw"], pt_pos=a["pt_pos"], edge_erase=np.zeros(len(a["edge_pt"]), bool),
                        iterations=(10, 0), aborted=False) for a in allv]
            m = merge_shards(pr, allv, res)
            ok_merge = np.array_equal(m["pt_pos"], pr["pt_pos"])
        q.put((rank, bool(ok_union), bool(ok_counts), bool(ok_merge)))
    finally:
        dist.destroy_process_group()


def test_gloo_two_ranks_exchange_and_merge():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_gloo_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(120)
    res = sorted(q.get(timeout=5) for _ in range(2))
    assert all(p.exitcode == 0 for p in ps)
    for rank, ok_union, ok_counts, ok_merge in res:
        assert ok_union and ok_counts and ok_merge, (rank, ok_union, ok_counts, ok_merge)


def test_sharded_entry_points_refuse_without_device():
    import c_orb_slam_amd as orb
    from c_orb_slam_amd.optimizer import BundleAdjustment, Comm, BundleAdjustmentSharded
    from c_orb_slam_amd._lib import OrbGpuError, ORB_E_INVALID, ORB_E_NODEVICE
    if orb.device_available():
        pytest.skip("device present")
    pr = global_ba_problem(0, n_kf=4, pts_per_kf=10)
    with pytest.raises(OrbGpuError) as e:
        BundleAdjustment(pr, -1, False)
    assert e.value.code == ORB_E_INVALID
    with pytest.raises(OrbGpuError) as e:
        BundleAdjustment(pr, 10, False)
    assert e.value.code == ORB_E_NODEVICE
    comms = Comm.local_group(2)
    assert comms[1].rank_size == (1, 2)
    with pytest.raises(OrbGpuError) as e:
        BundleAdjustmentSharded(pr, comms[0], 10, False)
    assert e.value.code == ORB_E_NODEVICE
    for c in comms:
        c.close()
