"""The sharded BA protocol across PROCESSES on one GPU (Optimizer.cc:49-237,
453-778).  Each rank is a fresh Python process (tests/ba_rank_worker.py, started like bench.py's
launch_ranks: a child process per rank) with its own HIP context, BA engine and shard; the ranks
exchange through orbgpu_comm_init_shm (host shared memory: RCCL cannot place two ranks on one
GPU).  This runs what the in-process thread group cannot: per-process shards, the group set-up
across processes and the per-LM-trial exchange order between independent processes.

Checks: every rank holds the same poses; the merged result is bit-identical to the in-process
group on the same partition (the shared-memory transport sums in the same rank order); against
the oracle the iteration count and the chi2 trace agree (1e-9) and poses / points to 1e-5."""
import os
import subprocess
import sys
import uuid
from pathlib import Path

import numpy as np
import pytest

import oracle_lib
from ba_cases import ba_problem, global_ba_problem

pytestmark = pytest.mark.gpu
WORKER = Path(__file__).resolve().parent / "ba_rank_worker.py"


def _run_processes(problem, pt_rank, nranks, mode, its, tmp_path, cap=8 << 20):
    from c_orb_slam_amd.optimizer import merge_shards, shard_problem
    shards = [shard_problem(problem, pt_rank, r) for r in range(nranks)]
    for r, sh in enumerate(shards):
        np.savez(tmp_path / f"shard{r}.npz", **{k: np.asarray(v) for k, v in sh.items()})
    name = f"/orbgpu_t{uuid.uuid4().hex[:16]}"
    env = dict(os.environ, ORBGPU_SHM_TIMEOUT="120")
    procs = [subprocess.Popen([sys.executable, str(WORKER), str(tmp_path), str(r), str(nranks), name, mode, str(its),
                               str(cap)], env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
             for r in range(nranks)]
    outs = []
    try:
        for p in procs:
            out, _ = p.communicate(timeout=240)
            outs.append(out)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    for r, (p, out) in enumerate(zip(procs, outs)):
        assert p.returncode == 0, f"rank {r} exit {p.returncode}:\n{out[-2000:]}"
    res = []
    for r in range(nranks):
        z = np.load(tmp_path / f"result{r}.npz")
        d = {k: z[k] for k in z.files}
        d["iterations"] = tuple(int(v) for v in d["iterations"])
        d["aborted"] = False
        res.append(d)
    return merge_shards(problem, shards, res), res


@pytest.mark.parametrize("nranks", [2, 3])
def test_global_ba_processes_sharded_factorisation(gpu, tmp_path, nranks):
    from c_orb_slam_amd.optimizer import partition_points_nd, run_sharded_local
    pr = global_ba_problem(7, n_kf=400, pts_per_kf=60, laps=4)
    pt_rank = partition_points_nd(pr, nranks)
    s, per = _run_processes(pr, pt_rank, nranks, "global", 10, tmp_path)
    for r in per:
        assert r["sharding"][0] == 1, r["sharding"]   # the separator-tree exchange ran
        assert np.array_equal(r["kf_Tcw"], per[0]["kf_Tcw"])
        assert r["iterations"] == per[0]["iterations"]
    # the same protocol on in-process ranks (threads): the same bits
    t, _ = run_sharded_local(pr, nranks, "global", 10, False, trace=True, pt_rank=pt_rank)
    assert s["iterations"] == t["iterations"]
    assert np.array_equal(s["kf_Tcw"], t["kf_Tcw"]) and np.array_equal(s["pt_pos"], t["pt_pos"])
    assert np.array_equal(s["solve_chi2"], t["solve_chi2"])
    o = oracle_lib.oracle_global_ba(pr, 10, False)
    assert s["iterations"] == o["iterations"]
    np.testing.assert_allclose(s["solve_chi2"], o["solve_chi2"], rtol=1e-9)
    np.testing.assert_allclose(s["kf_Tcw"], o["kf_Tcw"].reshape(s["kf_Tcw"].shape), rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(s["pt_pos"], o["pt_pos"].reshape(s["pt_pos"].shape), rtol=1e-5, atol=1e-5)


def test_local_ba_processes_keyframe_blocks(gpu, tmp_path):
    """LocalBundleAdjustment (config 4) keyframe-block sharded over two processes: optimize(5),
    the outlier gating (erased edges) and optimize(10), against the in-process group and the oracle."""
    from c_orb_slam_amd.optimizer import partition_points, run_sharded_local
    pr = ba_problem(3)
    pt_rank = partition_points(pr, 2)
    s, per = _run_processes(pr, pt_rank, 2, "local", 0, tmp_path)
    assert np.array_equal(per[1]["kf_Tcw"], per[0]["kf_Tcw"])
    t, _ = run_sharded_local(pr, 2, "local", trace=True, pt_rank=pt_rank)
    assert s["iterations"] == t["iterations"]
    assert np.array_equal(s["kf_Tcw"], t["kf_Tcw"]) and np.array_equal(s["pt_pos"], t["pt_pos"])
    assert np.array_equal(s["edge_erase"], t["edge_erase"])
    o = oracle_lib.oracle_local_ba(pr)
    assert s["iterations"] == o["iterations"]
    assert np.array_equal(s["edge_erase"], o["edge_erase"].astype(bool))
    np.testing.assert_allclose(s["kf_Tcw"], o["kf_Tcw"].reshape(s["kf_Tcw"].shape), rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(s["pt_pos"], o["pt_pos"].reshape(s["pt_pos"].shape), rtol=1e-5, atol=1e-5)
