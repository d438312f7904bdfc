"""One rank of a multi-process sharded BA run (tests/test_gpu_ba_multiprocess.py): loads its shard
from <dir>/shard<rank>.npz, joins the shared-memory group (orbgpu_comm_init_shm), runs
Optimizer_BundleAdjustment_sharded / Optimizer_LocalBundleAdjustment_sharded and writes
<dir>/result<rank>.npz.  Started as a fresh process (subprocess), one per rank.
usage: ba_rank_worker.py <dir> <rank> <nranks> <shm name> <mode: global|local> <its> <max doubles>"""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main():
    d, rank, nranks, name, mode, its, cap = sys.argv[1:8]
    rank, nranks, its, cap = int(rank), int(nranks), int(its), int(cap)
    from c_orb_slam_amd.optimizer import (BundleAdjustmentSharded, Comm, LocalBundleAdjustmentSharded,
                                          last_sharding)
    z = np.load(Path(d) / f"shard{rank}.npz")   # our own arrays: no pickle
    shard = {k: z[k] for k in z.files}
    comm = Comm.shm(name, nranks, rank, cap)
    assert comm.rank_size == (rank, nranks)
    if mode == "global":
        r = BundleAdjustmentSharded(shard, comm, its, False, trace=True)
    else:
        r = LocalBundleAdjustmentSharded(shard, comm, trace=True)
    out = {k: np.asarray(v) for k, v in r.items() if k in ("kf_Tcw", "pt_pos", "edge_erase", "iterations",
                                                         "solve_chi2", "trial_chi2", "trial_lambda")}
    out["sharding"] = np.asarray(last_sharding())
    comm.close()
    np.savez(Path(d) / f"result{rank}.npz", **out)
    print(f"rank {rank}/{nranks}: {mode} iterations {out['iterations'].tolist()} sharding {out['sharding'].tolist()}",
          flush=True)


if __name__ == "__main__":
    main()
