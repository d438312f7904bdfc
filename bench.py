#!/usr/bin/env python3
"""Benchmark: ORB extract + guided Hamming match on KITTI-00-shaped frames (MI355X).

Metric (BASELINE.json): "tracking FPS + ORB matches/sec, KITTI-00 stereo; local-BA iter/sec".
Workload at N=1 (BASELINE configs[1]): KITTI 00 monocular, 1241x376 u8 frames,
nFeatures 1200, 8 levels x1.2, FAST 20/7; one step = one batch of
B frames already resident in HBM: ORBextractor::operator() on every frame, then
ORBmatcher::SearchByProjection(CurrentFrame, LastFrame, th=15, mono) for the
B-1 consecutive pairs (Tracking::TrackWithMotionModel, Tracking.cc:867-892),
with the last frame's map points lifted from its keypoints (synthetic depth).

Extraction + matching do not shard within a sequence (frame t+1 needs frame t),
so N GPUs run N independent replicas ("replicas only"); value is
the frames of all ranks / the max-over-ranks wall time.

Prints ONE JSON line (rank 0) with roofline + cpu_baseline objects.
"""
import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

METRIC = "tracking FPS + ORB matches/sec, KITTI-00 stereo; local-BA iter/sec"
HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md (spec)
W, H, NFEAT = 1241, 376, 1200


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=64, help="frames per step")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="budget of the CPU-baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--gba-kf", type=int, default=512, help="keyframes of the sharded global-BA problem")
    ap.add_argument("--gba-reps", type=int, default=3)
    return ap.parse_args()


def lift_depth(rng, n):
    return rng.uniform(5.0, 50.0, size=n).astype(np.float32)


def main():
    args = parse()
    # stdout carries exactly one JSON line: libraries that print banners at init (RCCL prints
    # its version block when a communicator is created) write to fd 1, so point fd 1 at
    # stderr for the run and keep the real stdout for the result.
    sys.stdout.flush()
    json_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    dev = torch.device("cuda", local_rank if world > 1 else 0)
    torch.cuda.set_device(dev)

    import ctypes as C
    import c_orb_slam_amd as orb
    from c_orb_slam_amd import synthetic
    from c_orb_slam_amd._lib import lib, orb_frame, orb_mappoints, ptr, check

    B = args.batch
    frames, Hs, Rs = synthetic.sequence(1000 + rank, B, W, H, return_rotations=True)
    K4 = synthetic.intrinsics(W, H)
    fx, fy, cx, cy = (np.float32(v) for v in K4)
    cap = 2 * NFEAT + 64

    ex = orb.ORBextractor(NFEAT, 1.2, 8, 20, 7, max_width=W, max_height=H, max_batch=B)
    m = orb.ORBmatcher(0.9, True)
    L = lib()
    check(L.ORBmatcher_set_device_pointers(m._h, 1))

    d_imgs = torch.from_numpy(frames).to(dev)
    d_kps = torch.empty((B, cap, 7), dtype=torch.int32, device=dev)
    d_desc = torch.empty((B, cap, 32), dtype=torch.uint8, device=dev)
    rng = np.random.default_rng(5 + rank)
    d_depth = torch.from_numpy(lift_depth(rng, B * cap).reshape(B, cap)).to(dev)
    d_obs = torch.ones(cap, dtype=torch.int32, device=dev)
    d_arange = torch.arange(cap, dtype=torch.int32, device=dev)
    d_outlier = torch.zeros(cap, dtype=torch.uint8, device=dev)
    d_mp_pos = torch.empty((B, cap, 3), dtype=torch.float32, device=dev)
    d_cur_mp = torch.empty((B, cap), dtype=torch.int32, device=dev)
    scale = torch.from_numpy(ex.GetScaleFactors()).to(dev)
    eye = torch.eye(4, dtype=torch.float32, device=dev)
    poses = torch.from_numpy(np.stack([synthetic.pose_from_rotation(R) for R in Rs])).to(dev)
    kp_f = d_kps.view(torch.float32)
    gW = np.float32(np.float32(64) / np.float32(W))
    gH = np.float32(np.float32(48) / np.float32(H))
    P = B - 1

    def frame_struct(b, n, Tptr):
        f = orb_frame()
        f.N = int(n)
        f.keysUn = d_kps[b].data_ptr()
        f.desc = d_desc[b].data_ptr()
        f.uRight = None
        f.minX, f.maxX, f.minY, f.maxY = 0.0, float(W), 0.0, float(H)
        f.gridWInv, f.gridHInv = gW, gH
        f.scaleFactors = scale.data_ptr()
        f.nlevels = 8
        f.fx, f.fy, f.cx, f.cy, f.bf, f.b = fx, fy, cx, cy, 0.0, 0.0
        f.Tcw = Tptr
        return f

    stage_acc = {}
    kernel_ms = []   # k_fast_cells duration per step (HIP events on the extractor stream)

    # ctypes views of the batch, built once (device pointers do not move; only counts change)
    curs = (orb_frame * P)(*[frame_struct(b, 0, poses[b - 1].data_ptr()) for b in range(1, B)])
    lasts = (orb_frame * P)(*[frame_struct(b, 0, eye.data_ptr()) for b in range(0, B - 1)])
    mps = (orb_mappoints * P)()
    for p in range(P):
        mps[p].pos = d_mp_pos[p].data_ptr()
        mps[p].desc = d_desc[p].data_ptr()
        mps[p].observations = d_obs.data_ptr()
    arr = lambda xs: (C.c_void_p * P)(*xs)
    a_cur_mp = arr([d_cur_mp[b].data_ptr() for b in range(1, B)])
    a_last_kps = arr([d_kps[b].data_ptr() for b in range(P)])
    a_last_mp = arr([d_arange.data_ptr()] * P)
    a_last_out = arr([d_outlier.data_ptr()] * P)
    nm = np.zeros(P, np.int32)

    def step():
        n = ex.extract_device(d_imgs.data_ptr(), B, W, H, W, W * H, d_kps.data_ptr(), d_desc.data_ptr(), cap)
        # last-frame map points: X = d K^-1 [u v 1] (UpdateLastFrame-style lift), on device
        x, y = kp_f[..., 0], kp_f[..., 1]
        d_mp_pos[..., 0] = (x - float(cx)) / float(fx) * d_depth
        d_mp_pos[..., 1] = (y - float(cy)) / float(fy) * d_depth
        d_mp_pos[..., 2] = d_depth
        d_cur_mp.fill_(-1)
        for p in range(P):
            curs[p].N = int(n[p + 1])
            lasts[p].N = int(n[p])
            mps[p].n = int(n[p])
        torch.cuda.current_stream().synchronize()
        check(L.ORBmatcher_SearchByProjection_LastFrame_batch(m._h, P, curs, a_cur_mp, lasts, a_last_kps, a_last_mp,
                                                              a_last_out, mps, 15.0, 1, ptr(nm)),
              "SearchByProjection batch")
        t = ex.last_timings()
        for k, v in t.items():
            stage_acc[k] = stage_acc.get(k, 0.0) + v
        kernel_ms.append(t["fast_cells"])
        return int(n.sum()), int(nm.sum())

    for _ in range(args.warmup):
        step()
    stage_acc.clear()
    kernel_ms.clear()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    tot_kp = tot_match = 0
    for _ in range(args.steps):
        a, b = step()
        tot_kp += a
        tot_match += b
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
        c = torch.tensor([tot_match, tot_kp], dtype=torch.float64, device=dev)
        dist.all_reduce(c)
        tot_match, tot_kp = int(c[0].item()), int(c[1].item())
    frames_total = B * args.steps * world
    fps = frames_total / dt

    # roofline of the dominant device kernel (k_fast_cells): algorithmic bytes per launch
    # = every level pixel read once (sum P_l = 1,444,097 B per KITTI image) + 4 B per
    # candidate written + 4 B per cell count, over B images (DESIGN.md "Roofline").
    lvl_px = sum(int(round(W / 1.2 ** l)) * int(round(H / 1.2 ** l)) for l in range(8))
    cand_per_img = 13000  # measured order of magnitude of FAST candidates; refined by traffic json below
    alg_bytes = B * (lvl_px + 4 * cand_per_img + 4 * 1220)
    k_avg_ms = float(np.mean(kernel_ms))
    achieved = alg_bytes / (k_avg_ms * 1e-3) / 1e9
    traffic = None
    tf = ROOT / "profiles" / "traffic_r01.json"
    if tf.exists():
        try:
            traffic = json.loads(tf.read_text()).get("k_fast_cells_bytes_per_launch")
        except Exception:
            traffic = None
    roof = {"bound": "hbm", "kernel": "k_fast_cells", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
            "avg_launch_ms": round(k_avg_ms, 4), "alg_bytes_per_launch": alg_bytes}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(frames, Rs, args.cpu_seconds)

    # local BA (BASELINE metric part 3): SURVEY config 4 on every rank (replicas), own timed region
    ba = bench_local_ba(args, world, rank, dist if world > 1 else None, dev)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        ba["cpu_baseline"] = ba_cpu_baseline(args.cpu_seconds / 4)
    # global BA (SURVEY config 5): ONE problem keyframe-block sharded over the ranks, RCCL exchange
    gba = bench_global_ba(args, world, rank, dist if world > 1 else None, dev)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        gba["cpu_baseline"] = gba_cpu_baseline(args.gba_kf)

    if rank == 0:
        stage_ms = {k: round(v / args.steps, 4) for k, v in stage_acc.items()}
        out = {
            "metric": METRIC, "value": round(fps, 2), "unit": "frames/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u8",
            "data": "synthetic (seeded KITTI-shaped textured frames, camera-rotation motion)",
            "config": {"workload": "kitti00_mono_orb_extract+SearchByProjection(th=15)", "width": W, "height": H,
                       "nfeatures": NFEAT, "nlevels": 8, "scale_factor": 1.2, "fast_th": [20, 7],
                       "frames_per_step": B, "parallelism": f"replicas{world}"},
            "matches_per_s": round(tot_match / dt, 1), "keypoints_per_frame": round(tot_kp / frames_total, 1),
            "stage_ms_per_step": stage_ms, "roofline": roof, "cpu_baseline": cpu, "local_ba": ba,
            "global_ba": gba,
        }
        json_out.write(json.dumps(out) + "\n")
        json_out.flush()
    if world > 1:
        dist.destroy_process_group()


BA_KEYS = ("kf_id", "kf_Tcw", "kf_local", "kf_cam", "pt_id", "pt_pos", "edge_pt", "edge_kf", "edge_obs",
           "edge_inv_sigma2")


def bench_local_ba(args, world, rank, dist, dev):
    """Optimizer::LocalBundleAdjustment on SURVEY config 4 (EuRoC-shaped: 15 local + 15 fixed
    keyframes, 3000 points, ~15k edges, 70% stereo, 5% outliers); one iter = one LM solve()."""
    import torch
    sys.path.insert(0, str(ROOT / "tests"))
    from ba_cases import ba_problem
    from c_orb_slam_amd.optimizer import LocalBundleAdjustment
    pr = ba_problem(0)
    a = [pr[k] for k in BA_KEYS]
    for _ in range(3):
        LocalBundleAdjustment(*a)
    reps = max(5, args.steps * 2)
    if dist is not None:
        dist.barrier()
    t0 = time.perf_counter()
    its = 0
    for _ in range(reps):
        r = LocalBundleAdjustment(*a)
        its += sum(r["iterations"])
    dt = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([dt, its], dtype=torch.float64, device=dev)
        dist.all_reduce(t[:1], op=dist.ReduceOp.MAX)
        dist.all_reduce(t[1:])
        dt, its = float(t[0].item()), int(t[1].item())
    ne = len(pr["edge_pt"])
    return {"metric": "local-BA iter/s", "value": round(its / dt, 1), "unit": "iter/s",
            "ms_per_call": round(dt / (reps * max(world, 1)) * 1e3 * max(world, 1), 3),
            "edges_per_s": round(its * ne / dt, 1), "calls": reps * world,
            "config": {"workload": "euroc_mh05_stereo_local_ba (SURVEY config 4)", "local_kfs": 15, "fixed_kfs": 15,
                       "points": len(pr["pt_id"]), "edges": ne,
                       "stereo_edges": int((pr["edge_obs"][:, 2] >= 0).sum()),
                       "lm": "optimize(5) + gating + optimize(10)", "parallelism": f"replicas{world}"},
            "dtype": "f64 (f32 I/O)"}


def bench_global_ba(args, world, rank, dist, dev):
    """Optimizer::BundleAdjustment (nIterations=10, bRobust=false, LoopClosing.cc:650) on one
    merged-map-shaped problem (SURVEY config 5, KITTI intrinsics), keyframe-block sharded over
    the N ranks: per LM trial one RCCL all-reduce of the partial Schur complement over xGMI.
    Strong scaling: the problem is fixed, N ranks share it; iter = one LM solve()."""
    import torch
    sys.path.insert(0, str(ROOT / "tests"))
    from ba_cases import global_ba_problem
    from c_orb_slam_amd.optimizer import BundleAdjustmentSharded, Comm, partition_points, shard_problem
    pr = global_ba_problem(0, n_kf=args.gba_kf, pts_per_kf=150)
    shard = shard_problem(pr, partition_points(pr, world), rank)
    uid = [Comm.unique_id() if rank == 0 else None]
    if dist is not None:
        dist.broadcast_object_list(uid, src=0)
    comm = Comm.rccl(world, rank, uid[0])
    BundleAdjustmentSharded(shard, comm, 10, False)          # warm-up (allocations, structure)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    its = 0
    for _ in range(args.gba_reps):
        r = BundleAdjustmentSharded(shard, comm, 10, False)
        its += r["iterations"][0]
    dt = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    comm.close()
    ne = len(pr["edge_pt"])
    return {"metric": "global-BA iter/s", "value": round(its / dt, 2), "unit": "iter/s",
            "ms_per_call": round(dt / args.gba_reps * 1e3, 3), "edges_per_s": round(its * ne / dt, 1),
            "scaling": "strong", "calls": args.gba_reps,
            "config": {"workload": "kitti_merged_map_global_ba (SURVEY config 5)", "keyframes": args.gba_kf,
                       "points": len(pr["pt_id"]), "edges": ne, "edges_per_rank": len(shard["edge_pt"]),
                       "lm": "optimize(10), bRobust=false", "parallelism": f"keyframe-block shards x{world} (RCCL)"},
            "dtype": "f64 (f32 I/O)"}


def gba_cpu_baseline(n_kf):
    """Oracle BundleAdjustment (C restatement of the g2o path, 1 thread) on the same problem, one call."""
    sys.path.insert(0, str(ROOT / "tests"))
    import oracle_lib
    from ba_cases import global_ba_problem
    pr = global_ba_problem(0, n_kf=n_kf, pts_per_kf=150)
    t0 = time.perf_counter()
    o = oracle_lib.oracle_global_ba(pr, 2, False)   # bounded sample: the first 2 LM solves of the same call
    dt = time.perf_counter() - t0
    return {"value": round(o["iterations"][0] / dt, 3), "unit": "iter/s", "cores": 1, "kind": "port",
            "sample": f"BundleAdjustment(nIterations=2) on the same config-5 problem ({n_kf} KFs), "
                      f"oracle/ba.c -O2 (sparse Schur, envelope LDL^T), 1 thread"}


def ba_cpu_baseline(budget_s):
    """Oracle LocalBundleAdjustment (C restatement of the g2o path, 1 thread) on the same problem."""
    sys.path.insert(0, str(ROOT / "tests"))
    import oracle_lib
    from ba_cases import ba_problem
    pr = ba_problem(0)
    t0 = time.perf_counter()
    its = calls = 0
    while True:
        o = oracle_lib.oracle_local_ba(pr)
        its += sum(o["iterations"])
        calls += 1
        if time.perf_counter() - t0 > budget_s and calls >= 2:
            break
    dt = time.perf_counter() - t0
    return {"value": round(its / dt, 2), "unit": "iter/s", "cores": 1, "kind": "port",
            "sample": f"{calls} LocalBundleAdjustment calls on config 4 ({its} LM solves), oracle/ba.c -O2, 1 thread"}


def cpu_baseline(frames, Rs, budget_s):
    """Oracle (line-faithful C restatement, 1 thread) on a bounded sample of the same workload."""
    sys.path.insert(0, str(ROOT / "tests"))
    import oracle_lib
    from match_cases import frame_pair
    from c_orb_slam_amd import synthetic
    e = oracle_lib.OracleExtractor(NFEAT, 1.2, 8, 20, 7)
    scale = e.tables()["scale"]
    K4 = synthetic.intrinsics(W, H)
    t0 = time.perf_counter()
    done = 0
    prev = None
    extract_t = match_t = 0.0
    rng = np.random.default_rng(0)
    while True:
        img = frames[done % len(frames)]
        ta = time.perf_counter()
        k, d = e(img)
        tb = time.perf_counter()
        extract_t += tb - ta
        if prev is not None and done % len(frames) != 0:
            cur, last, mps, lm, lo = frame_pair(prev[0], prev[1], k, d, Rs[(done - 1) % len(Rs)], K4, W, H, scale,
                                                rng, obs_zero_fraction=0.0, outlier_fraction=0.0, mp_fraction=1.0)
            cm = np.full(cur.N, -1, np.int32)
            tc = time.perf_counter()
            oracle_lib.oracle_search_last(cur, cm, last, prev[0], lm, lo, mps, 15.0, True, 0.9, True)
            match_t += time.perf_counter() - tc
        prev = (k, d)
        done += 1
        if time.perf_counter() - t0 > budget_s and done >= 8:
            break
    fps = done / (extract_t + match_t)
    return {"value": round(fps, 3), "unit": "frames/s", "cores": 1, "kind": "port",
            "sample": f"{done} KITTI-shaped frames: oracle ORBextractor + SearchByProjection(Cur,Last,15) "
                      f"(extract {extract_t / done * 1e3:.1f} ms/frame, match {match_t / max(done - 1, 1) * 1e3:.2f} "
                      f"ms/pair, 1 thread, -O2 C restatement)"}


if __name__ == "__main__":
    main()
