#!/usr/bin/env python3
"""Benchmark: KITTI-00 stereo tracking front end on MI355X (+ local and global BA legs).

Metric (BASELINE.json): "tracking FPS + ORB matches/sec, KITTI-00 stereo; local-BA iter/sec".
Workload at N=1 (BASELINE configs[1]/[2]): KITTI 00 stereo, 1241x376 u8 pairs, nFeatures
1200, 8 levels x1.2, FAST 20/7.  One step = one batch of B stereo frames
already resident in HBM: Frame(imLeft, imRight) -- ORBextractor::operator() on both images
(Frame.cc:78-81) and ComputeStereoMatches (Frame.cc:466-640) -- then
TrackWithMotionModel's SearchByProjection(CurrentFrame, LastFrame, th=7, stereo) for the
B-1 consecutive pairs (Tracking.cc:867-885), the last frame's map points lifted from its
stereo depth (UpdateLastFrame), and Optimizer::PoseOptimization(&mCurrentFrame) on the
matched map points (Tracking.cc:887, Optimizer.cc:239-451), device-resident end to end.
value = stereo frames/s.

Extraction + matching do not shard within a sequence (frame t+1 needs frame t), so N GPUs
run N independent replicas ("replicas only"); value is the frames of all ranks /
the max-over-ranks wall time.  The global-BA leg is ONE problem keyframe-block sharded over
the N ranks with an RCCL exchange per LM trial (strong scaling, reported in `global_ba`).

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
ROOFLINE_REPS = 5
TRAFFIC_FILE = "traffic_r01.json"   # PMC FETCH_SIZE/WRITE_SIZE per launch (tools/pmc_traffic.py)
VALU_FILE = "valu_r01.json"   # PMC SQ_INSTS_VALU per launch (tools/pmc_valu.py)
VALU_PEAK_GINST = 1228.8   # 256 CUs x 2 wave64 VALU issues per cycle x 2.4 GHz (MI355X_MICROARCH.md)
W, H, NFEAT = 1241, 376, 1200


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None, help="GPUs (one rank each); default: WORLD_SIZE or 1")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher check without a GPU: ranks meet over gloo and rank 0 prints n_gpus")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=64, help="stereo frames per step")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="budget of the CPU-baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--reserve-cus", type=int, default=0,
                    help="extractor streams leave out one CU in N for the tracking lane (0: off)")
    ap.add_argument("--gba-kf", type=int, default=2000,
                    help="keyframes of the sharded global-BA problem (SURVEY config 5: 2k, 8k, 16k)")
    ap.add_argument("--gba-reps", type=int, default=3)
    return ap.parse_args()


def lift_depth(rng, n):
    return rng.uniform(5.0, 50.0, size=n).astype(np.float32)


def launch_ranks(args):
    """`bench.py --gpus N` without a launcher: start N fresh rank processes (one per GPU) before
    this process touches the GPU, relay rank 0's JSON line, exit with the worst exit code.
    Under torch.distributed.run WORLD_SIZE is already set and this is not used."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, str(Path(__file__).resolve())] + sys.argv[1:], env=env,
                                      stdout=subprocess.PIPE if r == 0 else subprocess.DEVNULL))
    out = procs[0].stdout.read()
    codes = [p.wait() for p in procs]
    sys.stdout.write(out.decode())
    sys.stdout.flush()
    return next((c for c in codes if c != 0), 0)


def dry_run(args):
    """The rank plumbing of main() on gloo (CPU): every rank joins, rank 0 prints what the real run
    would report as n_gpus / parallelism (tests/test_bench_launcher.py)."""
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    seen = world
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo")
        t = torch.ones(1)
        dist.all_reduce(t)
        seen = int(t.item())
        dist.destroy_process_group()
    if rank == 0:
        print(json.dumps({"n_gpus": world, "ranks_joined": seen, "parallelism": f"replicas{world}"}), flush=True)


def main():
    args = parse()
    env_world = os.environ.get("WORLD_SIZE")
    if args.gpus is None:
        args.gpus = int(env_world or 1)
    if env_world is None and args.gpus > 1:
        sys.exit(launch_ranks(args))
    if env_world is not None and int(env_world) != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={env_world} (launch one rank per GPU)")
    if args.dry_run:
        return dry_run(args)
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
    lefts, rights, Hs, Rs = synthetic.stereo_sequence(1000 + rank, B, W, H, return_rotations=True)
    K4 = synthetic.intrinsics(W, H)
    fx, fy, cx, cy = (np.float32(v) for v in K4)
    mbf = np.float32(synthetic.KITTI_BF)
    mb = np.float32(mbf / fx)
    cap = 2 * NFEAT + 64

    m = orb.ORBmatcher(0.9, True)
    L = lib()
    check(L.ORBmatcher_set_device_pointers(m._h, 1))
    d_L = torch.from_numpy(lefts).to(dev)
    d_R = torch.from_numpy(rights).to(dev)
    d_obs = torch.ones(cap, dtype=torch.int32, device=dev)
    d_outlier = torch.zeros(cap, dtype=torch.uint8, device=dev)
    eye = torch.eye(4, dtype=torch.float32, device=dev)
    poses = torch.from_numpy(np.stack([synthetic.pose_from_rotation(R) for R in Rs])).to(dev)
    gW = np.float32(np.float32(64) / np.float32(W))
    gH = np.float32(np.float32(48) / np.float32(H))
    P = B - 1
    arr = lambda xs: (C.c_void_p * len(xs))(*xs)
    from c_orb_slam_amd._lib import orb_unproject, pose_frame
    from concurrent.futures import ThreadPoolExecutor
    # HIP's current device is per thread: every worker binds it first
    pool = ThreadPoolExecutor(2, initializer=lambda: torch.cuda.set_device(dev))
    match_stream = torch.cuda.ExternalStream(L.ORBmatcher_stream(m._h), device=dev)

    def n_field(arr, cls, count):
        """int32 view of field 0 (the count N) of every struct of a ctypes struct array."""
        w = C.sizeof(cls) // 4
        return np.ctypeslib.as_array((C.c_int32 * (count * w)).from_address(C.addressof(arr))).reshape(count, w)[:, 0]

    class Lane:
        """One batch in flight: its own extractor pair (pyramids, keypoints) and tracking buffers."""

        def __init__(self):
            self.exL = orb.ORBextractor(NFEAT, 1.2, 8, 20, 7, max_width=W, max_height=H, max_batch=B)
            self.exR = orb.ORBextractor(NFEAT, 1.2, 8, 20, 7, max_width=W, max_height=H, max_batch=B)
            self.d_kps = torch.empty((B, cap, 7), dtype=torch.int32, device=dev)   # mvKeys (== mvKeysUn, KITTI k1=0)
            self.d_desc = torch.empty((B, cap, 32), dtype=torch.uint8, device=dev)
            self.d_kpsR = torch.empty((B, cap, 7), dtype=torch.int32, device=dev)
            self.d_descR = torch.empty((B, cap, 32), dtype=torch.uint8, device=dev)
            self.d_uR = torch.empty((B, cap), dtype=torch.float32, device=dev)      # mvuRight
            self.d_depth = torch.empty((B, cap), dtype=torch.float32, device=dev)   # mvDepth
            self.d_mp_pos = torch.empty((B, cap, 3), dtype=torch.float32, device=dev)
            self.d_last_mp = torch.empty((B, cap), dtype=torch.int32, device=dev)
            self.d_cur_mp = torch.empty((B, cap), dtype=torch.int32, device=dev)
            self.scale = torch.from_numpy(self.exL.GetScaleFactors()).to(dev)
            self.d_Tout = torch.empty((P, 16), dtype=torch.float32, device=dev)
            self.d_poutl = torch.zeros((P, cap), dtype=torch.uint8, device=dev)
            self.isig_tab = torch.from_numpy(self.exL.GetInverseScaleSigmaSquares()).to(dev)
            # ctypes views of the batch, built once (device pointers do not move; only counts change)
            self.curs = (orb_frame * P)(*[self.frame_struct(b, poses[b - 1].data_ptr()) for b in range(1, B)])
            self.lasts = (orb_frame * P)(*[self.frame_struct(b, eye.data_ptr()) for b in range(0, B - 1)])
            self.mps = (orb_mappoints * P)()
            for p in range(P):
                self.mps[p].pos = self.d_mp_pos[p].data_ptr()
                self.mps[p].desc = self.d_desc[p].data_ptr()
                self.mps[p].observations = d_obs.data_ptr()
            self.a_cur_mp = arr([self.d_cur_mp[b].data_ptr() for b in range(1, B)])
            self.a_last_kps = arr([self.d_kps[b].data_ptr() for b in range(P)])
            self.a_last_mp = arr([self.d_last_mp[b].data_ptr() for b in range(P)])
            self.a_last_out = arr([d_outlier.data_ptr()] * P)
            self.s_kL = arr([self.d_kps[b].data_ptr() for b in range(B)])
            self.s_dL = arr([self.d_desc[b].data_ptr() for b in range(B)])
            self.s_kR = arr([self.d_kpsR[b].data_ptr() for b in range(B)])
            self.s_dR = arr([self.d_descR[b].data_ptr() for b in range(B)])
            self.s_uR = arr([self.d_uR[b].data_ptr() for b in range(B)])
            self.s_dep = arr([self.d_depth[b].data_ptr() for b in range(B)])
            # UpdateLastFrame: Frame::UnprojectStereo of frame b's stereo keypoints (Twc = I: the last
            # frame is the reference) -> the map point table of pair b and LastFrame.mvpMapPoints
            self.unp = (orb_unproject * B)(*[
                orb_unproject(0, self.d_kps[b].data_ptr(), self.d_depth[b].data_ptr(), eye.data_ptr(), float(fx),
                              float(fy), float(cx), float(cy), self.d_mp_pos[b].data_ptr(),
                              self.d_last_mp[b].data_ptr()) for b in range(B)])
            # PoseOptimization(&mCurrentFrame): the frame's own arrays, map points by index
            self.pframes = (pose_frame * P)(*[
                pose_frame(0, poses[p].data_ptr(), self.d_cur_mp[p + 1].data_ptr(), self.d_mp_pos[p].data_ptr(),
                           self.d_kps[p + 1].data_ptr(), self.d_uR[p + 1].data_ptr(), self.isig_tab.data_ptr(), 8,
                           float(fx), float(fy), float(cx), float(cy), float(mbf)) for p in range(P)])
            self.a_Tout = arr([self.d_Tout[p].data_ptr() for p in range(P)])
            self.a_poutl = arr([self.d_poutl[p].data_ptr() for p in range(P)])
            self.n_unp = n_field(self.unp, orb_unproject, B)
            self.n_cur = n_field(self.curs, orb_frame, P)
            self.n_last = n_field(self.lasts, orb_frame, P)
            self.n_mps = n_field(self.mps, orb_mappoints, P)
            self.n_pose = n_field(self.pframes, pose_frame, P)
            self.ninl = np.zeros(P, np.int32)
            self.nm = np.zeros(P, np.int32)
            self.nst = np.zeros(B, np.int32)
            self.nL = self.nR = None

        def frame_struct(self, b, Tptr):
            f = orb_frame()
            f.N = 0
            f.keysUn = self.d_kps[b].data_ptr()
            f.desc = self.d_desc[b].data_ptr()
            f.uRight = self.d_uR[b].data_ptr()
            f.minX, f.maxX, f.minY, f.maxY = 0.0, float(W), 0.0, float(H)
            f.gridWInv, f.gridHInv = gW, gH
            f.scaleFactors = self.scale.data_ptr()
            f.nlevels = 8
            f.fx, f.fy, f.cx, f.cy, f.bf, f.b = fx, fy, cx, cy, mbf, mb
            f.Tcw = Tptr
            return f

        def extract(self):
            # Frame(imLeft, imRight): two ORBextractor calls (Frame.cc:78-81) on two host threads and
            # two HIP streams, like the reference's two extractor threads per stereo frame
            fR = pool.submit(self.exR.extract_device, d_R.data_ptr(), B, W, H, W, W * H, self.d_kpsR.data_ptr(),
                             self.d_descR.data_ptr(), cap)
            self.nL = np.ascontiguousarray(self.exL.extract_device(d_L.data_ptr(), B, W, H, W, W * H,
                                                                   self.d_kps.data_ptr(), self.d_desc.data_ptr(), cap),
                                           np.int32)
            self.nR = np.ascontiguousarray(fR.result(), np.int32)

        def track(self):
            """ComputeStereoMatches, UpdateLastFrame, SearchByProjection(Cur, Last, 7), PoseOptimization."""
            t1 = time.perf_counter()
            nL, nR = self.nL, self.nR
            check(L.ORBmatcher_ComputeStereoMatches_batch(m._h, self.exL._h, self.exR._h, B, ptr(nL), self.s_kL,
                                                          self.s_dL, ptr(nR), self.s_kR, self.s_dR, float(mbf),
                                                          float(mb), self.s_uR, self.s_dep, ptr(self.nst)),
                  "ComputeStereoMatches batch")
            t2 = time.perf_counter()
            # UpdateLastFrame (Frame::UnprojectStereo) and the current frames' empty mvpMapPoints, on
            # the matcher's stream ahead of the search
            self.n_unp[:] = nL
            self.n_cur[:] = nL[1:]
            self.n_last[:] = nL[:-1]
            self.n_mps[:] = nL[:-1]
            self.n_pose[:] = nL[1:]
            check(L.Frame_UnprojectStereo_batch_device(m._h, B, self.unp), "UnprojectStereo batch")
            with torch.cuda.stream(match_stream):
                self.d_cur_mp.fill_(-1)
            # TrackWithMotionModel: SearchByProjection(CurrentFrame, LastFrame, th=7, stereo) (Tracking.cc:869-885)
            check(L.ORBmatcher_SearchByProjection_LastFrame_batch(m._h, P, self.curs, self.a_cur_mp, self.lasts,
                                                                  self.a_last_kps, self.a_last_mp, self.a_last_out,
                                                                  self.mps, 7.0, 0, ptr(self.nm)),
                  "SearchByProjection batch")
            t3 = time.perf_counter()
            # Optimizer::PoseOptimization(&mCurrentFrame) (Tracking.cc:887) on the matched map points
            check(L.Optimizer_PoseOptimization_frames_device(P, self.pframes, self.a_Tout, self.a_poutl,
                                                             ptr(self.ninl)), "PoseOptimization batch")
            t4 = time.perf_counter()
            for k, v in (("stereo", t2 - t1), ("lift+search", t3 - t2), ("pose", t4 - t3)):
                phase_acc[k] = phase_acc.get(k, 0.0) + v * 1e3
            tl, tr = self.exL.last_timings(), self.exR.last_timings()
            for k in tl:
                stage_acc[k] = stage_acc.get(k, 0.0) + tl[k] + tr[k]
            kernel_ms.append(tl["fast_cells"])
            kernel_ms.append(tr["fast_cells"])
            pose_inl.append(int(self.ninl.sum()))
            return int(nL.sum() + nR.sum()), int(self.nm.sum()), int(self.nst.sum())

    stage_acc = {}
    phase_acc = {}
    pose_inl = []
    kernel_ms = []   # k_fast_cells duration per step (HIP events on the extractor streams)
    lanes = [Lane(), Lane()]
    exL = lanes[0].exL
    if args.reserve_cus:
        # the tracking lane's one-workgroup-per-frame kernels (k_select, k_pose_opt) need free
        # wave slots while a batch is extracted: the extractor streams leave 1 CU in N out
        for ln in lanes:
            for ex in (ln.exL, ln.exR):
                check(L.ORBextractor_reserve_cus(ex._h, args.reserve_cus), "ORBextractor_reserve_cus")
    ex_pool = ThreadPoolExecutor(1, initializer=lambda: torch.cuda.set_device(dev))
    state = {"k": 0, "ready": None}

    def step():
        """Software pipeline over two lanes: the extraction of batch k (worker threads, extractor
        streams) runs while batch k-1 is tracked on this thread (matcher / pose / torch streams)."""
        lane = lanes[state["k"] % 2]
        te = time.perf_counter()
        fut = ex_pool.submit(lane.extract)
        res = (0, 0, 0)
        if state["ready"] is not None:
            res = state["ready"].track()
        fut.result()
        phase_acc["step_wall"] = phase_acc.get("step_wall", 0.0) + (time.perf_counter() - te) * 1e3
        state["ready"] = lane
        state["k"] += 1
        return res

    def drain():
        if state["ready"] is not None:
            state["ready"].track()
            state["ready"] = None

    for _ in range(args.warmup):
        step()
    drain()
    step()   # prime the pipeline: one batch extracted, awaiting tracking
    stage_acc.clear()
    phase_acc.clear()
    kernel_ms.clear()
    pose_inl.clear()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    tot_kp = tot_match = tot_stereo = 0
    for _ in range(args.steps):
        a, b, c = step()
        tot_kp += a
        tot_match += b
        tot_stereo += c
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if os.environ.get("ORBGPU_PROF_DUMP"):   # instrumented build (make prof): k_select section timers
        buf = (C.c_ulonglong * 32)()
        L.orbgpu_debug_prof_match(buf)
        print("k_select sections (cycles, problem 0, summed over the timed steps):", list(buf)[:8], file=sys.stderr)
    drain()   # the batch extracted by the last timed step (outside the timed region)
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
        c = torch.tensor([tot_match, tot_kp, tot_stereo], dtype=torch.float64, device=dev)
        dist.all_reduce(c)
        tot_match, tot_kp, tot_stereo = (int(v) for v in c.tolist())
    frames_total = B * args.steps * world
    fps = frames_total / dt

    # roofline of the dominant extraction kernel (k_fast_cells), measured in its own pass after
    # the timed region: inside the pipeline the kernel shares the GPU with the other extractor
    # and the tracking lane, so its event duration there is a share of the chip, not its speed.
    # ROOFLINE_REPS extractions of the left batch on one extractor, nothing else in flight; the
    # duration is HIP events on that extractor's stream (last_timings()["fast_cells"]).  These
    # are the last ROOFLINE_REPS k_fast_cells launches of the run (tools/roofline_check.py).
    # Algorithmic bytes per launch = every level pixel read once (sum P_l = 1,444,097 B per
    # KITTI image) + 4 B per corner written + 4 B per cell count, over B images.
    torch.cuda.synchronize()
    check(L.ORBextractor_reserve_cus(exL._h, 0), "ORBextractor_reserve_cus")   # the whole device
    iso_ms = []
    for _ in range(ROOFLINE_REPS):
        exL.extract_device(d_L.data_ptr(), B, W, H, W, W * H, lanes[0].d_kps.data_ptr(), lanes[0].d_desc.data_ptr(), cap)
        iso_ms.append(exL.last_timings()["fast_cells"])
    lvl_px = sum(int(round(W / 1.2 ** l)) * int(round(H / 1.2 ** l)) for l in range(8))
    cand_per_img = 13000  # FAST corners kept per image after NMS (order of magnitude, measured)
    alg_bytes = B * (lvl_px + 4 * cand_per_img + 4 * 1220)
    k_avg_ms = float(np.mean(iso_ms))
    achieved = alg_bytes / (k_avg_ms * 1e-3) / 1e9
    traffic = traffic_src = None
    tf = ROOT / "profiles" / TRAFFIC_FILE
    if tf.exists():
        try:
            traffic = json.loads(tf.read_text())["k_fast_cells"]["hbm_bytes_per_launch"]
            traffic_src = f"profiles/{TRAFFIC_FILE}"
        except Exception:
            traffic = None
    valu = None
    vf = ROOT / "profiles" / VALU_FILE
    if vf.exists():
        try:
            vi = json.loads(vf.read_text())["k_fast_cells"]["valu_insts_per_launch"]
            vr = vi / (k_avg_ms * 1e-3) / 1e9
            valu = {"insts_per_launch": round(vi), "achieved": round(vr, 1), "peak": VALU_PEAK_GINST,
                    "unit": "G wave-instr/s", "frac": round(vr / VALU_PEAK_GINST, 4), "source": f"profiles/{VALU_FILE}"}
        except Exception:
            valu = None
    roof = {"bound": "hbm", "kernel": "k_fast_cells", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
            "traffic_source": traffic_src, "avg_launch_ms": round(k_avg_ms, 4), "launches": ROOFLINE_REPS,
            "alg_bytes_per_launch": alg_bytes,
            "avg_launch_ms_in_pipeline": round(float(np.mean(kernel_ms)), 4),
            "secondary_bound": "VALU (16-px circle test; DESIGN.md §3)", "valu": valu}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(lefts, rights, Rs, args.cpu_seconds)

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
            "data": "synthetic (seeded KITTI-shaped textured stereo frames: camera-rotation motion, "
                    "ground-plane disparity field 4..40 px)",
            "config": {"workload": "kitti00_stereo: ORB extract L+R, ComputeStereoMatches, "
                                   "SearchByProjection(Cur,Last,th=7), PoseOptimization", "width": W, "height": H,
                       "nfeatures": NFEAT, "nlevels": 8, "scale_factor": 1.2, "fast_th": [20, 7],
                       "stereo_frames_per_step": B, "parallelism": f"replicas{world}", "extractor_cu_reserve": args.reserve_cus},
            "matches_per_s": round(tot_match / dt, 1), "stereo_matches_per_s": round(tot_stereo / dt, 1),
            "keypoints_per_image": round(tot_kp / (2 * frames_total), 1),
            "pose_inliers_per_frame": round(float(np.sum(pose_inl)) / max(len(pose_inl) * P, 1), 1),
            "stage_ms_per_step": stage_ms,
            "phase_ms_per_step": {k: round(v / args.steps, 4) for k, v in phase_acc.items()}, "roofline": roof, "cpu_baseline": cpu, "local_ba": ba,
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


class _CpuStream:
    """One reference-structured CPU tracking stream on the oracle (line-faithful C restatement):
    per stereo frame extract L and R, ComputeStereoMatches, SearchByProjection(Cur, Last, 7),
    PoseOptimization.  The oracle's C calls release the GIL, so streams run on separate cores."""

    def __init__(self, lefts, rights, Rs):
        sys.path.insert(0, str(ROOT / "tests"))
        import oracle_lib
        from c_orb_slam_amd import synthetic
        self.ol = oracle_lib
        self.lefts, self.rights, self.Rs = lefts, rights, Rs
        self.eL = oracle_lib.OracleExtractor(NFEAT, 1.2, 8, 20, 7)
        self.eR = oracle_lib.OracleExtractor(NFEAT, 1.2, 8, 20, 7)
        self.scale = self.eL.tables()["scale"]
        self.isig = self.eL.tables()["inv_sigma2"]
        self.fx, self.fy, self.cx, self.cy = synthetic.intrinsics(W, H)
        self.mbf = np.float32(synthetic.KITTI_BF)
        self.mb = np.float32(self.mbf / np.float32(self.fx))
        self.synthetic = synthetic
        self.prev = None
        self.t = {"extract": 0.0, "stereo": 0.0, "match": 0.0, "pose": 0.0}
        self.done = 0

    def frame(self, i):
        from c_orb_slam_amd.orb import Frame, MapPoints
        ol, fx, fy, cx, cy, mbf = self.ol, self.fx, self.fy, self.cx, self.cy, self.mbf
        ta = time.perf_counter()
        kL, dL = self.eL(self.lefts[i])
        kR, dR = self.eR(self.rights[i])
        tb = time.perf_counter()
        uR, dep, _ = ol.oracle_stereo_matches(self.eL, self.eR, kL, dL, kR, dR, H, mbf, self.mb)
        tc = time.perf_counter()
        self.t["extract"] += tb - ta
        self.t["stereo"] += tc - tb
        if self.prev is not None and i != 0:
            pk, pd, pdep = self.prev
            last = Frame(pk, pd, self.scale, np.eye(4, dtype=np.float32), fx, fy, cx, cy, mbf, W, H)
            cur = Frame(kL, dL, self.scale, self.synthetic.pose_from_rotation(self.Rs[i - 1]), fx, fy, cx, cy, mbf,
                        W, H, uRight=uR)
            X, lm = ol.oracle_unproject_stereo(pk, pdep, np.eye(4, dtype=np.float32), fx, fy, cx, cy)
            X = np.nan_to_num(X)
            mps = MapPoints(X, pd, np.ones(len(pk), np.int32))
            cm = np.full(cur.N, -1, np.int32)
            td = time.perf_counter()
            ol.oracle_search_last(cur, cm, last, pk, lm, np.zeros(len(pk), np.uint8), mps, 7.0, False, 0.9, True)
            te = time.perf_counter()
            self.t["match"] += te - td
            has = (cm >= 0).astype(np.uint8)
            pr = dict(Tcw=cur.Tcw, has_mp=has, Xw=X[np.maximum(cm, 0)],
                      obs=np.stack([kL["x"], kL["y"], uR], 1).astype(np.float32),
                      inv_sigma2=self.isig[kL["octave"]].astype(np.float32), cam=(fx, fy, cx, cy, mbf))
            ol.oracle_pose_optimization(pr)
            self.t["pose"] += time.perf_counter() - te
        self.prev = (kL, dL, dep)
        self.done += 1

    def run(self, start, budget_s, min_frames):
        t0 = time.perf_counter()
        i = start
        while True:
            self.frame(i % len(self.lefts))
            i += 1
            if time.perf_counter() - t0 > budget_s and self.done >= min_frames:
                return time.perf_counter() - t0


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(lefts, rights, Rs, budget_s):
    """The oracle timed on the host cores on a bounded sample of the same workload:
    (i) one reference-structured stream on 1 thread; (ii) P independent streams on P threads
    (P = this box's CPU share, at most 16) -> whole-host frames/s, the figure `value` reports."""
    from concurrent.futures import ThreadPoolExecutor
    one = _CpuStream(lefts, rights, Rs)
    one.run(0, budget_s / 2, 4)
    fps1 = one.done / sum(one.t.values())
    try:
        share = len(os.sched_getaffinity(0))
    except AttributeError:
        share = os.cpu_count() or 1
    P = max(1, min(16, share))
    streams = [_CpuStream(lefts, rights, Rs) for _ in range(P)]
    with ThreadPoolExecutor(P) as ex:
        walls = list(ex.map(lambda a: a[1].run(a[0] * 7, budget_s / 2, 2), enumerate(streams)))
    framesP = sum(s.done for s in streams)
    fpsP = framesP / max(walls)
    t = one.t
    return {"value": round(fpsP, 3), "unit": "frames/s", "cores": P, "kind": "port",
            "sample": f"{P} independent reference-structured streams on {P} threads ({_cpu_model()}): oracle "
                      f"ORBextractor x2 + ComputeStereoMatches + SearchByProjection(Cur,Last,7) + PoseOptimization "
                      f"per stereo frame, -O2 C restatement; {framesP} frames in {max(walls):.1f} s",
            "single_thread": {"value": round(fps1, 3), "unit": "frames/s", "cores": 1,
                              "sample": f"{one.done} frames on 1 thread: extract {t['extract'] / one.done * 1e3:.1f} "
                                        f"ms/frame, stereo {t['stereo'] / one.done * 1e3:.2f} ms, match "
                                        f"{t['match'] / max(one.done - 1, 1) * 1e3:.2f} ms, pose "
                                        f"{t['pose'] / max(one.done - 1, 1) * 1e3:.2f} ms"}}


if __name__ == "__main__":
    main()
