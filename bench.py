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
TRAFFIC_FILE = "traffic_r05.json"   # PMC FETCH_SIZE/WRITE_SIZE per launch (tools/pmc_traffic.py)
VALU_FILE = "valu_r05.json"   # PMC SQ_INSTS_VALU per launch (tools/pmc_valu.py)
MATCH_PMC_FILE = "match_pmc_r05.json"   # matcher kernels: HBM bytes and VALU instructions per launch (tools/pmc_match.py)
STEREO_WINDOW_BYTES = 11 * 11 + 11 * 21   # per SAD-evaluated keypoint: left window + right search band
VALU_PEAK_GINST = 1228.8   # 256 CUs x 2 wave64 VALU issues per cycle x 2.4 GHz (MI355X_MICROARCH.md)
W, H, NFEAT = 1241, 376, 1200
K_LOCAL = 5   # local map = the map points of the last K_LOCAL frames (UpdateLocalMap's local keyframes)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None, help="GPUs (one rank each); default: WORLD_SIZE or 1")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher check without a GPU: ranks meet over gloo and rank 0 prints n_gpus")
    ap.add_argument("--steps", type=int, default=60)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=64, help="stereo frames per step")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="budget of the CPU-baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--reserve-cus", type=int, default=0,
                    help="extractor streams leave out one CU in N for the tracking lane (0: off)")
    ap.add_argument("--gba-kf", type=int, default=2000,
                    help="keyframes of the sharded global-BA problem (SURVEY config 5: 2k, 8k, 16k)")
    ap.add_argument("--gba-reps", type=int, default=3)
    ap.add_argument("--gba-laps", type=int, default=-1,
                    help="loop-closed map: the keyframes drive this many laps of one circuit (-1: one lap per "
                         "500 keyframes; 0: an open drive, a pure band)")
    ap.add_argument("--nfeatures", type=int, default=NFEAT,
                    help="ORBextractor nFeatures of the stereo pipeline (1200: the metric's; 2000: KITTI00-02.yaml)")
    ap.add_argument("--lanes", type=int, default=2,
                    help="batches in flight (buffer sets): extraction of batch k waits for the tracking chain "
                         "of batch k - lanes, which last used its buffers")
    ap.add_argument("--sequence", type=int, default=0,
                    help="1: sequence-shaped pipeline -- the B frame pairs of a step are B sequences in lock step "
                         "(sequence s tracks image s+t at step t): each pair's LastFrame pose and motion-model "
                         "prediction come from the previous steps' ESTIMATES (Tracking.cc:867-928), not the "
                         "generator's poses, so step t's tracking waits for step t-1's")
    ap.add_argument("--depth", type=int, default=1,
                    help="extractions in flight: 1 = batch k's extraction is submitted after batch k-1's chain "
                         "is enqueued and waited for within the step; 2 = batch k's extraction is queued at the "
                         "start of step k, before the host waits for batch k-1's (no idle extraction lane while "
                         "the host enqueues a chain; needs --lanes >= 3)")
    ap.add_argument("--shared-ex-stream", type=int, default=0,
                    help="1: every lane's extractor launches on the first lane's stream "
                         "(ORBextractor_share_stream), so with --depth 2 batch k+1's extraction is queued behind "
                         "batch k's on the device and starts with no gap; allows --depth 2 with 2 lanes (a lane's "
                         "extraction waits for its previous chain: ORBmatcher_chain_wait)")
    ap.add_argument("--h2d-streams", type=int, default=1,
                    help="host-IO leg: the step's H2D copy split over this many copy streams; 1 (default): "
                         "2 and 4 pieces were slower, 0.86 / 0.54-0.60 of value against 0.93-0.97 "
                         "(profiles/r06h2d_host_io_streams_ab.txt)")
    ap.add_argument("--lane-matchers", type=int, default=1,
                    help="1 (default): every lane after the first tracks on its own ORBmatcher (own stream, "
                         "arena and deferred chain), so the tracking chains of consecutive batches overlap on "
                         "the device instead of queueing on one stream (32.3-32.5k vs 29.6-29.7k frames/s with "
                         "0, profiles/r04n_lanes_ab.txt); 0: one matcher for every lane")
    ap.add_argument("--stereo-batch", type=int, default=1,
                    help="1 (default): Frame(imLeft, imRight)'s two extractions as ONE batch call of 2B images on "
                         "one extractor stream (ComputeStereoMatches_batch_at pairs image b with image B + b; "
                         "31.4-32.1k vs 30.2-30.4k frames/s with 0, profiles/r04b_lanes_ab.txt); 0: two "
                         "extractors on two host threads and two streams")
    ap.add_argument("--pipeline-only", action="store_true",
                    help="only the timed stereo pipeline (+ its CPU baseline): one compact JSON line")
    ap.add_argument("--launch-timeout", type=float, default=3000.0,
                    help="bound on the whole job when bench.py spawns its own ranks (seconds)")
    ap.add_argument("--enqueue-first", type=int, default=1,
                    help="1 (default): a step enqueues the ready batch's tracking chain before it starts the "
                         "next extraction, so the chain's and the extraction's host launches do not interleave "
                         "(32.9-33.1k vs 32.1-32.4k frames/s with 0, profiles/r04s_enqueue_first_ab.txt)")
    ap.add_argument("--latency-stereo-batch", type=int, default=1,
                    help="batch-1 latency leg, device path: 1 (default) one extractor call over the frame's two "
                         "images; 0: two extractors on two host threads")
    ap.add_argument("--latency-only", action="store_true",
                    help="only the batch-1 tracking latency legs (device and host path): one JSON line (A/B runs)")
    ap.add_argument("--passes-only", action="store_true",
                    help="only the isolated roofline passes (extraction + matcher kernels), for rocprofv3 --pmc runs")
    return ap.parse_args()


def lift_depth(rng, n):
    return rng.uniform(5.0, 50.0, size=n).astype(np.float32)


def launch_ranks(args):
    """`bench.py --gpus N` without a launcher: start N fresh rank processes (one per GPU) before
    this process touches the GPU, relay rank 0's JSON line, exit with the worst exit code.
    Every child is polled: when one exits non-zero (e.g. at RCCL init) the others, which would
    block in the rendezvous or a collective, are terminated and that code is returned; the
    whole job is bounded by --launch-timeout.  Under torch.distributed.run WORLD_SIZE is already
    set and this is not used."""
    import socket
    import subprocess
    import threading
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, str(Path(__file__).resolve())] + sys.argv[1:], env=env,
                                      stdout=subprocess.PIPE if r == 0 else subprocess.DEVNULL))
    out = []
    reader = threading.Thread(target=lambda: out.append(procs[0].stdout.read()), daemon=True)
    reader.start()
    deadline = time.monotonic() + args.launch_timeout
    failed = 0
    while True:
        codes = [p.poll() for p in procs]
        bad = [(r, c) for r, c in enumerate(codes) if c is not None and c != 0]
        if bad:
            failed = bad[0][1]
            sys.stderr.write(f"bench.py: rank {bad[0][0]} exited with {failed}; stopping the other ranks\n")
            break
        if all(c is not None for c in codes):
            break
        if time.monotonic() > deadline:
            failed = 124
            sys.stderr.write(f"bench.py: ranks still running after {args.launch_timeout:.0f} s; stopping them\n")
            break
        time.sleep(0.2)
    if failed:
        for p in procs:
            if p.poll() is None:
                p.terminate()
        for p in procs:
            try:
                p.wait(timeout=20)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
    reader.join(timeout=5)
    sys.stdout.write(b"".join(out).decode())
    sys.stdout.flush()
    return failed


def dry_run(args):
    """The rank plumbing of main() on gloo (CPU): every rank joins, rank 0 prints what the real run
    would report as n_gpus / parallelism (tests/test_bench_launcher.py)."""
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if os.environ.get("BENCH_DRY_FAIL_RANK") == str(rank):   # launcher test: a rank dying before the rendezvous
        sys.exit(3)
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


def _coherent_host_f32(n):
    """n float32 in coherent pinned host memory (hipHostMallocCoherent), as a torch view.  The
    allocation lives for the process (one small block per bench leg)."""
    import ctypes as C
    import torch
    rt = C.CDLL("libamdhip64.so")
    rt.hipHostMalloc.argtypes = [C.POINTER(C.c_void_p), C.c_size_t, C.c_uint]
    rt.hipHostMalloc.restype = C.c_int
    p = C.c_void_p()
    if rt.hipHostMalloc(C.byref(p), 4 * n, 0x40000000) != 0:
        raise RuntimeError("hipHostMalloc(hipHostMallocCoherent)")
    buf = (C.c_float * n).from_address(p.value)
    t = torch.frombuffer(buf, dtype=torch.float32, count=n)
    t.zero_()
    return t


def relabel_valu(e, note):
    """A matcher entry whose algorithmic bytes are mostly cache/LDS re-reads: its `frac` is the
    VALU issue fraction (never an 'HBM' fraction above 1); the algorithmic rate stays as an
    equivalent figure without a fraction, and the real HBM rate as hbm_achieved / hbm_frac."""
    alg = e.pop("achieved", None)
    e.pop("frac", None)
    e.pop("peak", None)
    e.pop("unit", None)
    e["alg_equivalent_GBps"] = alg
    e["alg_equivalent_note"] = note
    e["bound"] = "valu"
    v = e.get("valu")
    if v:
        e.update({"achieved": v["achieved"], "peak": v["peak"], "unit": v["unit"], "frac": v["frac"]})


def pose_roofline(ep, roof_fast):
    """`roofline` of the step's dominant kernel: k_pose_opt (TrackWithMotionModel's and
    TrackLocalMap's PoseOptimization, the tracking lane's critical path).  It
    is neither HBM- nor MFMA-bound: one workgroup per frame runs the serial LM chain, so the
    bound reported is VALU issue (SQ_INSTS_VALU from its PMC pass / isolated launch time) against
    the chip's issue roof and against the issue roof of the CUs the launch occupies (one per
    frame).  Its HBM traffic (PMC FETCH+WRITE) rides along.  k_fast_cells, the dominant extraction kernel, is `secondary`."""
    t = ep["avg_launch_ms"]
    out = {"kernel": "k_pose_opt", "bound": "valu", "unit": "G wave-instr/s", "peak": VALU_PEAK_GINST,
           "achieved": ep.get("achieved"), "frac": ep.get("frac"), "frac_of_occupied_cus": ep.get("frac_of_occupied_cus"),
           "insts_per_launch": ep.get("insts_per_launch"), "avg_launch_ms": t, "launches": ROOFLINE_REPS,
           "frames_per_launch": ep["frames_per_launch"], "traffic": ep.get("traffic"),
           "pmc_source": ep.get("pmc_source"), "workload": ep["workload"],
           "timing": "HIP events on the pose engine's stream around the isolated launch (Optimizer_pose_timing), "
                     f"mean of {ROOFLINE_REPS}; tools/roofline_check.py compares the rocprofv3 trace",
           "secondary": roof_fast}
    if ep.get("traffic"):
        gbs = ep["traffic"] / (t * 1e-3) / 1e9
        out["hbm"] = {"traffic_per_launch": ep["traffic"], "achieved": round(gbs, 2), "peak": HBM_PEAK_GBS,
                      "unit": "GB/s", "frac": round(gbs / HBM_PEAK_GBS, 5)}
    return out


def main():
    global NFEAT
    args = parse()
    NFEAT = args.nfeatures
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
    d_LR = torch.from_numpy(np.concatenate([lefts, rights])).to(dev)   # [lefts | rights], one allocation
    d_L, d_R = d_LR[:B], d_LR[B:]
    d_obs = torch.ones(cap, dtype=torch.int32, device=dev)
    d_outlier = torch.zeros(cap, dtype=torch.uint8, device=dev)
    eye = torch.eye(4, dtype=torch.float32, device=dev)
    poses = torch.from_numpy(np.stack([synthetic.pose_from_rotation(R) for R in Rs])).to(dev)
    gW = np.float32(np.float32(64) / np.float32(W))
    gH = np.float32(np.float32(48) / np.float32(H))
    P = B - 1
    arr = lambda xs: (C.c_void_p * len(xs))(*xs)
    from c_orb_slam_amd._lib import orb_unproject, pose_frame, orb_localmap, orb_newpoints, orb_localprep
    lsf = np.float32(np.log(np.float32(1.2)))   # Frame::mfLogScaleFactor
    from concurrent.futures import ThreadPoolExecutor
    # HIP's current device is per thread: every worker binds it first
    pool = ThreadPoolExecutor(2, initializer=lambda: torch.cuda.set_device(dev))
    match_stream = torch.cuda.ExternalStream(L.ORBmatcher_stream(m._h), device=dev)

    def n_field(arr, cls, count):
        """int32 view of field 0 (the count N) of every struct of a ctypes struct array."""
        w = C.sizeof(cls) // 4
        return np.ctypeslib.as_array((C.c_int32 * (count * w)).from_address(C.addressof(arr))).reshape(count, w)[:, 0]

    # absolute poses in the batch's world (frame 0's camera): frame b+1 is frame b rotated by Rs[b]
    Tabs = [np.eye(4, dtype=np.float32)]
    for R in Rs:
        Tabs.append(synthetic.pose_from_rotation(np.asarray(R, np.float64) @ Tabs[-1][:3, :3].astype(np.float64)))
    d_Tcw = torch.from_numpy(np.stack([T.reshape(16) for T in Tabs])).to(dev)                 # mTcw (motion model)
    d_Twc = torch.from_numpy(np.stack([np.linalg.inv(T).astype(np.float32).reshape(16) for T in Tabs])).to(dev)
    d_obs = torch.ones(B * cap, dtype=torch.int32, device=dev)

    class Lane:
        """One batch in flight: its own extractor pair (pyramids, keypoints) and tracking buffers.
        Map: every frame b's stereo keypoints become map points (UnprojectStereo with its absolute
        Twc), block b of a (B x cap) table; the local map of pair p (current frame p+1) is the blocks
        of frames max(0, p-K+1)..p, contiguous in the table (UpdateLocalMap's local keyframes)."""

        def __init__(self, mt):
            # the lane's matcher: the shared one, or (--lane-matchers) its own for every lane but the
            # first, whose chains then run beside the other lanes' on their own streams
            self.m = mt
            self.ms = match_stream if mt is m else torch.cuda.ExternalStream(L.ORBmatcher_stream(mt._h), device=dev)
            if args.stereo_batch:   # one extractor, one stream: [lefts | rights] as one batch of 2B images
                self.exL = orb.ORBextractor(NFEAT, 1.2, 8, 20, 7, max_width=W, max_height=H, max_batch=2 * B)
                self.exR = self.exL
                self.d_kps_all = torch.empty((2 * B, cap, 7), dtype=torch.int32, device=dev)
                self.d_desc_all = torch.empty((2 * B, cap, 32), dtype=torch.uint8, device=dev)
                self.d_kps, self.d_kpsR = self.d_kps_all[:B], self.d_kps_all[B:]
                self.d_desc, self.d_descR = self.d_desc_all[:B], self.d_desc_all[B:]
            else:
                self.exL = orb.ORBextractor(NFEAT, 1.2, 8, 20, 7, max_width=W, max_height=H, max_batch=B)
                self.exR = orb.ORBextractor(NFEAT, 1.2, 8, 20, 7, max_width=W, max_height=H, max_batch=B)
                self.d_kps = torch.empty((B, cap, 7), dtype=torch.int32, device=dev)   # mvKeys (== mvKeysUn, KITTI k1=0)
                self.d_desc = torch.empty((B, cap, 32), dtype=torch.uint8, device=dev)
                self.d_kpsR = torch.empty((B, cap, 7), dtype=torch.int32, device=dev)
                self.d_descR = torch.empty((B, cap, 32), dtype=torch.uint8, device=dev)
            self.d_uR = torch.empty((B, cap), dtype=torch.float32, device=dev)      # mvuRight
            self.d_depth = torch.empty((B, cap), dtype=torch.float32, device=dev)   # mvDepth
            self.d_mp_pos = torch.zeros((B, cap, 3), dtype=torch.float32, device=dev)
            self.d_slot = torch.empty((B, cap), dtype=torch.int32, device=dev)      # UnprojectStereo slots
            self.d_cur_mp = torch.empty((B, cap), dtype=torch.int32, device=dev)
            self.d_maxd = torch.zeros((B, cap), dtype=torch.float32, device=dev)    # MapPoint::mfMaxDistance
            self.d_mind = torch.zeros((B, cap), dtype=torch.float32, device=dev)
            self.d_nrm = torch.zeros((B, cap, 3), dtype=torch.float32, device=dev)
            self.d_skip = torch.ones((P, K_LOCAL * cap), dtype=torch.uint8, device=dev)
            self.scale = torch.from_numpy(self.exL.GetScaleFactors()).to(dev)
            self.d_Tout = torch.empty((P, 16), dtype=torch.float32, device=dev)
            self.d_Tout2 = torch.empty((P, 16), dtype=torch.float32, device=dev)
            self.d_poutl = torch.zeros((P, cap), dtype=torch.uint8, device=dev)
            self.d_poutl2 = torch.zeros((P, cap), dtype=torch.uint8, device=dev)
            self.isig_tab = torch.from_numpy(self.exL.GetInverseScaleSigmaSquares()).to(dev)
            self.bs = [max(0, p - K_LOCAL + 1) for p in range(P)]                   # first local block of pair p
            # the poses the chain reads: the generator's (batch mode) or, with --sequence, the lane's
            # own arrays rewritten at the start of every chain from the previous steps' estimates
            if args.sequence:
                self.sPred = d_Tcw.clone()   # [b]: motion-model prediction for current frame b
                self.sLast = d_Tcw.clone()   # [b]: LastFrame.mTcw of frame b
                self.sTwc = d_Twc.clone()    # [b]: its inverse (UnprojectStereo of frame b)
                Tpred_, Tlast_, Twc_ = self.sPred, self.sLast, self.sTwc
            else:
                Tpred_, Tlast_, Twc_ = d_Tcw, d_Tcw, d_Twc
            # ctypes views of the batch, built once (device pointers do not move; only counts change)
            self.curs = (orb_frame * P)(*[self.frame_struct(b, Tpred_[b].data_ptr()) for b in range(1, B)])
            # TrackLocalMap sees mCurrentFrame.mTcw as set by the first PoseOptimization
            self.curs_local = (orb_frame * P)(*[self.frame_struct(b, self.d_Tout[b - 1].data_ptr())
                                                for b in range(1, B)])

            self.lasts = (orb_frame * P)(*[self.frame_struct(b, Tlast_[b].data_ptr()) for b in range(0, B - 1)])
            self.mps = (orb_mappoints * P)()
            self.lmaps = (orb_localmap * P)()
            for p in range(P):
                q = self.bs[p]
                self.mps[p].n = (p - q + 1) * cap
                self.mps[p].pos = self.d_mp_pos[q].data_ptr()
                self.mps[p].desc = self.d_desc[q].data_ptr()
                self.mps[p].observations = d_obs.data_ptr()
                self.lmaps[p] = orb_localmap((p - q + 1) * cap, self.d_mp_pos[q].data_ptr(), self.d_desc[q].data_ptr(),
                                             d_obs.data_ptr(), self.d_maxd[q].data_ptr(), self.d_mind[q].data_ptr(),
                                             self.d_nrm[q].data_ptr(), self.d_skip[p].data_ptr())
            self.a_cur_mp = arr([self.d_cur_mp[b].data_ptr() for b in range(1, B)])
            self.a_last_kps = arr([self.d_kps[b].data_ptr() for b in range(P)])
            self.a_last_mp = arr([self.d_slot[b].data_ptr() for b in range(P)])   # LastFrame.mvpMapPoints
            self.a_last_out = arr([d_outlier.data_ptr()] * P)
            self.s_kL = arr([self.d_kps[b].data_ptr() for b in range(B)])
            self.s_dL = arr([self.d_desc[b].data_ptr() for b in range(B)])
            self.s_kR = arr([self.d_kpsR[b].data_ptr() for b in range(B)])
            self.s_dR = arr([self.d_descR[b].data_ptr() for b in range(B)])
            self.s_uR = arr([self.d_uR[b].data_ptr() for b in range(B)])
            self.s_dep = arr([self.d_depth[b].data_ptr() for b in range(B)])
            # UpdateLastFrame / CreateNewKeyFrame: new MapPoints from frame b's stereo keypoints
            # (UnprojectStereo with its absolute Twc + UpdateNormalAndDepth) -> block b of the
            # table; row ids relative to the local map of pair b, whose last frame b is
            self.newp = (orb_newpoints * B)(*[
                orb_newpoints(0, self.d_kps[b].data_ptr(), self.d_depth[b].data_ptr(), Twc_[b].data_ptr(),
                              float(fx), float(fy), float(cx), float(cy), self.scale.data_ptr(), 8,
                              (b - max(0, b - K_LOCAL + 1)) * cap, self.d_mp_pos[b].data_ptr(),
                              self.d_slot[b].data_ptr(), self.d_nrm[b].data_ptr(), self.d_maxd[b].data_ptr(),
                              self.d_mind[b].data_ptr()) for b in range(B)])
            self.prep = (orb_localprep * P)(*[
                orb_localprep(0, self.d_cur_mp[p + 1].data_ptr(), self.d_poutl[p].data_ptr(),
                              (p - self.bs[p] + 1) * cap, self.d_slot[self.bs[p]].data_ptr(),
                              self.d_skip[p].data_ptr()) for p in range(P)])
            # PoseOptimization(&mCurrentFrame): the frame's own arrays, map points by local-map index;
            # TrackWithMotionModel's call from the motion-model pose, TrackLocalMap's from its result
            self.pframes = (pose_frame * P)(*[
                pose_frame(0, Tpred_[p + 1].data_ptr(), self.d_cur_mp[p + 1].data_ptr(),
                           self.d_mp_pos[self.bs[p]].data_ptr(), self.d_kps[p + 1].data_ptr(),
                           self.d_uR[p + 1].data_ptr(), self.isig_tab.data_ptr(), 8, float(fx), float(fy), float(cx),
                           float(cy), float(mbf)) for p in range(P)])
            self.pframes2 = (pose_frame * P)(*[
                pose_frame(0, self.d_Tout[p].data_ptr(), self.d_cur_mp[p + 1].data_ptr(),
                           self.d_mp_pos[self.bs[p]].data_ptr(), self.d_kps[p + 1].data_ptr(),
                           self.d_uR[p + 1].data_ptr(), self.isig_tab.data_ptr(), 8, float(fx), float(fy), float(cx),
                           float(cy), float(mbf)) for p in range(P)])
            self.a_Tout = arr([self.d_Tout[p].data_ptr() for p in range(P)])
            self.a_poutl = arr([self.d_poutl[p].data_ptr() for p in range(P)])
            self.a_Tout2 = arr([self.d_Tout2[p].data_ptr() for p in range(P)])
            self.a_poutl2 = arr([self.d_poutl2[p].data_ptr() for p in range(P)])
            self.n_unp = n_field(self.newp, orb_newpoints, B)
            self.n_prep = n_field(self.prep, orb_localprep, P)
            self.n_cur = n_field(self.curs, orb_frame, P)
            self.n_last = n_field(self.lasts, orb_frame, P)
            self.n_pose = n_field(self.pframes, pose_frame, P)
            self.n_pose2 = n_field(self.pframes2, pose_frame, P)
            self.n_curl = n_field(self.curs_local, orb_frame, P)
            self.ninl = np.zeros(P, np.int32)
            self.ninl2 = np.zeros(P, np.int32)
            self.nm = np.zeros(P, np.int32)
            self.nml = np.zeros(P, np.int32)
            self.nvis = np.zeros(P, np.int32)
            self.nst = np.zeros(B, np.int32)
            self.epoch = 0        # the deferred-chain epoch of this lane's last tracking chain
            self.kp_count = 0
            self.nL = self.nR = None
            self.kidx = torch.arange(cap, dtype=torch.int32, device=dev)
            self.img_ptr = d_LR.data_ptr()   # the batch's 2B images in HBM ([lefts | rights])
            self.img_ev = None               # host-IO pass: the upload event the extraction waits on

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
            # two HIP streams, like the reference's two extractor threads per stereo frame.  The
            # lane's buffers may still be read by the tracking chain of its previous batch: wait
            # for that chain's device work first (not for its counts)
            if self.epoch:
                check(L.ORBmatcher_chain_wait(self.m._h, self.epoch), "ORBmatcher_chain_wait")
            if self.img_ev is not None:   # host-IO pass: the batch's upload must have landed
                torch.cuda.ExternalStream(self.exL.stream, device=dev).wait_event(self.img_ev)
            if args.stereo_batch:
                n = np.ascontiguousarray(self.exL.extract_device(self.img_ptr, 2 * B, W, H, W, W * H,
                                                                 self.d_kps_all.data_ptr(), self.d_desc_all.data_ptr(),
                                                                 cap), np.int32)
                self.nL, self.nR = np.ascontiguousarray(n[:B]), np.ascontiguousarray(n[B:])
                self.tl = self.exL.last_timings()
                self.tr = {k: 0.0 for k in self.tl}
                return
            fR = pool.submit(self.exR.extract_device, self.img_ptr + B * W * H, B, W, H, W, W * H,
                             self.d_kpsR.data_ptr(), self.d_descR.data_ptr(), cap)
            self.nL = np.ascontiguousarray(self.exL.extract_device(self.img_ptr, B, W, H, W, W * H,
                                                                   self.d_kps.data_ptr(), self.d_desc.data_ptr(), cap),
                                           np.int32)
            self.nR = np.ascontiguousarray(fR.result(), np.int32)
            # per-stage event times now: the extractors are shared by the lanes, and the next
            # lane's extraction re-records their events before this lane's chain is collected
            self.tl, self.tr = self.exL.last_timings(), self.exR.last_timings()

        def stereo(self):
            nL, nR = self.nL, self.nR
            check(L.ORBmatcher_ComputeStereoMatches_batch_at(self.m._h, self.exL._h, 0, self.exR._h,
                                                             B if args.stereo_batch else 0, B, ptr(nL), self.s_kL,
                                                             self.s_dL, ptr(nR), self.s_kR, self.s_dR, float(mbf),
                                                             float(mb), self.s_uR, self.s_dep, ptr(self.nst)),
                  "ComputeStereoMatches batch")

        def search(self):
            # UpdateLastFrame (Frame::UnprojectStereo) of every frame of the batch, the map points'
            # normal and scale-invariance distances (MapPoint::UpdateNormalAndDepth, MapPoint.cc:
            # 331-371: one observation, the creating frame), LastFrame.mvpMapPoints as local-map
            # rows and the current frames' empty mvpMapPoints, on the matcher's stream
            nL = self.nL
            self.n_unp[:] = nL
            self.n_cur[:] = nL[1:]
            self.n_last[:] = nL[:-1]
            self.n_pose[:] = nL[1:]
            self.n_pose2[:] = nL[1:]
            with torch.cuda.stream(self.ms):
                self.d_slot.fill_(-1)
                self.d_cur_mp.fill_(-1)
            check(L.MapPoint_CreateStereo_batch_device(self.m._h, B, self.newp), "MapPoint_CreateStereo batch")
            # TrackWithMotionModel: SearchByProjection(CurrentFrame, LastFrame, th=7, stereo) (Tracking.cc:869-885)
            check(L.ORBmatcher_SearchByProjection_LastFrame_batch(self.m._h, P, self.curs, self.a_cur_mp, self.lasts,
                                                                  self.a_last_kps, self.a_last_mp, self.a_last_out,
                                                                  self.mps, 7.0, 0, ptr(self.nm)),
                  "SearchByProjection batch")

        def local_map(self):
            """TrackLocalMap (Tracking.cc:930-974) after TrackWithMotionModel's PoseOptimization:
            discard its outliers (Tracking.cc:893-913), skip the points already in the frame
            (SearchLocalPoints 1146-1161) and the table rows without a map point, isInFrustum +
            SearchByProjection(F, mvpLocalMapPoints, th=1) (stereo, ORBmatcher(0.8)), then the
            second PoseOptimization."""
            self.n_prep[:] = self.nL[1:]
            check(L.Tracking_PrepareLocalSearch_batch_device(self.m._h, P, self.prep), "PrepareLocalSearch batch")
            self.n_curl[:] = self.nL[1:]
            check(L.ORBmatcher_SearchLocalPoints_batch(self.m._h, P, self.curs_local, self.a_cur_mp, self.lmaps,
                                                       float(lsf), 1.0, 0.8, ptr(self.nml), ptr(self.nvis)),
                  "SearchLocalPoints batch")
            check(L.Optimizer_PoseOptimization_frames_device_deferred(self.m._h, P, self.pframes2, self.a_Tout2,
                                                                      self.a_poutl2, ptr(self.ninl2)),
                  "PoseOptimization (local map)")

        def enqueue(self):
            """ComputeStereoMatches, UpdateLastFrame, SearchByProjection(Cur, Last, 7), PoseOptimization,
            TrackLocalMap (SearchLocalPoints, PoseOptimization): one deferred chain on the matcher's
            stream (ORBmatcher_set_deferred), every call queued behind the previous one -- and the
            whole chain behind the previous batch's -- without a host round trip; the chain is
            closed into an epoch whose counts collect() writes."""
            t1 = time.perf_counter()
            nL, nR = self.nL, self.nR
            self.kp_count = int(nL.sum() + nR.sum())
            check(L.ORBmatcher_set_deferred(self.m._h, 1), "ORBmatcher_set_deferred")
            if args.sequence:
                seq_predict(self)
            self.stereo()
            t2 = time.perf_counter()
            self.search()
            t3 = time.perf_counter()
            # Optimizer::PoseOptimization(&mCurrentFrame) (Tracking.cc:887) on the matched map points
            check(L.Optimizer_PoseOptimization_frames_device_deferred(self.m._h, P, self.pframes, self.a_Tout,
                                                                      self.a_poutl, ptr(self.ninl)),
                  "PoseOptimization batch")
            t4 = time.perf_counter()
            self.local_map()
            if args.sequence:
                seq_record(self)
            t5 = time.perf_counter()
            eid = C.c_longlong(0)
            check(L.ORBmatcher_chain_close(self.m._h, C.byref(eid)), "ORBmatcher_chain_close")
            self.epoch = eid.value
            for k, v in (("stereo", t2 - t1), ("lift+search", t3 - t2), ("pose", t4 - t3), ("local_map", t5 - t4)):
                phase_acc[k] = phase_acc.get(k, 0.0) + v * 1e3

        def collect(self):
            """Finish this lane's chain (counts land) and book its statistics."""
            t5 = time.perf_counter()
            check(L.ORBmatcher_chain_finish(self.m._h, self.epoch), "ORBmatcher_chain_finish")
            phase_acc["finish"] = phase_acc.get("finish", 0.0) + (time.perf_counter() - t5) * 1e3
            tl, tr = self.tl, self.tr
            for k in tl:
                stage_acc[k] = stage_acc.get(k, 0.0) + tl[k] + tr[k]
                stage_lr["left"][k] = stage_lr["left"].get(k, 0.0) + tl[k]
                stage_lr["right"][k] = stage_lr["right"].get(k, 0.0) + tr[k]
            kernel_ms.append(tl["fast_cells"])
            kernel_ms.append(tr["fast_cells"])
            pose_inl.append(int(self.ninl2.sum()))
            local_acc.append((int(self.nml.sum()), int(self.nvis.sum())))
            return self.kp_count, int(self.nm.sum() + self.nml.sum()), int(self.nst.sum())

    def rigid_inv(T):
        """Twc from Tcw as the reference forms it (Frame::UpdatePoseMatrices: R^T, -R^T t)."""
        Ti = np.eye(4, dtype=np.float32)
        R = T[:3, :3]
        Ti[:3, :3] = R.T
        Ti[:3, 3] = -(R.T @ T[:3, 3])
        return Ti

    def latency_leg(nf, host_io=False, mm=None, barrier=None):
        """Per-frame tracking latency, the reference's own figure (wall time of one TrackStereo,
        stereo_kitti.cc:80-97): batch 1, frames in sequence, each frame's motion model from the
        previous frames' optimised poses (Tracking.cc:869, mVelocity), the local map from the last
        K_LOCAL frames' map points; every call synchronous as Tracking makes them.
        host_io: the drop-in path System::TrackStereo(const cv::Mat&, const cv::Mat&) times
        (System.cc:116): both images start in pageable host memory (the H2D copies are inside the
        extractor calls) and the frame's results end on the host -- mvKeys / mDescriptors of both
        images, mvuRight, mvDepth, mTcw, mvpMapPoints (local-map rows) and mvbOutlier -- before the
        clock stops.  Otherwise the images are HBM-resident and the results stay on the device."""
        nf = min(nf, B)
        # mm: this leg's own ORBmatcher (sequence_leg runs several legs on their own threads);
        # barrier: a threading.Barrier the legs pass together right before their timed frames
        own_gc = mm is None
        if mm is None:
            mm = m
        mstream = match_stream if mm is m else torch.cuda.ExternalStream(L.ORBmatcher_stream(mm._h), device=dev)
        if host_io:
            hk = torch.empty((cap, 7), dtype=torch.int32).pin_memory()
            hd = torch.empty((cap, 32), dtype=torch.uint8).pin_memory()
            hkR = torch.empty((cap, 7), dtype=torch.int32).pin_memory()
            hdR = torch.empty((cap, 32), dtype=torch.uint8).pin_memory()
            huR = torch.empty(cap, dtype=torch.float32).pin_memory()
            hdep = torch.empty(cap, dtype=torch.float32).pin_memory()
            hT = torch.empty(16, dtype=torch.float32).pin_memory()
            hmp = torch.empty(cap, dtype=torch.int32).pin_memory()
            hout = torch.empty(cap, dtype=torch.uint8).pin_memory()
            d2h_bytes = []
        eL1 = orb.ORBextractor(NFEAT, 1.2, 8, 20, 7, max_width=W, max_height=H, max_batch=1)
        eR1 = orb.ORBextractor(NFEAT, 1.2, 8, 20, 7, max_width=W, max_height=H, max_batch=1)
        # device path: Frame(imLeft, imRight)'s two extractions as one call over the frame's two
        # HBM-resident images (left t, right t = left t + B images), the right image's results
        # landing in the next frame's slot of k / d (overwritten by that frame's left image)
        eLR = None if host_io or not args.latency_stereo_batch else orb.ORBextractor(NFEAT, 1.2, 8, 20, 7, max_width=W, max_height=H, max_batch=2)
        # host path: Frame(imLeft, imRight)'s two host images in one extractor call (one staging block,
        # one H2D copy, one stream); BENCH_LAT_HOST_THREADS=1 keeps the reference's shape of two
        # extractor calls on two threads (A/B: concurrent blocking waits on two streams there show
        # sporadic ~7 ms wake-ups, profiles/r05vlat_slowest_frames.txt)
        host_pair = host_io and os.environ.get("BENCH_LAT_HOST_THREADS") != "1"
        eLRh = orb.ORBextractor(NFEAT, 1.2, 8, 20, 7, max_width=W, max_height=H, max_batch=2) if host_pair else None
        k = torch.empty((nf + 1, cap, 7), dtype=torch.int32, device=dev)
        d = torch.empty((nf + 1, cap, 32), dtype=torch.uint8, device=dev)
        kR = torch.empty((cap, 7), dtype=torch.int32, device=dev)
        dR = torch.empty((cap, 32), dtype=torch.uint8, device=dev)
        uR = torch.empty((nf, cap), dtype=torch.float32, device=dev)
        dep = torch.empty((nf, cap), dtype=torch.float32, device=dev)
        pos = torch.zeros((nf, cap, 3), dtype=torch.float32, device=dev)
        slot = torch.full((nf, cap), -1, dtype=torch.int32, device=dev)
        maxd = torch.zeros((nf, cap), dtype=torch.float32, device=dev)
        mind = torch.zeros((nf, cap), dtype=torch.float32, device=dev)
        nrm = torch.zeros((nf, cap, 3), dtype=torch.float32, device=dev)
        skip = torch.ones(K_LOCAL * cap, dtype=torch.uint8, device=dev)
        # the frame's three 4x4 poses (motion-model prediction, last Tcw, last Twc) travel in ONE
        # pinned H2D copy, as a C++ caller would pass them, not three pageable copies
        # ... and the current frame's map-point slots (mvpMapPoints, all NULL = -1 at the start of
        # the frame) ride in the same copy: one H2D per frame sets the poses and clears the slots
        Tbuf = torch.zeros(48 + cap, dtype=torch.int32, device=dev)
        Thbuf = torch.zeros(48 + cap, dtype=torch.int32).pin_memory()
        Thbuf[48:] = -1
        Tdev, Thost, cur_mp = Tbuf[:48].view(torch.float32), Thbuf[:48].view(torch.float32), Tbuf[48:]
        # the copy as a C++ caller issues it: hipMemcpyAsync on the matcher's stream (no framework
        # dispatch per frame); the framework copy if the runtime library cannot be bound
        try:
            hip_rt = C.CDLL("libamdhip64.so")
            hip_rt.hipMemcpyAsync.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int, C.c_void_p]
            hip_rt.hipMemcpyAsync.restype = C.c_int
        except OSError:
            hip_rt = None
        tb_args = (C.c_void_p(Tbuf.data_ptr()), C.c_void_p(Thbuf.data_ptr()), C.c_size_t(4 * (48 + cap)), 1,
                   C.c_void_p(mstream.cuda_stream))
        Tpred, Tlast, Twc_l = Tdev[0:16], Tdev[16:32], Tdev[32:48]
        T1, T2 = (torch.zeros(16, dtype=torch.float32, device=dev) for _ in range(2))
        o1, o2 = (torch.zeros(cap, dtype=torch.uint8, device=dev) for _ in range(2))
        isig = lanes[0].isig_tab
        scale = lanes[0].scale
        one = np.zeros(1, np.int32)
        Tcw = [np.eye(4, dtype=np.float32)]
        walls = []
        nmatch = []
        marks = []   # per frame: (phase, ms since the frame's start) -- where a slow frame spent its time
        # Every call's argument block built before the timed frames, as a C++ caller holds its
        # Frame / MapPoint arrays at fixed addresses: per frame only the counts the previous calls
        # returned are written into them (the interpreter's marshalling is not the library's cost).
        kp = [k[t].data_ptr() for t in range(nf + 1)]
        dp = [d[t].data_ptr() for t in range(nf + 1)]
        dL_ptr = [d_L[t].data_ptr() for t in range(nf)]
        # the final pose lands in coherent pinned memory (hipHostMallocCoherent: the GPU's stores go
        # straight to host memory; the kernel also fences them at system scope)
        hT2 = _coherent_host_f32(16)
        pre = [None] * nf
        for t in range(nf):
            q = max(0, t - K_LOCAL)
            nloc = (t - q) * cap
            g = {"stereo_lr": (arr([kp[t]]), arr([dp[t]]), arr([kp[t + 1]]), arr([dp[t + 1]]),
                               arr([uR[t].data_ptr()]), arr([dep[t].data_ptr()])),
                 "stereo_r": (arr([kR.data_ptr()]), arr([dR.data_ptr()])), "nloc": nloc}
            if t > 0:
                g["u"] = orb_newpoints(0, kp[t - 1], dep[t - 1].data_ptr(), Twc_l.data_ptr(), float(fx), float(fy),
                                       float(cx), float(cy), scale.data_ptr(), 8, (t - 1 - q) * cap,
                                       pos[t - 1].data_ptr(), slot[t - 1].data_ptr(), nrm[t - 1].data_ptr(),
                                       maxd[t - 1].data_ptr(), mind[t - 1].data_ptr())
                fc = lanes[0].frame_struct(0, Tpred.data_ptr())
                fc.keysUn, fc.desc, fc.uRight = kp[t], dp[t], uR[t].data_ptr()
                fl = lanes[0].frame_struct(0, Tlast.data_ptr())
                fl.keysUn, fl.desc, fl.uRight = kp[t - 1], dp[t - 1], uR[t - 1].data_ptr()
                g["fc"], g["fl"] = fc, fl
                g["mp"] = orb_mappoints(nloc, pos[q].data_ptr(), dp[q], d_obs.data_ptr())
                g["last"] = (arr([cur_mp.data_ptr()]), arr([kp[t - 1]]), arr([slot[t - 1].data_ptr()]),
                             arr([d_outlier.data_ptr()]))
                g["pf"] = pose_frame(0, Tpred.data_ptr(), cur_mp.data_ptr(), pos[q].data_ptr(), kp[t],
                                     uR[t].data_ptr(), isig.data_ptr(), 8, float(fx), float(fy), float(cx), float(cy),
                                     float(mbf))
                g["pose1"] = (arr([T1.data_ptr()]), arr([o1.data_ptr()]))
                # device path: the frame's final pose written by the pose kernel straight into pinned
                # host memory (device-visible), where Tracking keeps mTcw; the host path copies
                # it back with the Frame's other members
                g["pose2"] = (arr([T2.data_ptr() if host_io else hT2.data_ptr()]), arr([o2.data_ptr()]))
                g["prep"] = orb_localprep(0, cur_mp.data_ptr(), o1.data_ptr(), nloc, slot[q].data_ptr(), skip.data_ptr())
                g["lmap"] = orb_localmap(nloc, pos[q].data_ptr(), dp[q], d_obs.data_ptr(), maxd[q].data_ptr(),
                                         mind[q].data_ptr(), nrm[q].data_ptr(), skip.data_ptr())
                g["cur"] = arr([cur_mp.data_ptr()])
            pre[t] = g
        T1p, Tpp = T1.data_ptr(), Tpred.data_ptr()
        nl, nr = np.zeros(1, np.int32), np.zeros(1, np.int32)
        nm1, ni, nm2, nv2 = (np.zeros(1, np.int32) for _ in range(4))
        # the drop-in caller is C++ (System::TrackStereo): no interpreter garbage collection runs
        # between its frames, so none runs inside this leg's timed frames either
        import gc
        gc_was = gc.isenabled() and own_gc
        if own_gc:
            gc.collect()
            gc.disable()
        if barrier is not None:
            barrier.wait()
        t_begin = time.perf_counter()
        try:  # a failing check() must not leave the collector off for the rest of the bench
            for t in range(nf):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                mk = []
                marks.append(mk)

                def mark(name):
                    mk.append((name, (time.perf_counter() - t0) * 1e3))

                if host_pair:   # Frame(imLeft, imRight) on pageable host images (Frame.cc:78-81), one call
                    nLR = eLRh.extract_host_images_to_device([lefts[t], rights[t]], k[t].data_ptr(), d[t].data_ptr(), cap)
                    mark("extract_both")
                    nL, nR = nLR[:1], nLR[1:]
                    nl[0], nr[0] = nLR[0], nLR[1]
                    a0, a1, a2, a3, a4, a5 = pre[t]["stereo_lr"]
                    check(L.ORBmatcher_ComputeStereoMatches_batch_at(mm._h, eLRh._h, 0, eLRh._h, 1, 1, ptr(nl), a0, a1,
                                                                     ptr(nr), a2, a3, float(mbf), float(mb), a4, a5,
                                                                     ptr(one)), "ComputeStereoMatches")
                elif host_io:   # the same as two extractor calls on two threads
                    def right_host(img):
                        r = eR1.extract_host_to_device(img, kR.data_ptr(), dR.data_ptr(), cap)
                        mark("extract_right")
                        return r

                    fR = pool.submit(right_host, rights[t])
                    nL = eL1.extract_host_to_device(lefts[t], k[t].data_ptr(), d[t].data_ptr(), cap)
                    mark("extract_left")
                elif eLR is None:
                    fR = pool.submit(eR1.extract_device, d_R[t].data_ptr(), 1, W, H, W, W * H, kR.data_ptr(), dR.data_ptr(),
                                     cap)
                    nL = eL1.extract_device(d_L[t].data_ptr(), 1, W, H, W, W * H, k[t].data_ptr(), d[t].data_ptr(), cap)
                if host_pair:
                    pass
                elif host_io or eLR is None:
                    nR = fR.result()
                    mark("extract_both")
                    nl, nr = np.array([nL[0]], np.int32), np.array([nR[0]], np.int32)
                    check(L.ORBmatcher_ComputeStereoMatches_batch(mm._h, eL1._h, eR1._h, 1, ptr(nl), arr([k[t].data_ptr()]),
                                                                  arr([d[t].data_ptr()]), ptr(nr), arr([kR.data_ptr()]),
                                                                  arr([dR.data_ptr()]), float(mbf), float(mb),
                                                                  arr([uR[t].data_ptr()]), arr([dep[t].data_ptr()]),
                                                                  ptr(one)), "ComputeStereoMatches")
                else:
                    nLR = eLR.extract_device(dL_ptr[t], 2, W, H, W, B * W * H, kp[t], dp[t], cap)
                    nL = nLR[:1]
                    nl[0], nr[0] = nLR[0], nLR[1]
                    a0, a1, a2, a3, a4, a5 = pre[t]["stereo_lr"]
                    check(L.ORBmatcher_ComputeStereoMatches_batch_at(mm._h, eLR._h, 0, eLR._h, 1, 1, ptr(nl), a0, a1,
                                                                     ptr(nr), a2, a3, float(mbf), float(mb), a4, a5,
                                                                     ptr(one)), "ComputeStereoMatches")
                mark("stereo")
                if t > 0:
                    V = Tcw[t - 1] @ rigid_inv(Tcw[t - 2]) if t >= 2 else np.eye(4, dtype=np.float32)
                    Tp = (V @ Tcw[t - 1]).astype(np.float32)
                    nlast = int(last_n[0])
                    g = pre[t]
                    hv = Thost.numpy()
                    hv[0:16] = Tp.reshape(16)
                    hv[16:32] = Tcw[t - 1].reshape(16)
                    hv[32:48] = rigid_inv(Tcw[t - 1]).reshape(16)
                    if hip_rt is not None:   # ordered before the matcher's launches (its stream)
                        if hip_rt.hipMemcpyAsync(*tb_args) != 0:
                            raise RuntimeError("hipMemcpyAsync")
                    else:
                        with torch.cuda.stream(mstream):
                            Tbuf.copy_(Thbuf, non_blocking=True)
                    u = g["u"]
                    u.N = nlast
                    check(L.MapPoint_CreateStereo_batch_device(mm._h, 1, C.byref(u)), "MapPoint_CreateStereo")
                    fc, fl, mp, pf = g["fc"], g["fl"], g["mp"], g["pf"]
                    fc.N, fl.N, pf.N = int(nL[0]), nlast, int(nL[0])
                    fc.Tcw, pf.Tcw = Tpp, Tpp
                    a0, a1, a2, a3 = g["last"]
                    check(L.ORBmatcher_SearchByProjection_LastFrame_batch(mm._h, 1, C.byref(fc), a0, C.byref(fl), a1, a2, a3,
                                                                          C.byref(mp), 7.0, 0, ptr(nm1)),
                          "SearchByProjection(Last)")
                    b0, b1 = g["pose1"]
                    check(L.Optimizer_PoseOptimization_frames_device(1, C.byref(pf), b0, b1, ptr(ni)), "PoseOptimization")
                    mark("motion_model")
                    prep = g["prep"]
                    prep.N = int(nL[0])
                    check(L.Tracking_PrepareLocalSearch_batch_device(mm._h, 1, C.byref(prep)), "PrepareLocalSearch")
                    fc.Tcw = T1p
                    check(L.ORBmatcher_SearchLocalPoints_batch(mm._h, 1, C.byref(fc), g["cur"], C.byref(g["lmap"]), float(lsf),
                                                               1.0, 0.8, ptr(nm2), ptr(nv2)), "SearchLocalPoints")
                    mark("local_search")
                    pf.Tcw = T1p
                    b0, b1 = g["pose2"]
                    check(L.Optimizer_PoseOptimization_frames_device(1, C.byref(pf), b0, b1, ptr(ni)), "PoseOptimization 2")
                    mark("local_pose")
                    if host_io:   # the Frame's members back on the host (one stream sync)
                        n0, n1 = int(nL[0]), int(nR[0])
                        with torch.cuda.stream(mstream):
                            hk[:n0].copy_(k[t, :n0], non_blocking=True)
                            hd[:n0].copy_(d[t, :n0], non_blocking=True)
                            hkR[:n1].copy_((k[t + 1] if host_pair else kR)[:n1], non_blocking=True)
                            hdR[:n1].copy_((d[t + 1] if host_pair else dR)[:n1], non_blocking=True)
                            huR[:n0].copy_(uR[t, :n0], non_blocking=True)
                            hdep[:n0].copy_(dep[t, :n0], non_blocking=True)
                            hT.copy_(T2, non_blocking=True)
                            hmp[:n0].copy_(cur_mp[:n0], non_blocking=True)
                            hout[:n0].copy_(o2[:n0], non_blocking=True)
                        mstream.synchronize()
                        d2h_bytes.append(n0 * (28 + 32 + 4 + 4 + 4 + 1) + n1 * 60 + 64)
                        Tcw.append(hT.numpy().reshape(4, 4).copy())
                    else:
                        Tcw.append(hT2.numpy().reshape(4, 4).copy())
                    nmatch.append(int(nm1[0] + nm2[0]))
                last_n = nL
                mark("end")
                walls.append((time.perf_counter() - t0) * 1e3)
        finally:
            if gc_was:
                gc.enable()
        t_end = time.perf_counter()
        w = np.array(walls[2:])   # the first two frames have no motion model / local map yet
        err = [float(np.abs(Tcw[t][:3, :3] - Tabs[t][:3, :3]).max()) for t in range(1, len(Tcw))]
        out = {"metric": "tracking latency per stereo frame (batch 1, sequential)", "mean_ms": round(float(w.mean()), 3),
               "_span_s": (t_begin, t_end),
               "p50_ms": round(float(np.percentile(w, 50)), 3), "p90_ms": round(float(np.percentile(w, 90)), 3),
               "frames": int(len(w)), "matches_per_frame": round(float(np.mean(nmatch)), 1),
               "frame_ms": [round(float(v), 3) for v in walls],
               "max_rotation_error": round(max(err), 6),
               "note": "Frame(imLeft, imRight) + TrackWithMotionModel + TrackLocalMap per frame, synchronous C-ABI "
                       "calls; pose t from pose t-1 and t-2 (constant-velocity model). Every call's argument "
                       "structs are built before the timed frames and Python's gc is off inside them (a C++ "
                       "caller has neither cost), so these figures exclude the interpreter's per-frame "
                       "marshalling that round-4 and earlier figures included"}
        # the slowest timed frame's phase marks beside the median frame's (ms since the frame's start)
        tw = int(np.argmax(walls[2:])) + 2
        med = {}
        for mk in marks[2:]:
            for name, v in mk:
                med.setdefault(name, []).append(v)
        out["slowest_frame"] = {"frame": tw, "marks_ms": {nm: round(v, 3) for nm, v in marks[tw]},
                                "median_marks_ms": {nm: round(float(np.median(v)), 3) for nm, v in med.items()}}
        if host_io:
            out["io"] = ("host: both 1241x376 images read from pageable host memory inside the extractor call "
                         + ("(ORBextractor_extract_images: one call for the pair, staged in one pinned block, "
                            if host_pair else "(two extractor calls on two threads, ")
                         + f"2 x {W * H} B H2D), the Frame's results copied back before the clock stops "
                         f"(~{int(np.mean(d2h_bytes))} B D2H: keypoints + descriptors L/R, mvuRight, mvDepth, "
                         "mTcw, mvpMapPoints, mvbOutlier) -- System::TrackStereo semantics (System.cc:116)")
        else:
            out["io"] = "device: images HBM-resident, results left in HBM"
        return out

    def sequence_leg(S, nf):
        """Sequence-shaped throughput: S independent stereo sequences tracked concurrently, each
        frame by frame in order exactly as the latency leg tracks one (the motion model from the
        sequence's own previous estimated poses, Tracking.cc:867-928; the local map from its last
        K_LOCAL frames; every call synchronous, Frame + TrackWithMotionModel + TrackLocalMap), each
        sequence on its own host thread with its own matcher, extractor and buffers (a serving
        process with S camera streams, or S SLAM sessions).  -> frames/s over all sequences."""
        import threading
        import gc
        mts = []
        for _ in range(S):
            mt = orb.ORBmatcher(0.9, True)
            check(L.ORBmatcher_set_device_pointers(mt._h, 1))
            mts.append(mt)
        bar = threading.Barrier(S)
        outs, errs = [None] * S, [None] * S

        def work(i):
            try:
                torch.cuda.set_device(dev)
                outs[i] = latency_leg(nf, mm=mts[i], barrier=bar)
            except Exception as e:  # noqa: BLE001 -- re-raised below
                errs[i] = e
                bar.abort()

        gc_was = gc.isenabled()
        gc.collect()
        gc.disable()
        try:
            ts = [threading.Thread(target=work, args=(i,)) for i in range(S)]
            for t in ts:
                t.start()
            for t in ts:
                t.join()
        finally:
            if gc_was:
                gc.enable()
        for e in errs:
            if e is not None:
                raise e
        t0 = min(o["_span_s"][0] for o in outs)
        t1 = max(o["_span_s"][1] for o in outs)
        frames = S * min(nf, B)
        p50 = [o["p50_ms"] for o in outs]
        return {"metric": "tracked stereo frames/s, S concurrent sequences (frames in order, batch 1 each)",
                "value": round(frames / (t1 - t0), 1), "unit": "frames/s", "sequences": S,
                "frames_per_sequence": min(nf, B), "wall_s": round(t1 - t0, 4),
                "p50_ms_per_frame_range": [round(min(p50), 3), round(max(p50), 3)],
                "max_rotation_error": round(max(o["max_rotation_error"] for o in outs), 6),
                "io": "device: images HBM-resident, results left in HBM (each sequence as latency.p50_ms)"}

    def matcher_pass(lane, reps):
        """Isolated matcher launches with device timing and work counters:
        algorithmic bytes per SURVEY §8d = 32 B streamed candidate descriptor + 4 B index per
        scored pair + 16 B per query (query descriptor held in registers)."""
        check(L.ORBmatcher_enable_timing(m._h, 1), "ORBmatcher_enable_timing")
        ms = np.zeros(8, np.float32)
        cnt = np.zeros(8, np.int64)
        acc = {k: [] for k in ("k_build_grid", "k_candidates", "k_select", "k_stereo_rows", "k_stereo_match",
                               "k_stereo_filter", "k_csr_hamming")}
        work = {k: [] for k in ("search_pairs", "search_queries", "stereo_pairs", "stereo_queries", "csr_pairs",
                                "csr_queries", "stereo_sad")}

        def grab(kernels, counters):
            check(L.ORBmatcher_last_timings(m._h, ms.ctypes.data, cnt.ctypes.data), "ORBmatcher_last_timings")
            for k, i in kernels:
                acc[k].append(float(ms[i]))
            for k, i in counters:
                work[k].append(int(cnt[i]))

        # dense tiles: frame b's left descriptors against frame b+1's (16 pairs of ~1200 x 1200)
        B2 = min(16, B - 1)
        nL = lane.nL
        qd = torch.cat([lane.d_desc[b, :nL[b]] for b in range(B2)]).contiguous()
        td = torch.cat([lane.d_desc[b + 1, :nL[b + 1]] for b in range(B2)]).contiguous()
        tbase = np.concatenate([[0], np.cumsum(nL[1:B2 + 1])])[:B2]
        cand = torch.cat([(int(tbase[b]) + torch.arange(int(nL[b + 1]), dtype=torch.int32, device=dev)).repeat(int(nL[b]))
                          for b in range(B2)]).contiguous()
        per_q = torch.cat([torch.full((int(nL[b]),), int(nL[b + 1]), dtype=torch.int32, device=dev) for b in range(B2)])
        off = torch.zeros(len(per_q) + 1, dtype=torch.int32, device=dev)
        off[1:] = torch.cumsum(per_q, 0)
        nq = len(per_q)
        dist = torch.empty(len(cand), dtype=torch.int32, device=dev)
        bi, bd, sd = (torch.empty(nq, dtype=torch.int32, device=dev) for _ in range(3))
        pose_ms, pose_edges, pms = [], [], C.c_float()
        torch.cuda.synchronize()
        for _ in range(reps):
            lane.stereo()
            grab((("k_stereo_rows", 3), ("k_stereo_match", 4), ("k_stereo_filter", 5)),
                 (("stereo_pairs", 2), ("stereo_queries", 3), ("stereo_sad", 7)))
            lane.search()
            grab((("k_build_grid", 0), ("k_candidates", 1), ("k_select", 2)),
                 (("search_pairs", 0), ("search_queries", 1)))
            # PoseOptimization of the same batch (TrackWithMotionModel's call), k_pose_opt timed alone
            check(L.Optimizer_pose_timing(1, None), "Optimizer_pose_timing")
            check(L.Optimizer_PoseOptimization_frames_device(P, lane.pframes, lane.a_Tout, lane.a_poutl,
                                                             ptr(lane.ninl)), "PoseOptimization (isolated)")
            check(L.Optimizer_pose_timing(0, C.byref(pms)), "Optimizer_pose_timing")
            pose_ms.append(pms.value)
            pose_edges.append((int(lane.n_pose.sum()), int(lane.ninl.sum())))
            check(L.ORBmatcher_SearchCandidates(m._h, C.c_void_p(qd.data_ptr()), nq, C.c_void_p(td.data_ptr()),
                                                len(td), C.c_void_p(off.data_ptr()), C.c_void_p(cand.data_ptr()),
                                                None, C.c_void_p(bi.data_ptr()),
                                                C.c_void_p(bd.data_ptr()), C.c_void_p(sd.data_ptr())), "SearchCandidates")
            grab((("k_csr_hamming", 6),), (("csr_pairs", 4), ("csr_queries", 5)))
        # the same 16 tiles through the brute-force kernel (LDS-resident train blocks, no
        # candidate lists): SURVEY config 2 (ii) as the north star states it
        bi_l = [torch.empty(int(nL[b]), dtype=torch.int32, device=dev) for b in range(B2)]
        bd_l = [torch.empty(int(nL[b]), dtype=torch.int32, device=dev) for b in range(B2)]
        sd_l = [torch.empty(int(nL[b]), dtype=torch.int32, device=dev) for b in range(B2)]
        qp = arr([lane.d_desc[b].data_ptr() for b in range(B2)])
        tp = arr([lane.d_desc[b + 1].data_ptr() for b in range(B2)])
        nq_d = np.ascontiguousarray(nL[:B2], np.int32)
        nt_d = np.ascontiguousarray(nL[1:B2 + 1], np.int32)
        dense_ms, dense_pairs = [], []
        dms, dpairs = C.c_float(), C.c_longlong()
        for _ in range(reps):
            check(L.ORBmatcher_SearchDense_batch(m._h, B2, qp, ptr(nq_d), tp, ptr(nt_d),
                                                 arr([x.data_ptr() for x in bi_l]), arr([x.data_ptr() for x in bd_l]),
                                                 arr([x.data_ptr() for x in sd_l])), "SearchDense_batch")
            check(L.ORBmatcher_last_dense_timing(m._h, C.byref(dms), C.byref(dpairs)), "last_dense_timing")
            dense_ms.append(dms.value)
            dense_pairs.append(dpairs.value)
        # the dense kernel's answer equals the CSR engine's on the same tiles (bit-exact)
        csr_bd = bd.cpu().numpy()
        dense_ok = bool(np.array_equal(np.concatenate([x.cpu().numpy() for x in bd_l]), csr_bd) and
                        np.array_equal(np.concatenate([x.cpu().numpy() for x in sd_l]), sd.cpu().numpy()))
        check(L.ORBmatcher_enable_timing(m._h, 0), "ORBmatcher_enable_timing")
        pmc = {}
        pf = ROOT / "profiles" / MATCH_PMC_FILE
        if pf.exists():
            try:
                pmc = json.loads(pf.read_text())
            except Exception:
                pmc = {}
        out = {}
        for k, pk, qk in (("k_candidates", "search_pairs", "search_queries"), ("k_stereo_match", "stereo_pairs",
                                                                               "stereo_queries"),
                          ("k_csr_hamming", "csr_pairs", "csr_queries")):
            t = float(np.mean(acc[k]))
            pairs, qs = float(np.mean(work[pk])), float(np.mean(work[qk]))
            alg = pairs * 36 + qs * 16
            sad = float(np.mean(work["stereo_sad"])) if k == "k_stereo_match" else 0.0
            alg += sad * STEREO_WINDOW_BYTES   # the SAD windows ComputeStereoMatches reads (Frame.cc:560-588)
            gbs = alg / (t * 1e-3) / 1e9
            e = {"avg_launch_ms": round(t, 4), "pairs_per_launch": int(pairs), "queries_per_launch": int(qs),
                 "alg_bytes_per_launch": int(alg), "achieved": round(gbs, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                 "frac": round(gbs / HBM_PEAK_GBS, 5), "pairs_per_s": round(pairs / (t * 1e-3), 1)}
            if k in pmc:
                e["traffic"] = pmc[k].get("hbm_bytes_per_launch")
                if e["traffic"]:   # what HBM actually moved (descriptor re-reads are L2/MALL hits)
                    e["hbm_achieved"] = round(e["traffic"] / (t * 1e-3) / 1e9, 2)
                    e["hbm_frac"] = round(e["hbm_achieved"] / HBM_PEAK_GBS, 5)
                vi = pmc[k].get("valu_insts_per_launch")
                if vi:
                    vr = vi / (t * 1e-3) / 1e9
                    e["valu"] = {"insts_per_launch": int(vi), "achieved": round(vr, 1), "peak": VALU_PEAK_GINST,
                                 "unit": "G wave-instr/s", "frac": round(vr / VALU_PEAK_GINST, 4)}
                e["pmc_source"] = f"profiles/{MATCH_PMC_FILE}"
            if k == "k_stereo_match":
                e["sad_keypoints_per_launch"] = int(sad)
                e["alg_bytes_note"] = (f"36 B per scored pair + 16 B per query + {STEREO_WINDOW_BYTES} B per keypoint "
                                       "whose SAD windows are read (11x11 left window + the 11x21 right band it "
                                       "slides over)")
            if k == "k_csr_hamming":
                relabel_valu(e, "36 B per (query, candidate) pair: the dense tiles' candidates are L2/MALL-resident "
                                "re-reads (see traffic), so this kernel is bound by VALU popcount issue, not HBM")
            out[k] = e
        out["k_csr_hamming"]["workload"] = f"dense tiles: {B2} frame pairs, every left descriptor of frame b against " \
                                           f"every left descriptor of frame b+1 (SURVEY config 2 (ii))"
        t = float(np.mean(dense_ms))
        pairs = float(np.mean(dense_pairs))
        qs = float(nq_d.sum())
        alg = pairs * 32 + qs * 16          # streamed train descriptor per pair + 16 B out per query
        ed = {"avg_launch_ms": round(t, 4), "pairs_per_launch": int(pairs), "queries_per_launch": int(qs),
              "alg_bytes_per_launch": int(alg), "pairs_per_s": round(pairs / (t * 1e-3), 1),
              "achieved": round(alg / (t * 1e-3) / 1e9, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
              "equals_csr_result": dense_ok,
              "workload": f"the same {B2} dense tiles as k_csr_hamming, brute force over LDS-resident 256-row train "
                          "blocks (k_dense_hamming + k_dense_merge; time = both kernels)",
              "note": "alg bytes count 32 B per pair as if every pair streamed its train descriptor; the kernel "
                      "reads each train block once per 256 queries (LDS broadcast), so it is VALU-bound: see valu"}
        if "k_dense_hamming" in pmc:
            e2 = pmc["k_dense_hamming"]
            if e2.get("hbm_bytes_per_launch"):
                ed["traffic"] = e2["hbm_bytes_per_launch"]
                ed["hbm_achieved"] = round(ed["traffic"] / (t * 1e-3) / 1e9, 2)
                ed["hbm_frac"] = round(ed["hbm_achieved"] / HBM_PEAK_GBS, 5)
            vi = e2.get("valu_insts_per_launch")
            if vi:
                vr = vi / (t * 1e-3) / 1e9
                ed["valu"] = {"insts_per_launch": int(vi), "achieved": round(vr, 1), "peak": VALU_PEAK_GINST,
                              "unit": "G wave-instr/s", "frac": round(vr / VALU_PEAK_GINST, 4)}
            ed["pmc_source"] = f"profiles/{MATCH_PMC_FILE}"
        # popcount bound: 8 XOR + 8 POPC per pair = 16 lane-ops at the chip's VALU issue roof
        pk_peak = VALU_PEAK_GINST * 64 / 16 * 1e9
        ed["popcount_bound"] = {"pairs_per_s": ed["pairs_per_s"], "peak_pairs_per_s": round(pk_peak, 1),
                                "frac": round(ed["pairs_per_s"] / pk_peak, 4),
                                "definition": "8 v_xor + 8 v_bcnt lane-ops per 256-bit pair at 1228.8 G wave64 "
                                              "VALU instructions/s (256 CUs x 2 issues/cycle x 2.4 GHz)"}
        relabel_valu(ed, "32 B per pair if every pair streamed its train descriptor; each train block is read "
                         "once per 256 queries (LDS broadcast), so the kernel is bound by VALU popcount issue")
        out["k_dense_hamming"] = ed
        # k_pose_opt (the tracking lane's critical path): one workgroup per frame runs the whole LM
        # loop; bound by the VALU issue of the CUs it occupies
        t = float(np.mean(pose_ms))
        ep = {"avg_launch_ms": round(t, 4), "frames_per_launch": P,
              "keypoints_per_launch": int(np.mean([a for a, _ in pose_edges])),
              "inliers_per_launch": int(np.mean([b for _, b in pose_edges])),
              "bound": "valu", "workload": "TrackWithMotionModel's PoseOptimization of the batch (one 512-thread "
                                           "workgroup per frame: 4 rounds of optimize(10))"}
        pk = next((k for k in pmc if k.startswith("k_pose_opt")), None)
        if pk and pmc[pk].get("valu_insts_per_launch"):
            vi = pmc[pk]["valu_insts_per_launch"]
            vr = vi / (t * 1e-3) / 1e9
            ep.update({"insts_per_launch": int(vi), "achieved": round(vr, 1), "peak": VALU_PEAK_GINST,
                       "unit": "G wave-instr/s", "frac": round(vr / VALU_PEAK_GINST, 4),
                       "frac_of_occupied_cus": round(vr / (VALU_PEAK_GINST * P / 256), 4),
                       "pmc_source": f"profiles/{MATCH_PMC_FILE}"})
            if pmc[pk].get("hbm_bytes_per_launch"):
                ep["traffic"] = pmc[pk]["hbm_bytes_per_launch"]
        out["k_pose_opt"] = ep
        for k in ("k_build_grid", "k_select", "k_stereo_rows", "k_stereo_filter"):
            out[k] = {"avg_launch_ms": round(float(np.mean(acc[k])), 4), "bound": "latency (one workgroup per frame)"}
        out["definition"] = ("alg bytes = 36 B per scored (query, candidate) pair (32 B candidate descriptor + 4 B "
                             "index) + 16 B per query, SURVEY §8d; duration = HIP events on the matcher stream, "
                             f"mean of {reps} isolated launches; hbm_achieved = PMC HBM bytes per launch / duration "
                             "(the candidate descriptors of a frame are re-read from L2/MALL, so alg bytes exceed "
                             "HBM traffic: the dense tile's 36 B/pair run at L2 rate)")
        return out

    stage_acc = {}
    stage_lr = {"left": {}, "right": {}}   # the same per extractor stream (left / right images)
    phase_acc = {}
    local_acc = []
    pose_inl = []
    kernel_ms = []   # k_fast_cells duration per step (HIP events on the extractor streams)
    # every lane's matcher before any extractor: HIP deals new streams to its hardware queues in
    # creation order, so the matchers' streams come out on queues of their own
    lane_m = [m]
    for _ in range(1, args.lanes):
        if args.lane_matchers:
            lane_m.append(orb.ORBmatcher(0.9, True))
            check(L.ORBmatcher_set_device_pointers(lane_m[-1]._h, 1))
        else:
            lane_m.append(m)
    # --sequence: a ring of three (B, 4, 4) estimate sets (est[t % 3][b] = the estimate of image b
    # made at step t; image 0 has no pair and keeps the generator's pose as the anchor) and the
    # event after the last chain's estimates
    seq = {"est": [d_Tcw.view(B, 4, 4).clone() for _ in range(3)], "t": 0, "ev": None}

    def rigid_inv_t(T):
        """Batched Twc from Tcw (Frame::UpdatePoseMatrices: R^T, -R^T t)."""
        Ti = torch.zeros_like(T)
        Rt = T[:, :3, :3].transpose(1, 2)
        Ti[:, :3, :3] = Rt
        Ti[:, :3, 3] = -(Rt @ T[:, :3, 3:4])[:, :, 0]
        Ti[:, 3, 3] = 1.0
        return Ti

    def seq_predict(lane):
        """Per sequence (pair p: LastFrame = image p, CurrentFrame = image p + 1): LastFrame.mTcw is
        image p's estimate from the previous step, mVelocity = T_{c-1} T_{c-2}^-1 from the previous
        two steps' estimates, the prediction mVelocity T_{c-1} (Tracking.cc:867-928, 1281-1291), all
        on the lane's matcher stream after the previous step's estimates landed."""
        t = seq["t"]
        e1, e2 = seq["est"][(t - 1) % 3], seq["est"][(t - 2) % 3]
        with torch.cuda.stream(lane.ms):
            if seq["ev"] is not None:
                lane.ms.wait_event(seq["ev"])
            lane.sLast.copy_(e1.reshape(B, 16))
            lane.sTwc.copy_(rigid_inv_t(e1).reshape(B, 16))
            Tm1 = e1[:-1]                                            # T_{c-1}, c = 1 .. B-1
            V = torch.eye(4, dtype=torch.float32, device=dev).repeat(B - 1, 1, 1)
            V[1:] = Tm1[1:] @ rigid_inv_t(e2[:-2])                    # c >= 2: T_{c-1} T_{c-2}^-1
            lane.sPred[1:].copy_((V @ Tm1).reshape(B - 1, 16))

    def seq_record(lane):
        """This step's estimates (TrackLocalMap's PoseOptimization) into the ring, then the event the
        next step's chain waits on."""
        t = seq["t"]
        with torch.cuda.stream(lane.ms):
            seq["est"][t % 3][1:].copy_(lane.d_Tout2.view(P, 4, 4))
            ev = torch.cuda.Event()
            ev.record(lane.ms)
        seq["ev"] = ev
        seq["t"] = t + 1

    lanes = [Lane(mt) for mt in lane_m]
    exL = lanes[0].exL
    if args.reserve_cus:
        # the tracking lane's one-workgroup-per-frame kernels (k_select, k_pose_opt) need free
        # wave slots while a batch is extracted: the extractor streams leave 1 CU in N out
        for ln in lanes:
            for ex in (ln.exL, ln.exR):
                check(L.ORBextractor_reserve_cus(ex._h, args.reserve_cus), "ORBextractor_reserve_cus")
    if args.shared_ex_stream:
        if not args.stereo_batch:
            sys.exit("bench.py: --shared-ex-stream needs --stereo-batch 1 (one extractor per lane)")
        for ln in lanes[1:]:
            check(L.ORBextractor_share_stream(ln.exL._h, lanes[0].exL._h), "ORBextractor_share_stream")
    if args.depth > 1 and len(lanes) < 3 and not args.shared_ex_stream:
        sys.exit("bench.py: --depth 2 needs --lanes >= 3 (a lane's buffers are reused by batch k + lanes) "
                 "or --shared-ex-stream 1")
    ex_pool = ThreadPoolExecutor(2 if args.depth > 1 else 1, initializer=lambda: torch.cuda.set_device(dev))
    state = {"k": 0, "ready": None, "pending": None, "inflight": None}

    def step_deep():
        """Two extractions in flight: batch k's extraction is queued first (a worker thread; its
        kernels wait only for the GPU), then the host waits for batch k-1's extraction, enqueues its
        tracking chain and collects batch k-2's counts.  The extraction lane never idles while the
        host enqueues a chain.  -> the collected batch's counts (None before the pipeline is full)."""
        lane = lanes[state["k"] % len(lanes)]
        te = time.perf_counter()
        fut = ex_pool.submit(lane.extract)
        res = None
        if state["inflight"] is not None:
            pl, pf = state["inflight"]
            pf.result()
            pl.enqueue()
            if state["pending"] is not None:
                res = state["pending"].collect()
            state["pending"] = pl
        state["inflight"] = (lane, fut)
        phase_acc["step_wall"] = phase_acc.get("step_wall", 0.0) + (time.perf_counter() - te) * 1e3
        state["k"] += 1
        return res

    def step():
        if args.depth > 1:
            return step_deep()
        """Software pipeline over two lanes: the extraction of batch k (worker threads, extractor
        streams) runs while batch k-1's tracking chain is queued on the matcher stream right
        behind batch k-2's; batch k-2's counts are collected while k-1's chain runs.  -> the
        collected batch's counts (None before the pipeline is full)."""
        lane = lanes[state["k"] % len(lanes)]
        te = time.perf_counter()
        if args.enqueue_first and state["ready"] is not None:
            # the tracking chain's launches first, then the extraction's: the two threads' launch
            # streams do not interleave on the host
            state["ready"].enqueue()
            fut = ex_pool.submit(lane.extract)
        else:
            fut = ex_pool.submit(lane.extract)
            if state["ready"] is not None:
                state["ready"].enqueue()
        res = None
        if state["ready"] is not None:
            if state["pending"] is not None:
                res = state["pending"].collect()
            state["pending"] = state["ready"]
        fut.result()
        phase_acc["step_wall"] = phase_acc.get("step_wall", 0.0) + (time.perf_counter() - te) * 1e3
        state["ready"] = lane
        state["k"] += 1
        return res

    def host_io_pass(nsteps):
        """The headline pipeline with host-resident input, as System::TrackStereo receives it
        (System.cc:116-165: cv::Mats in pageable host memory): each step's 2B images are copied from
        one pageable host array into a pinned staging block (host memcpy, torch's intra-op threads)
        and DMA'd to the lane's own device buffer on a copy stream, one step ahead, so the upload of
        batch k+1 overlaps batch k's extraction and tracking; the extraction of a batch waits on its
        upload's event.  -> frames/s over nsteps timed steps and the achieved H2D rate."""
        src = torch.from_numpy(np.ascontiguousarray(np.concatenate([lefts, rights])))   # pageable
        nbytes = src.numel()
        stage = [torch.empty_like(src).pin_memory() for _ in lanes]
        dimg = [torch.empty_like(d_LR) for _ in lanes]
        cs = torch.cuda.Stream(dev)
        # the copy in max(1, --h2d-streams) pieces on as many streams (DMA engines side by side); cs
        # starts and joins them, so its events bracket the whole step's upload
        nsplit = max(1, args.h2d_streams)
        cs_more = [torch.cuda.Stream(dev) for _ in range(nsplit - 1)]
        ev_piece = [torch.cuda.Event() for _ in range(nsplit - 1)]
        ev_done = [torch.cuda.Event() for _ in lanes]
        ev_t = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in lanes]
        up_pool = ThreadPoolExecutor(1, initializer=lambda: torch.cuda.set_device(dev))
        stats = {"memcpy_s": 0.0, "dma_ms": [], "n": 0}

        def upload(j):
            ev_done[j].synchronize()            # the previous DMA out of stage[j] is finished
            t = time.perf_counter()
            stage[j].copy_(src)                 # pageable -> pinned (host memcpy)
            stats["memcpy_s"] += time.perf_counter() - t
            n = dimg[j].numel()
            cuts = [n * q // nsplit for q in range(nsplit + 1)]
            dflat, sflat = dimg[j].view(-1), stage[j].view(-1)
            with torch.cuda.stream(cs):
                ev_t[j][0].record(cs)
            for q, sq in enumerate(cs_more):
                sq.wait_event(ev_t[j][0])
                with torch.cuda.stream(sq):
                    dflat[cuts[q + 1]:cuts[q + 2]].copy_(sflat[cuts[q + 1]:cuts[q + 2]], non_blocking=True)
                    ev_piece[q].record(sq)
            with torch.cuda.stream(cs):
                dflat[cuts[0]:cuts[1]].copy_(sflat[cuts[0]:cuts[1]], non_blocking=True)
                for e in ev_piece:
                    cs.wait_event(e)
                ev_t[j][1].record(cs)
                ev_done[j].record(cs)
            stats["n"] += 1

        saved = [(ln.img_ptr, ln.img_ev) for ln in lanes]
        import copy
        acc_saved = copy.deepcopy((stage_acc, stage_lr, phase_acc, kernel_ms, pose_inl, local_acc))
        try:
            for j, ln in enumerate(lanes):
                ln.img_ptr, ln.img_ev = dimg[j].data_ptr(), ev_done[j]
            drain()
            torch.cuda.synchronize()
            nl = len(lanes)
            k0 = state["k"]
            pend = up_pool.submit(upload, k0 % nl)
            pend.result()
            for _ in range(2):   # warm: the pipeline primed with host-uploaded batches
                pend = up_pool.submit(upload, (state["k"] + 1) % nl)
                step()
                pend.result()
            drain()
            pend = up_pool.submit(upload, state["k"] % nl)
            pend.result()
            pend = up_pool.submit(upload, (state["k"] + 1) % nl)
            step()   # prime: batch extracted, awaiting tracking
            pend.result()
            stats.update(memcpy_s=0.0, n=0)
            if world > 1:
                dist.barrier()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(nsteps):
                pend = up_pool.submit(upload, (state["k"] + 1) % nl)   # the next batch, during this step
                step()
                pend.result()
            torch.cuda.synchronize()
            if world > 1:
                dist.barrier()
            dt_h = time.perf_counter() - t0
            dma_ms = [ev_t[j][0].elapsed_time(ev_t[j][1]) for j in range(nl)]
            drain()
        finally:
            for ln, (ip, ie) in zip(lanes, saved):
                ln.img_ptr, ln.img_ev = ip, ie
            up_pool.shutdown()
            # the headline's per-stage accumulators are the main timed region's only
            for cur, old in zip((stage_acc, stage_lr, phase_acc, kernel_ms, pose_inl, local_acc), acc_saved):
                cur.clear()
                (cur.update if isinstance(cur, dict) else cur.extend)(old)
        if world > 1:
            t = torch.tensor([dt_h], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            dt_h = float(t.item())
        fps_h = P * nsteps * world / dt_h
        return {"value": round(fps_h, 2), "unit": "frames/s", "steps": nsteps,
                "ms_per_step": round(dt_h / nsteps * 1e3, 3),
                "h2d_bytes_per_step": int(nbytes),
                "h2d_GBps_achieved": round(nbytes / (float(np.mean(dma_ms)) * 1e-3) / 1e9, 2),
                "host_memcpy_GBps": round(nbytes * stats["n"] / max(stats["memcpy_s"], 1e-9) / 1e9, 2),
                "h2d_streams": nsplit,
                "io": "host: each step's 2B images from one pageable host array -> pinned staging (host memcpy) "
                      "-> H2D DMA in h2d_streams pieces on as many copy streams, one step ahead of the "
                      "extraction that waits on it; h2d_GBps_achieved = bytes / the DMA's HIP-event time"}

    def drain():
        """Track the extracted batch, collect every chain in order, leave the matcher synchronous."""
        out = []
        if state["inflight"] is not None:   # (--depth 2) the batch being extracted
            pl, pf = state["inflight"]
            pf.result()
            state["inflight"] = None
            state["ready"] = pl
        if state["ready"] is not None:
            state["ready"].enqueue()
            if state["pending"] is not None:
                out.append(state["pending"].collect())
            state["pending"] = state["ready"]
            state["ready"] = None
        if state["pending"] is not None:
            out.append(state["pending"].collect())
            state["pending"] = None
        for ln in lanes:
            check(L.ORBmatcher_set_deferred(ln.m._h, 0), "ORBmatcher_set_deferred")
        return out

    def stage_by_stream():
        """Extraction stage ms per step by extractor stream (--stereo-batch: one stream, both images)."""
        per = {side: {k: round(v / args.steps, 4) for k, v in d.items()} for side, d in stage_lr.items()}
        return {"left+right (one 2B-image stream)": per["left"]} if args.stereo_batch else per

    if args.passes_only or args.latency_only:   # one extracted, tracked batch; then the legs below
        args.warmup, args.steps = 1, 0
    for _ in range(args.warmup):
        step()
    drain()
    step()   # prime the pipeline: one batch extracted, awaiting tracking
    stage_acc.clear()
    for d in stage_lr.values():
        d.clear()
    phase_acc.clear()
    kernel_ms.clear()
    pose_inl.clear()
    local_acc.clear()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    got = []
    for _ in range(args.steps):
        r = step()
        if r is not None:
            got.append(r)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if os.environ.get("ORBGPU_PROF_DUMP"):   # instrumented build (make prof): k_select section timers
        buf = (C.c_ulonglong * 32)()
        L.orbgpu_debug_prof_match(buf)
        print("k_select sections (cycles, problem 0, summed over the timed steps):", list(buf)[:16], file=sys.stderr)
    # the last timed chain's counts (its device work finished inside the timed region), then the
    # batch extracted by the last timed step, tracked outside it
    got += drain()[:1] if args.steps else []
    tot_kp = sum(r[0] for r in got)
    tot_match = sum(r[1] for r in got)
    tot_stereo = sum(r[2] for r in got)
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
        c = torch.tensor([tot_match, tot_kp, tot_stereo], dtype=torch.float64, device=dev)
        dist.all_reduce(c)
        tot_match, tot_kp, tot_stereo = (int(v) for v in c.tolist())
    # value credits the frames a step TRACKS: every one of the B stereo pairs is extracted and
    # stereo-matched, but frame 0 of a batch has no LastFrame, so P = B - 1 frames go through
    # TrackWithMotionModel + TrackLocalMap
    frames_total = P * args.steps * world
    fps = frames_total / dt
    host_io = None
    if args.steps and not args.latency_only and not args.passes_only:
        host_io = host_io_pass(min(args.steps, 30))
    if args.latency_only:
        if rank == 0:
            lat = latency_leg(24)
            lat["host_path"] = latency_leg(24, host_io=True)
            lat["sequences"] = {str(S): sequence_leg(S, 24) for S in (4, 16)}
            for v in (lat, lat["host_path"]):
                v.pop("_span_s", None)
            print(json.dumps({"latency": lat}), file=json_out, flush=True)
        return
    if args.pipeline_only:   # the yaml feature count's line: pipeline + its CPU baseline
        if rank == 0:
            cpu = None if args.no_cpu_baseline else cpu_baseline(lefts, rights, Rs, args.cpu_seconds)
            line = {"nfeatures": NFEAT, "value": round(fps, 2), "unit": "frames/s", "steps": args.steps,
                    "sequence": bool(args.sequence),
                    "ms_per_step": round(dt / args.steps * 1e3, 3), "tracked_frames_per_step": P,
                    "matches_per_s": round(tot_match / dt, 1),
                    "keypoints_per_image": round(tot_kp / (2 * B * args.steps * world), 1), "cpu_baseline": cpu,
                    "stage_ms_per_step_by_image": stage_by_stream(),
                    "phase_ms_per_step": {k: round(v / args.steps, 4) for k, v in phase_acc.items()},
                    "value_host_io": host_io}
            if cpu:
                line["speedup_vs_cpu_all_core"] = round(fps / cpu["value"], 1)
            if args.sequence:   # the estimates stay on the true trajectory (rotation, max abs entry)
                torch.cuda.synchronize()
                est = seq["est"][(seq["t"] - 1) % 3][1:, :3, :3]
                line["max_rotation_error"] = round(float((est - d_Tcw.view(B, 4, 4)[1:, :3, :3]).abs().max()), 6)
                line["note"] = ("B sequences in lock step: every pair's LastFrame pose and motion-model prediction "
                                "from the previous steps' estimates (device-side, no host round trip), so each step's "
                                "tracking chain waits for the previous step's")
            json_out.write(json.dumps(line) + "\n")
            json_out.flush()
        if world > 1:
            dist.destroy_process_group()
        return

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
    corners = exL.last_corner_count()   # FAST corners this pass wrote (all B images)
    alg_bytes = B * (lvl_px + 4 * 1220) + 4 * corners
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
    roof_fast = {"bound": "hbm", "kernel": "k_fast_cells", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
            "traffic_source": traffic_src, "avg_launch_ms": round(k_avg_ms, 4), "launches": ROOFLINE_REPS,
            "alg_bytes_per_launch": alg_bytes, "corners_per_launch": corners,
            "avg_launch_ms_in_pipeline": round(float(np.mean(kernel_ms)), 4),
            "secondary_bound": "VALU (16-px circle test; DESIGN.md §3)", "valu": valu}

    # matcher roofline (north star: "achieved HBM GB/s for the matcher ... against the chip's
    # peak"): the ready lane's ComputeStereoMatches and SearchByProjection batches and a dense
    # 1200x1200 descriptor tile per frame pair (SURVEY config 2 (ii)) through the CSR engine,
    # each ROOFLINE_REPS times with nothing else in flight, HIP events on the matcher stream
    if args.stereo_batch:
        # the roofline pass above left the shared [lefts | rights] extractor's last batch at the B
        # left images: extract the lane's stereo batch again for the matcher passes
        lanes[0].extract()
    mroof = matcher_pass(lanes[0], ROOFLINE_REPS)
    roof = pose_roofline(mroof["k_pose_opt"], roof_fast)
    if args.passes_only:
        return
    latency = latency_leg(24)
    latency["host_path"] = latency_leg(24, host_io=True)
    latency["sequences"] = {str(S): sequence_leg(S, 24) for S in (4, 16)}
    for v in [latency] + [latency["host_path"]]:
        v.pop("_span_s", None)

    # CPU baselines (the reference CPU path timed "in the same run"): rank 0 only.  At
    # N = 1 each runs right after its GPU leg; at N > 1 rank 0 runs them all after every GPU leg,
    # while the other ranks wait at a barrier, so no GPU leg shares the host cores with them.
    want_cpu = rank == 0 and not args.no_cpu_baseline
    inline_cpu = want_cpu and world == 1
    cpu = None
    if inline_cpu:
        cpu = cpu_baseline(lefts, rights, Rs, args.cpu_seconds)

    # local BA (BASELINE metric part 3): SURVEY config 4 on every rank (replicas), own timed region
    ba = bench_local_ba(args, world, rank, dist if world > 1 else None, dev)
    if inline_cpu:
        ba["cpu_baseline"] = ba_cpu_baseline(args.cpu_seconds / 4)
    # global BA (SURVEY config 5): ONE problem keyframe-block sharded over the ranks, RCCL exchange
    gba = bench_global_ba(args, world, rank, dist if world > 1 else None, dev)
    if inline_cpu:
        gba["cpu_baseline"] = gba_cpu_baseline(args.gba_kf, gba_laps(args))
    # RANSAC hypothesis scoring (SURVEY config 3): every rank runs it (replicas), rank 0 reports
    ransac = bench_ransac(cpu=inline_cpu, cpu_budget_s=args.cpu_seconds / 3)
    if want_cpu and world > 1:
        cpu = cpu_baseline(lefts, rights, Rs, args.cpu_seconds)
        ba["cpu_baseline"] = ba_cpu_baseline(args.cpu_seconds / 4)
        gba["cpu_baseline"] = gba_cpu_baseline(args.gba_kf, gba_laps(args))
        ransac_cpu_into(ransac, args.cpu_seconds / 3)
    if world > 1:
        dist.barrier()

    ransac.pop("_cpu_args", None)
    nf2000 = seqline = None
    if rank == 0 and world == 1 and NFEAT != 2000:
        # the same pipeline at the yaml's nFeatures 2000 (KITTI00-02.yaml:38) in a
        # fresh process (its own extractors and arenas), with its own CPU baseline
        import subprocess
        cmd = [sys.executable, str(Path(__file__).resolve()), "--nfeatures", "2000", "--pipeline-only",
               "--steps", str(max(10, args.steps // 3)), "--warmup", "3", "--cpu-seconds", str(args.cpu_seconds / 2)]
        if args.no_cpu_baseline:
            cmd.append("--no-cpu-baseline")
        try:
            r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
            nf2000 = json.loads(r.stdout.strip().splitlines()[-1]) if r.returncode == 0 else \
                {"error": f"exit {r.returncode}", "stderr_tail": r.stderr[-400:]}
        except Exception as e:  # noqa: BLE001 -- reported in the line, the headline stands
            nf2000 = {"error": f"{type(e).__name__}: {e}"}
        # the sequence-shaped pipeline (--sequence 1): the same step with each pair's poses from the
        # previous steps' estimates, in a fresh process
        cmd = [sys.executable, str(Path(__file__).resolve()), "--sequence", "1", "--pipeline-only", "--no-cpu-baseline",
               "--steps", str(max(10, args.steps // 2)), "--warmup", "3"]
        try:
            r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
            seqline = json.loads(r.stdout.strip().splitlines()[-1]) if r.returncode == 0 else \
                {"error": f"exit {r.returncode}", "stderr_tail": r.stderr[-400:]}
        except Exception as e:  # noqa: BLE001 -- reported in the line, the headline stands
            seqline = {"error": f"{type(e).__name__}: {e}"}
    if rank == 0:
        stage_ms = {k: round(v / args.steps, 4) for k, v in stage_acc.items()}
        out = {
            "metric": METRIC, "value": round(fps, 2), "unit": "frames/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u8",
            "data": "synthetic (seeded KITTI-shaped textured stereo frames: camera-rotation motion, "
                    "ground-plane disparity field 4..40 px)",
            "config": {"workload": "kitti00_stereo: ORB extract L+R, ComputeStereoMatches, "
                                   "TrackWithMotionModel (UpdateLastFrame, SearchByProjection(Cur,Last,th=7), "
                                   "PoseOptimization), TrackLocalMap (isInFrustum + SearchByProjection(F, local map "
                                   f"of the last {K_LOCAL} frames' map points, th=1) + PoseOptimization)",
                       "width": W, "height": H,
                       "nfeatures": NFEAT, "nlevels": 8, "scale_factor": 1.2, "fast_th": [20, 7],
                       "stereo_frames_per_step": B, "tracked_frames_per_step": P, "parallelism": f"replicas{world}", "extractor_cu_reserve": args.reserve_cus},
            "sequence_frames_per_s": round(1000.0 / latency["host_path"]["p50_ms"], 1),
            "sequence_frames_per_s_note": "one SLAM sequence (frames in order, batch 1) through the drop-in host "
                                          "path: 1000 / latency.host_path.p50_ms; `value` is batch throughput",
            "matches_per_s": round(tot_match / dt, 1), "stereo_matches_per_s": round(tot_stereo / dt, 1),
            "keypoints_per_image": round(tot_kp / (2 * B * args.steps * world), 1),
            "pose_inliers_per_frame": round(float(np.sum(pose_inl)) / max(len(pose_inl) * P, 1), 1),
            "local_map_matches_per_frame": round(float(sum(a for a, _ in local_acc)) / max(len(local_acc) * P, 1), 1),
            "local_map_visible_per_frame": round(float(sum(b for _, b in local_acc)) / max(len(local_acc) * P, 1), 1),
            "stage_ms_per_step": stage_ms,
            "stage_ms_per_step_by_image": stage_by_stream(),
            "phase_ms_per_step": {k: round(v / args.steps, 4) for k, v in phase_acc.items()}, "roofline": roof,
            "matcher_roofline": mroof, "latency": latency, "cpu_baseline": cpu, "local_ba": ba,
            "global_ba": gba, "ransac": ransac, "nfeatures_2000": nf2000, "sequence_pipeline": seqline,
        }
        if host_io is not None:
            host_io["frac_of_value"] = round(host_io["value"] / fps, 3)
            out["value_host_io"] = host_io
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
    # throughput form, the CPU baseline's shape (P independent LocalBundleAdjustment streams): S host
    # threads, each with its own engine, workspace and HIP stream, calling LocalBundleAdjustment in a
    # loop (the C calls release the GIL); one problem leaves most CUs idle, S of them share the chip
    from concurrent.futures import ThreadPoolExecutor
    S = LOCAL_BA_STREAMS

    def stream(i):
        n = 0
        for _ in range(reps):
            n += sum(LocalBundleAdjustment(*a)["iterations"])
        return n
    with ThreadPoolExecutor(S) as ex:
        list(ex.map(lambda i: LocalBundleAdjustment(*a), range(S)))   # per-thread engine warm-up
        if dist is not None:
            dist.barrier()
        t1 = time.perf_counter()
        its_s = sum(ex.map(stream, range(S)))
        dt_s = time.perf_counter() - t1
    if dist is not None:
        t = torch.tensor([dt_s, its_s], dtype=torch.float64, device=dev)
        dist.all_reduce(t[:1], op=dist.ReduceOp.MAX)
        dist.all_reduce(t[1:])
        dt_s, its_s = float(t[0].item()), int(t[1].item())
    sharded = bench_local_ba_sharded(args, world, rank, dist, dev, pr)
    return {"metric": "local-BA iter/s", "value": round(its_s / dt_s, 1), "unit": "iter/s", "sharded": sharded,
            "streams": S, "single_stream": {"value": round(its / dt, 1), "unit": "iter/s",
                                            "ms_per_call": round(dt / reps * 1e3, 3),
                                            "note": "one problem at a time (the LocalMapping thread's latency)"},
            "ms_per_call": round(dt / (reps * max(world, 1)) * 1e3 * max(world, 1), 3),
            "edges_per_s": round(its_s * ne / dt_s, 1), "calls": reps * world * (S + 1),
            "config": {"workload": "euroc_mh05_stereo_local_ba (SURVEY config 4)", "local_kfs": 15, "fixed_kfs": 15,
                       "points": len(pr["pt_id"]), "edges": ne,
                       "stereo_edges": int((pr["edge_obs"][:, 2] >= 0).sum()),
                       "lm": "optimize(5) + gating + optimize(10)", "parallelism": f"replicas{world}"},
            "dtype": "f64 (f32 I/O)"}


def bench_local_ba_sharded(args, world, rank, dist, dev, pr):
    """Optimizer_LocalBundleAdjustment_sharded on config 4 (north_star: "Local-BA
    residual/Jacobian evaluation shards by keyframe block across the GPUs ... with an RCCL
    all-reduce of the normal-equation update"): ONE problem, its map points partitioned by the
    block of their reference keyframe over the N ranks, an RCCL exchange per LM trial (strong
    scaling; at N = 1 the exchange steps are identities).  iter = one LM solve()."""
    import torch
    from c_orb_slam_amd.optimizer import Comm, LocalBundleAdjustmentSharded, partition_points, shard_problem
    shard = shard_problem(pr, partition_points(pr, world), rank)
    uid = [Comm.unique_id() if rank == 0 else None]
    if dist is not None:
        dist.broadcast_object_list(uid, src=0)
    comm = Comm.rccl(world, rank, uid[0])
    for _ in range(2):
        LocalBundleAdjustmentSharded(shard, comm)       # warm-up (allocations, structure)
    reps = max(5, args.steps)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    its = 0
    for _ in range(reps):
        its += sum(LocalBundleAdjustmentSharded(shard, comm)["iterations"])
    dt = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    comm.close()
    return {"metric": "local-BA iter/s, keyframe-block sharded", "value": round(its / dt, 1), "unit": "iter/s",
            "ms_per_call": round(dt / reps * 1e3, 3), "calls": reps, "scaling": "strong",
            "edges_per_rank": len(shard["edge_pt"]),
            "parallelism": f"keyframe-block shards x{world} (RCCL all-reduce of the Schur system per LM trial)",
            "note": "one problem split over the ranks; the replicas figure (`value`) runs one problem per stream"}


def gba_laps(args):
    return args.gba_kf // 500 if args.gba_laps < 0 else args.gba_laps


def bench_global_ba(args, world, rank, dist, dev):
    """Optimizer::BundleAdjustment (nIterations=10, bRobust=false, LoopClosing.cc:650) on one
    merged-map-shaped problem (SURVEY config 5, KITTI intrinsics), keyframe-block sharded over
    the N ranks: per LM trial one RCCL all-reduce of the partial Schur complement over xGMI.
    Strong scaling: the problem is fixed, N ranks share it; iter = one LM solve()."""
    import torch
    sys.path.insert(0, str(ROOT / "tests"))
    from ba_cases import global_ba_problem
    from c_orb_slam_amd.optimizer import BundleAdjustmentSharded, Comm, last_sharding, partition_points_nd, shard_problem
    pr = global_ba_problem(0, n_kf=args.gba_kf, pts_per_kf=150, laps=gba_laps(args))
    # separator-tree partition: at N > 1 each rank factors its own subtrees of the pose system
    # and only the separators' tiles and rows travel (Optimizer_partition_points_nd)
    pt_rank, kf_owner = partition_points_nd(pr, world, with_kf_owner=True)
    shard = shard_problem(pr, pt_rank, rank)
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
    used, sh_tiles, sh_rows, pattern = last_sharding()
    comm.close()
    ne = len(pr["edge_pt"])
    poses = int((kf_owner >= -1).sum())
    sharding = {"factorisation": "sharded (own subtrees + replicated separators)" if used else "replicated",
                "separator_poses": int((kf_owner == -1).sum()), "free_poses": poses,
                "rank_poses": [int((kf_owner == q).sum()) for q in range(world)],
                "exchange_doubles_per_trial": (sh_tiles * 4096 + sh_rows + 6 * poses) if used else (pattern * 4096 + 6 * poses),
                "schur_pattern_tiles": pattern, "separator_tiles": sh_tiles}
    return {"metric": "global-BA iter/s", "value": round(its / dt, 2), "unit": "iter/s", "sharding": sharding,
            "ms_per_call": round(dt / args.gba_reps * 1e3, 3), "edges_per_s": round(its * ne / dt, 1),
            "scaling": "strong", "calls": args.gba_reps,
            "config": {"workload": "kitti_merged_map_global_ba (SURVEY config 5): loop-closed map, "
                                   f"{gba_laps(args)} laps of one circuit, 5% of the points covisible across laps",
                       "keyframes": args.gba_kf, "laps": gba_laps(args),
                       "points": len(pr["pt_id"]), "edges": ne, "edges_per_rank": len(shard["edge_pt"]),
                       "lm": "optimize(10), bRobust=false", "parallelism": f"keyframe-block shards x{world} (RCCL)"},
            "dtype": "f64 (f32 I/O)"}


# concurrent LocalBundleAdjustment streams of the local-BA throughput figure (ORBGPU_LBA_STREAMS
# overrides: rocprofv3 7.0's kernel-trace callbacks have crashed twice inside a memcpy under 16
# host threads launching at once, never without the profiler; profile runs use 1)
LOCAL_BA_STREAMS = int(os.environ.get("ORBGPU_LBA_STREAMS", "16"))
RANSAC_PROBLEMS, RANSAC_HYP = 100, 300
PNP_BYTES_PER_PAIR = 24   # p3d 12 B + p2d 8 B + maxErr 4 B read per (hypothesis, correspondence)
SIM3_BYTES_PER_PAIR = 48  # X1, X2 24 B + p1, p2 16 B + two maxErr 8 B


def bench_ransac(reps=5, cpu=True, cpu_budget_s=8.0):
    """SURVEY config 3: batched RANSAC hypothesis scoring.  EPnP (PnPsolver::iterate,
    PnPsolver.cc:165-339) over 100 relocalization-shaped problems x 300 hypotheses per call for
    N in {50, 150, 500}, and Sim3Solver::iterate (Sim3Solver.cc:180-224) over 100 loop
    candidates x 300 hypotheses.  minInliers = N, so no hypothesis reaches the acceptance test:
    every draw is solved and scored on both sides, the reference loop's full 300 iterations
    (no early exit).  One call = one PnPsolver_iterate_batch; device time = the two hypothesis
    launches (solve, CheckInliers) by HIP events on the batch stream."""
    import ctypes as C
    sys.path.insert(0, str(ROOT / "tests"))
    from c_orb_slam_amd._lib import check, lib
    from c_orb_slam_amd.ransac import BatchCall, PnPsolver, Rng, Sim3Solver, iterate_batch, sim3_iterate_batch
    from pnp_cases import pnp_problem
    from sim3_cases import sim3_problem
    L = lib()
    check(L.PnPsolver_enable_timing(1), "PnPsolver_enable_timing")
    check(L.Sim3Solver_enable_timing(1), "Sim3Solver_enable_timing")
    ms2 = (C.c_float * 2)()
    cnt2 = (C.c_longlong * 2)()

    def run(kind, make, batch_fn, timings_fn, bytes_per_pair, reset=None):
        solvers = make()
        rngs = [Rng(1 + k) for k in range(len(solvers))]
        batch_fn(solvers, RANSAC_HYP, rngs)   # warm-up: allocations, upload
        call = BatchCall(kind, solvers, RANSAC_HYP, rngs)
        walls, pywalls, solve, chk = [], [], [], []
        for rep in range(2 * reps):
            if reset:
                reset(solvers)
            # even reps: the C-ABI call alone (the drop-in boundary: argument arrays kept by the
            # caller, results in its buffers); odd reps: the Python wrapper around it
            t0 = time.perf_counter()
            if rep % 2 == 0:
                call()
            else:
                batch_fn(solvers, RANSAC_HYP, rngs)
            (walls if rep % 2 == 0 else pywalls).append(time.perf_counter() - t0)
            check(timings_fn(ms2, cnt2), "last_timings")
            solve.append(ms2[0])
            chk.append(ms2[1])
        hyp, pairs = int(cnt2[0]), int(cnt2[1])
        dev_ms = float(np.mean(solve)) + float(np.mean(chk))
        c_ms = float(np.mean(chk))
        ach = pairs * (bytes_per_pair + 1 / 8) / (c_ms * 1e-3) / 1e9
        wall = float(np.median(walls))
        return {"hypotheses_per_call": hyp, "pairs_per_call": pairs,
                "device_hyp_per_s": round(hyp / (dev_ms * 1e-3), 1),
                "wall_hyp_per_s": round(hyp / wall, 1),
                "wall_over_device": round(dev_ms * 1e-3 / wall, 3),
                "ms_solve": round(float(np.mean(solve)), 4), "ms_check": round(c_ms, 4),
                "ms_call_wall": round(wall * 1e3, 3),
                "ms_call_wall_python": round(float(np.median(pywalls)) * 1e3, 3),
                "check_roofline": {"bound": "hbm", "achieved": round(ach, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                   "frac": round(ach / HBM_PEAK_GBS, 5),
                                   "alg_bytes_per_pair": bytes_per_pair + 1 / 8,
                                   "note": "algorithmic bytes (every hypothesis reads every correspondence, writes "
                                           "1 bit); the kernel stages a solver's correspondences in LDS once per "
                                           "16 hypotheses, so its HBM traffic is ~1/16 of this"}}

    out = {"workload": f"SURVEY config 3: {RANSAC_PROBLEMS} problems x {RANSAC_HYP} hypotheses per call, "
                       "minInliers = N (no early exit)", "pnp": {}, "sim3": {}}
    pnp_sets = {}
    for N in (50, 150, 500):
        prs = [pnp_problem(1000 + s, N) for s in range(RANSAC_PROBLEMS)]
        pnp_sets[N] = prs

        def make(prs=prs, N=N):
            ss = []
            for pr in prs:
                s = PnPsolver(pr["p3d"], pr["p2d"], pr["sigma2"], pr["kp_idx"], pr["n_matches"], *pr["K"])
                s.SetRansacParameters(0.99, N, RANSAC_HYP, 4, 0.4, 5.991)
                ss.append(s)
            return ss
        out["pnp"][str(N)] = run("pnp", make, iterate_batch, L.PnPsolver_last_timings, PNP_BYTES_PER_PAIR)
    # Sim3Solver's loop runs while BOTH mnIterations < mRansacMaxIts and the call's budget hold
    # (Sim3Solver.cc:197), so mRansacMaxIts must reach 300: minInliers = 0.24 N gives
    # ceil(log(0.01) / log(1 - 0.24^3)) = 331 -> 300; 90% outliers keep every hypothesis below it
    N3 = 150
    min3 = int(0.24 * N3)
    s3 = [sim3_problem(2000 + s, N3, outlier_frac=0.9) for s in range(RANSAC_PROBLEMS)]

    def make3():
        ss = []
        for pr in s3:
            s = Sim3Solver(pr["X1"], pr["X2"], pr["s1"], pr["s2"], pr["idx1"], pr["N1"], pr["K1"], pr["K2"], pr["fix"])
            s.SetRansacParameters(0.99, min3, RANSAC_HYP)
            ss.append(s)
        return ss

    def reset3(ss):   # SetRansacParameters restarts mnIterations
        for s in ss:
            s.SetRansacParameters(0.99, min3, RANSAC_HYP)
    out["sim3"][str(N3)] = run("sim3", make3, sim3_iterate_batch, L.Sim3Solver_last_timings, SIM3_BYTES_PER_PAIR, reset3)
    out["sim3"][str(N3)]["min_inliers"] = min3
    check(L.PnPsolver_enable_timing(0), "PnPsolver_enable_timing")
    check(L.Sim3Solver_enable_timing(0), "Sim3Solver_enable_timing")
    out["_cpu_args"] = (pnp_sets, s3, N3, min3)
    if cpu:
        ransac_cpu_into(out, cpu_budget_s)
    return out


def ransac_cpu_into(out, budget_s):
    """The RANSAC leg's CPU baseline on the leg's own problems, and the per-N speedups."""
    pnp_sets, s3, N3, min3 = out.pop("_cpu_args")
    out["cpu_baseline"] = ransac_cpu_baseline(pnp_sets, s3, N3, min3, budget_s)
    for kind in ("pnp", "sim3"):
        for N, r in out[kind].items():
            c = out["cpu_baseline"][kind].get(N)
            if c:
                r["speedup_vs_cpu_all_core"] = round(r["wall_hyp_per_s"] / c["hyp_per_s"], 1)


def ransac_cpu_baseline(pnp_sets, s3, N3, min3, budget_s):
    """Oracle PnPsolver / Sim3Solver iterate(300) with the same parameters on the same problems
    (full 300 hypotheses each): P independent threads, each taking whole problems, bounded to
    ~budget_s per configuration."""
    sys.path.insert(0, str(ROOT / "tests"))
    import oracle_lib
    flags = timing_oracle()
    P, aff, quota = cpu_share()
    out = {"pnp": {}, "cores": P, "kind": "port"}

    def timed(fn, n_items):
        # one item on one thread sizes the sample, then P threads take items round-robin
        t0 = time.perf_counter()
        fn(0)
        one = time.perf_counter() - t0
        n = int(min(20 * n_items, max(P, budget_s / max(one, 1e-6) * P / 3)))
        res, wall = _streams(P, lambda i: [fn(j) for j in range(i, n, P)])
        return n, wall, one

    for N, prs in pnp_sets.items():
        def fn(j, prs=prs, N=N):
            pr = prs[j % len(prs)]
            o = oracle_lib.OraclePnP(pr["p3d"], pr["p2d"], pr["sigma2"], pr["kp_idx"], pr["n_matches"], *pr["K"])
            o.set_ransac(0.99, N, RANSAC_HYP, 4, 0.4, 5.991)
            o.iterate(RANSAC_HYP, oracle_lib.new_rng(1 + j))
        n, wall, one = timed(fn, len(prs))
        out["pnp"][str(N)] = {"hyp_per_s": round(n * RANSAC_HYP / wall, 1), "problems": n, "seconds": round(wall, 2),
                              "single_thread_hyp_per_s": round(RANSAC_HYP / one, 1)}

    def fn3(j):
        pr = s3[j % len(s3)]
        o = oracle_lib.OracleSim3(pr["X1"], pr["X2"], pr["s1"], pr["s2"], pr["idx1"], pr["N1"], pr["K1"], pr["K2"],
                                  pr["fix"])
        o.set_ransac(0.99, min3, RANSAC_HYP)
        o.iterate(RANSAC_HYP, oracle_lib.new_rng(1 + j))
    n, wall, one = timed(fn3, len(s3))
    out["sim3"] = {str(N3): {"hyp_per_s": round(n * RANSAC_HYP / wall, 1), "problems": n, "seconds": round(wall, 2),
                             "single_thread_hyp_per_s": round(RANSAC_HYP / one, 1)}}
    out["sample"] = (f"oracle/pnp.c + sim3.c {flags}, {P} threads ({_cpu_model()}; affinity {aff}, cgroup quota "
                     f"{quota}); each problem a fresh solver, iterate({RANSAC_HYP}) = {RANSAC_HYP} hypotheses")
    return out


_ORACLE_TIMING = {}


def timing_oracle():
    """The oracle as SURVEY §8d times it: a separate build with the reference's own flags
    (CMakeLists.txt:10-11: -O3 -march=native, FP contraction allowed), compiled on this host at
    run time (-march=native must see the CPU that runs it); the -ffp-contract=off -O2 build stays
    the parity oracle.  Loads it into tests/oracle_lib and returns the flags used."""
    if _ORACLE_TIMING:
        return _ORACLE_TIMING["flags"]
    import subprocess
    import tempfile
    sys.path.insert(0, str(ROOT / "tests"))
    import oracle_lib
    src = ROOT / "oracle"
    out = Path(tempfile.gettempdir()) / f"liborb_oracle_timing_{os.getpid()}.so"
    flags = ["-O3", "-march=native", "-std=gnu11", "-fPIC"]
    srcs = [str(src / f) for f in ("ocv_semantics.c", "orb_extract.c", "orb_match.c", "rng.c", "linalg.c", "pnp.c",
                                   "sim3.c", "ba.c", "stereo.c", "matchers2.c", "matchers3.c", "dbow2.c",
                                   "ordering.c")]
    try:
        subprocess.run(["gcc"] + flags + ["-shared", "-o", str(out)] + srcs + ["-lm"], check=True,
                       capture_output=True, timeout=300)
        oracle_lib.use_library(out)
        _ORACLE_TIMING["flags"] = " ".join(flags)
    except Exception as e:  # noqa: BLE001 -- fall back to the parity build, say so
        _ORACLE_TIMING["flags"] = f"-O2 -ffp-contract=off (timing build failed: {type(e).__name__})"
    return _ORACLE_TIMING["flags"]


def cpu_share():
    """Host cores this process may use: the affinity set, capped by a cgroup CPU quota (a GPU
    box shares its host; nproc shows the whole machine)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) / int(per)))
    except (OSError, ValueError):
        pass
    return (min(n, quota) if quota else n), n, quota


def _streams(P, fn):
    """Run fn(i) on P threads at once (the oracle's C calls release the GIL); wall of the slowest."""
    from concurrent.futures import ThreadPoolExecutor
    t0 = time.perf_counter()
    with ThreadPoolExecutor(P) as ex:
        res = list(ex.map(fn, range(P)))
    return res, time.perf_counter() - t0


def gba_cpu_baseline(n_kf, laps, n_its=10):
    """Oracle BundleAdjustment(nIterations=n_its, bRobust=false) on the same config-5 problem: one
    call per stream, P independent streams (all-core) and the single stream alongside.  Rate =
    LM iterations (solve() calls) per second including the per-call set-up, with the GPU leg's
    nIterations (10, LoopClosing.cc:650) so both spread their set-up over the same iterations."""
    sys.path.insert(0, str(ROOT / "tests"))
    import oracle_lib
    from ba_cases import global_ba_problem
    flags = timing_oracle()
    pr = global_ba_problem(0, n_kf=n_kf, pts_per_kf=150, laps=laps)
    t0 = time.perf_counter()
    o = oracle_lib.oracle_global_ba(pr, n_its, False)
    dt1 = time.perf_counter() - t0
    P, aff, quota = cpu_share()
    # one full call per stream on every core of the share (memory per stream ~ the problem's:
    # ~1 GB at 2k keyframes, within the box's host budget at 16 streams)
    res, wall = _streams(P, lambda i: oracle_lib.oracle_global_ba(pr, n_its, False)["iterations"][0])
    return {"value": round(sum(res) / wall, 3), "unit": "iter/s", "cores": P, "kind": "port",
            "sample": f"{P} independent oracle BundleAdjustment(nIterations={n_its}) calls on the same config-5 "
                      f"problem ({n_kf} KFs, {laps} laps) on {P} threads ({_cpu_model()}; affinity {aff}, cgroup quota {quota}), "
                      f"oracle/ba.c {flags} (sparse Schur, nested-dissection block-sparse LDL^T); {sum(res)} LM solves in {wall:.1f} s",
            "single_thread": {"value": round(o["iterations"][0] / dt1, 3), "unit": "iter/s", "cores": 1,
                              "sample": f"one full call, {o['iterations'][0]} LM solves in {dt1:.1f} s"}}


def ba_cpu_baseline(budget_s):
    """Oracle LocalBundleAdjustment on the same config-4 problem: P independent streams of whole
    calls (all-core) and one stream alongside."""
    sys.path.insert(0, str(ROOT / "tests"))
    import oracle_lib
    from ba_cases import ba_problem
    flags = timing_oracle()
    pr = ba_problem(0)

    def stream(i, budget):
        t0 = time.perf_counter()
        its = calls = 0
        while True:
            o = oracle_lib.oracle_local_ba(pr)
            its += sum(o["iterations"])
            calls += 1
            if time.perf_counter() - t0 > budget and calls >= 2:
                return its, calls, time.perf_counter() - t0

    its1, calls1, dt1 = stream(0, budget_s / 2)
    P, aff, quota = cpu_share()
    res, wall = _streams(P, lambda i: stream(i, budget_s / 2))
    its = sum(r[0] for r in res)
    calls = sum(r[1] for r in res)
    return {"value": round(its / max(r[2] for r in res), 2), "unit": "iter/s", "cores": P, "kind": "port",
            "sample": f"{P} independent streams of LocalBundleAdjustment calls on config 4 on {P} threads "
                      f"({_cpu_model()}; affinity {aff}, cgroup quota {quota}): {calls} calls, {its} LM solves; "
                      f"oracle/ba.c {flags}",
            "single_thread": {"value": round(its1 / dt1, 2), "unit": "iter/s", "cores": 1,
                              "sample": f"{calls1} calls ({its1} LM solves) on 1 thread"}}


class _CpuStream:
    """One reference-structured CPU tracking stream on the oracle (line-faithful C restatement):
    per stereo frame extract L and R, ComputeStereoMatches, TrackWithMotionModel (UnprojectStereo,
    SearchByProjection(Cur, Last, 7), PoseOptimization) and TrackLocalMap (isInFrustum +
    SearchByProjection(F, local map, 1) + PoseOptimization) over the map points of the last
    K_LOCAL frames -- the GPU step's work.  The oracle's C calls release the GIL, so streams run
    on separate cores."""

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
        self.lsf = np.float32(np.log(np.float32(1.2)))
        self.synthetic = synthetic
        Tabs = [np.eye(4, dtype=np.float32)]
        for R in Rs:
            Tabs.append(synthetic.pose_from_rotation(np.asarray(R, np.float64) @ Tabs[-1][:3, :3].astype(np.float64)))
        self.Tabs = Tabs
        self.hist = []   # the last K_LOCAL frames: (keys, desc, depth, map point block)
        self.t = {"extract": 0.0, "stereo": 0.0, "match": 0.0, "pose": 0.0, "local_map": 0.0}
        self.done = 0

    def _block(self, k, d, dep, i):
        """UnprojectStereo of frame i with its absolute Twc + UpdateNormalAndDepth."""
        Twc = np.linalg.inv(self.Tabs[i]).astype(np.float32)
        X, slot = self.ol.oracle_unproject_stereo(k, dep, Twc, self.fx, self.fy, self.cx, self.cy)
        X = np.nan_to_num(X)
        PO = X - Twc[:3, 3]
        dist = np.maximum(np.linalg.norm(PO, axis=1), 1e-6).astype(np.float32)
        mx = (dist * self.scale[np.clip(k["octave"], 0, 7)]).astype(np.float32)
        return dict(pos=X, desc=d, slot=slot, normal=(PO / dist[:, None]).astype(np.float32), max_dist=mx,
                    min_dist=(mx / self.scale[7]).astype(np.float32))

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
        if i == 0:
            self.hist = []
        if self.hist:
            pk, pd, pdep = self.hist[-1][:3]
            self.hist[-1] = self.hist[-1][:3] + (self._block(pk, pd, pdep, i - 1),)   # UpdateLastFrame
            blocks = [h[3] for h in self.hist]
            off = np.cumsum([0] + [len(b["pos"]) for b in blocks])
            M = {k: np.concatenate([b[k] for b in blocks]) for k in ("pos", "desc", "normal", "max_dist", "min_dist")}
            M["obs"] = np.ones(len(M["pos"]), np.int32)
            nolm = np.concatenate([b["slot"] < 0 for b in blocks])
            last = Frame(pk, pd, self.scale, self.Tabs[i - 1], fx, fy, cx, cy, mbf, W, H)
            cur = Frame(kL, dL, self.scale, self.Tabs[i], fx, fy, cx, cy, mbf, W, H, uRight=uR)
            lm = np.where(blocks[-1]["slot"] >= 0, blocks[-1]["slot"] + off[-2], -1).astype(np.int32)
            mps = MapPoints(M["pos"], M["desc"], M["obs"])
            cm = np.full(cur.N, -1, np.int32)
            td = time.perf_counter()
            ol.oracle_search_last(cur, cm, last, pk, lm, np.zeros(len(pk), np.uint8), mps, 7.0, False, 0.9, True)
            te = time.perf_counter()
            self.t["match"] += te - td
            obs = np.stack([kL["x"], kL["y"], uR], 1).astype(np.float32)
            isg = self.isig[kL["octave"]].astype(np.float32)
            pr = dict(Tcw=cur.Tcw, has_mp=(cm >= 0).astype(np.uint8), Xw=M["pos"][np.maximum(cm, 0)], obs=obs,
                      inv_sigma2=isg, cam=(fx, fy, cx, cy, mbf))
            o1 = ol.oracle_pose_optimization(pr)
            tf = time.perf_counter()
            self.t["pose"] += tf - te
            # TrackLocalMap: discard outliers, skip points in the frame, SearchLocalPoints, PoseOptimization
            skip = nolm.copy()
            skip[cm[cm >= 0]] = True
            cm[o1["outlier"].astype(bool)] = -1
            M["skip"] = skip.astype(np.uint8)
            cur.Tcw = np.ascontiguousarray(o1["Tcw"], np.float32)
            ol.oracle_search_local_points(cur, cm, M, self.lsf, 1.0, 0.8)
            pr2 = dict(Tcw=cur.Tcw, has_mp=(cm >= 0).astype(np.uint8), Xw=M["pos"][np.maximum(cm, 0)], obs=obs,
                       inv_sigma2=isg, cam=(fx, fy, cx, cy, mbf))
            ol.oracle_pose_optimization(pr2)
            self.t["local_map"] += time.perf_counter() - tf
        self.hist.append((kL, dL, dep))
        self.hist = self.hist[-K_LOCAL:]
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
    (P = the cores this process may use: affinity capped by the cgroup quota) -> whole-host
    frames/s, the figure `value` reports.  Timing build of the oracle (-O3 -march=native)."""
    flags = timing_oracle()
    one = _CpuStream(lefts, rights, Rs)
    one.run(0, budget_s / 2, 4)
    fps1 = one.done / sum(one.t.values())
    P, aff, quota = cpu_share()
    streams = [_CpuStream(lefts, rights, Rs) for _ in range(P)]
    walls, _ = _streams(P, lambda i: streams[i].run(i * 7, budget_s / 2, 2))
    framesP = sum(s.done for s in streams)
    fpsP = framesP / max(walls)
    t = one.t
    return {"value": round(fpsP, 3), "unit": "frames/s", "cores": P, "kind": "port",
            "sample": f"{P} independent reference-structured streams on {P} threads ({_cpu_model()}; affinity {aff}, "
                      f"cgroup quota {quota}): oracle ORBextractor x2 + ComputeStereoMatches + "
                      f"SearchByProjection(Cur,Last,7) + PoseOptimization + TrackLocalMap (isInFrustum + "
                      f"SearchByProjection(F, local map, 1) + PoseOptimization) per stereo frame, C restatement built "
                      f"{flags}; {framesP} frames in {max(walls):.1f} s",
            "single_thread": {"value": round(fps1, 3), "unit": "frames/s", "cores": 1,
                              "sample": f"{one.done} frames on 1 thread: extract {t['extract'] / one.done * 1e3:.1f} "
                                        f"ms/frame, stereo {t['stereo'] / one.done * 1e3:.2f} ms, match "
                                        f"{t['match'] / max(one.done - 1, 1) * 1e3:.2f} ms, pose "
                                        f"{t['pose'] / max(one.done - 1, 1) * 1e3:.2f} ms, local map "
                                        f"{t['local_map'] / max(one.done - 1, 1) * 1e3:.2f} ms"}}


if __name__ == "__main__":
    main()
