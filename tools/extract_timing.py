"""Stage timings of ONE extractor on a batch of KITTI-shaped images (no concurrent stream)."""
import sys
import time

sys.path.insert(0, ".")
import numpy as np  # noqa: E402
import torch  # noqa: E402

import c_orb_slam_amd as orb  # noqa: E402
from c_orb_slam_amd import synthetic  # noqa: E402

W, H, B = 1241, 376, int(sys.argv[1]) if len(sys.argv) > 1 else 64
dev = torch.device("cuda", 0)
lefts, rights, Hs, Rs = synthetic.stereo_sequence(1000, B, W, H, return_rotations=True)
ex = orb.ORBextractor(1200, 1.2, 8, 20, 7, max_width=W, max_height=H, max_batch=B)
d_L = torch.from_numpy(lefts).to(dev)
cap = 2 * 1200 + 64
d_kps = torch.empty((B, cap, 7), dtype=torch.int32, device=dev)
d_desc = torch.empty((B, cap, 32), dtype=torch.uint8, device=dev)
acc = {}
for it in range(13):
    torch.cuda.synchronize()
    t = time.perf_counter()
    ex.extract_device(d_L.data_ptr(), B, W, H, W, W * H, d_kps.data_ptr(), d_desc.data_ptr(), cap)
    wall = (time.perf_counter() - t) * 1e3
    if it >= 3:
        for k, v in ex.last_timings().items():
            acc[k] = acc.get(k, 0) + v / 10
        acc["wall"] = acc.get("wall", 0) + wall / 10
print({k: round(v, 4) for k, v in acc.items()}, flush=True)

if __import__("os").environ.get("ORBGPU_PROF_DUMP"):
    import ctypes as C
    from c_orb_slam_amd._lib import lib
    buf = (C.c_ulonglong * 32)()
    lib().orbgpu_debug_prof_extract(buf)
    print("k_fast_cells sections (cycles, cell 0 of image 0, 13 calls):", list(buf)[:6], flush=True)
    names = ["init", "phase1", "p2_setup", "p2_sort", "p2_partition", "p2_serial", "p2_final", "p1_best"]
    print("k_octree sections (cycles per call, job 0 = image 0 level 0):",
          {n: round(buf[16 + i] / 13) for i, n in enumerate(names)},
          "phase-2 rounds", round(buf[24] / 13, 1), "phase-1 rounds", round(buf[25] / 13, 1), flush=True)
    print("k_octree jobs: slowest", buf[26] >> 4, "cycles (level", buf[26] & 15, "), mean",
          round(buf[27] / max(buf[28], 1)), "cycles over", buf[28], "jobs", flush=True)
