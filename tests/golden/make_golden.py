"""Generate the golden extraction fixtures (run in the build container).

Inputs are regenerated from the seed by c_orb_slam_amd.synthetic (their
SHA-256 is stored so generator drift is detected); expected outputs are the
CPU oracle's keypoints and descriptors.  The reference itself cannot be run
here (no OpenCV/Eigen), so these pin the oracle against regressions, not
against the reference ("parity unpinned" at the OpenCV boundary).
"""
import hashlib
import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parents[1]))
sys.path.insert(0, str(HERE.parent))

from c_orb_slam_amd import synthetic  # noqa: E402
import oracle_lib  # noqa: E402

CASES = [  # name, seed, w, h, nfeatures (KITTI stereo yaml: 2000; metric: 1200; EuRoC 1200; TUM1 1000)
    ("kitti_1200", 100, 1241, 376, 1200),
    ("kitti_2000", 101, 1241, 376, 2000),
    ("euroc_1200", 102, 752, 480, 1200),
    ("tum_1000", 103, 640, 480, 1000),
]


def image_for(seed, w, h):
    frames, _ = synthetic.sequence(seed, 1, w, h)
    return frames[0]


def main():
    for name, seed, w, h, nf in CASES:
        img = image_for(seed, w, h)
        k, d = oracle_lib.OracleExtractor(nf, 1.2, 8, 20, 7)(img)
        np.savez_compressed(HERE / f"extract_{name}.npz", seed=seed, w=w, h=h, nfeatures=nf,
                            sha256=hashlib.sha256(img.tobytes()).hexdigest(), kps=k.view(np.uint8).reshape(-1, 28),
                            desc=d)
        print(name, len(k))


if __name__ == "__main__":
    main()
