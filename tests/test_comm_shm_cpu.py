"""orbgpu_comm_init_shm on the CPU (no device needed for the group set-up): ranks as separate
processes attach to one shared-memory segment, agree on (rank, size) through its cross-process
barrier, and leave no name behind in /dev/shm; mismatched groups and a missing rank 0 fail
loudly within the bounded wait instead of hanging."""
import os
import subprocess
import sys
import uuid
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
CHILD = r"""
import sys
sys.path.insert(0, {root!r})
from c_orb_slam_amd.optimizer import Comm
name, n, r, cap = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
try:
    c = Comm.shm(name, n, r, cap)
except RuntimeError as e:
    print("ERR", e)
    sys.exit(3)
print("OK", c.rank_size)
c.close()
"""


def _spawn(name, n, r, cap, timeout_s="30"):
    env = dict(os.environ, ORBGPU_SHM_TIMEOUT=timeout_s)
    return subprocess.Popen([sys.executable, "-c", CHILD.format(root=str(ROOT)), name, str(n), str(r), str(cap)],
                            env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)


def test_shm_group_of_processes_attaches():
    for n in (2, 4):
        name = f"/orbgpu_c{uuid.uuid4().hex[:16]}"
        ps = [_spawn(name, n, r, 1024) for r in range(n)]
        outs = [p.communicate(timeout=120)[0] for p in ps]
        for r, (p, out) in enumerate(zip(ps, outs)):
            assert p.returncode == 0, out
            assert f"OK ({r}, {n})" in out, out
        assert not os.path.exists("/dev/shm" + name)   # unlinked once every rank attached


def test_shm_group_disagreement_fails():
    name = f"/orbgpu_c{uuid.uuid4().hex[:16]}"
    ps = [_spawn(name, 2, 0, 1024, "5"), _spawn(name, 2, 1, 2048, "5")]   # different slot sizes
    outs = [p.communicate(timeout=120)[0] for p in ps]
    assert ps[1].returncode == 3 and "ERR" in outs[1], outs
    assert ps[0].returncode == 3, outs          # rank 0 times out waiting for its peer
    if os.path.exists("/dev/shm" + name):
        os.unlink("/dev/shm" + name)


def test_shm_missing_rank0_times_out():
    name = f"/orbgpu_c{uuid.uuid4().hex[:16]}"
    p = _spawn(name, 2, 1, 1024, "2")
    out = p.communicate(timeout=60)[0]
    assert p.returncode == 3 and "ERR" in out, out
