"""bench.py's rank launcher (CPU): `--gpus N` without a launcher starts N rank processes and
n_gpus reports N; a WORLD_SIZE that contradicts --gpus is refused (bench.py)."""
import json
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def _run(args, env_extra=None):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, str(ROOT / "bench.py")] + args, env=env, capture_output=True,
                          text=True, timeout=240)


def test_gpus_flag_spawns_ranks():
    r = _run(["--gpus", "2", "--dry-run"])
    assert r.returncode == 0, r.stderr
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == 2 and line["ranks_joined"] == 2 and line["parallelism"] == "replicas2"


def test_default_is_one_rank():
    r = _run(["--dry-run"])
    assert r.returncode == 0, r.stderr
    assert json.loads(r.stdout.strip())["n_gpus"] == 1


def test_world_size_mismatch_refused():
    r = _run(["--gpus", "4", "--dry-run"], {"WORLD_SIZE": "2", "RANK": "0"})
    assert r.returncode != 0 and "WORLD_SIZE" in r.stderr


def test_failed_rank_stops_the_job():
    """A rank > 0 that dies before the rendezvous leaves rank 0 blocked in init_process_group: the
    launcher must notice, stop rank 0 and return the failing rank's code."""
    import time
    t0 = time.monotonic()
    r = _run(["--gpus", "2", "--dry-run"], {"BENCH_DRY_FAIL_RANK": "1"})
    assert r.returncode == 3, (r.returncode, r.stderr)
    assert "rank 1 exited with 3" in r.stderr
    assert time.monotonic() - t0 < 120
