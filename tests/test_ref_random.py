"""CPU: the RANSAC sample stream pinned to the reference's own code.

`oracle/ref/Makefile` compiles the reference's DUtils::Random and DUtils::Timestamp
(/root/reference/Thirdparty/DBoW2/DUtils/Random.cpp, Timestamp.cpp: libc only) from the
reference sources into oracle/_ref/libdutils_ref.so.  These tests draw RandomInt streams
from it and check them against
  - the product library's orb_rng (the explicit stream the C ABI takes, include/orbslam_gpu.h),
  - the oracle's ora_rng_random_int,
  - the oracle's PnPsolver::iterate / Sim3Solver::iterate draw consumption (the RNG stream
    position after each call, which the GPU tests in turn hold the device solvers to).
Only this piece of the hot path can be built from the reference here; everything else needs
OpenCV or Eigen and stays "parity unpinned" (DESIGN.md §4).
"""
import ctypes as C
import subprocess
from pathlib import Path

import numpy as np
import pytest

import oracle_lib
from oracle_lib import lib as oracle

ROOT = Path(__file__).resolve().parents[1]
REF_SO = ROOT / "oracle" / "_ref" / "libdutils_ref.so"
REF_SRC = Path("/root/reference/Thirdparty/DBoW2/DUtils/Random.cpp")


def ref_lib():
    if REF_SRC.exists():   # the recipe rebuilds it when the reference sources are present
        subprocess.run(["make", "-s", "-C", str(ROOT / "oracle" / "ref")], check=True)
    if not REF_SO.exists():
        pytest.skip("oracle/_ref/libdutils_ref.so not built and /root/reference absent")
    L = C.CDLL(str(REF_SO))
    L.ref_seed_rand.argtypes = [C.c_int]
    L.ref_seed_rand_once.argtypes = [C.c_int]
    L.ref_random_int.argtypes = [C.c_int, C.c_int]
    L.ref_random_int.restype = C.c_int
    L.ref_libc_rand.restype = C.c_int
    return L


def product_rng(seed):
    from c_orb_slam_amd._lib import lib, orb_rng
    g = orb_rng()
    lib().orb_rng_seed(C.byref(g), seed)
    return g, (lambda: lib().orb_rng_rand(C.byref(g)))


def random_int_from(rand, mn, mx):
    """Random.cpp:47-50 on a rand() value (the formula the product's host replay uses)."""
    return int((rand() / (2147483647 + 1.0)) * (mx - mn + 1)) + mn


def pnp_pattern(N, iters, min_set=4):
    """(min, max) of every RandomInt call of `iters` PnPsolver::iterate passes (PnPsolver.cc:
    189-201: vAvailableIndices reset per pass, swap-remove after each draw)."""
    return [(0, N - 1 - i) for _ in range(iters) for i in range(min_set)]


@pytest.mark.parametrize("seeding", ["SeedRand(1)", "SeedRandOnce(0)", "SeedRand(12345)"])
def test_reference_random_int_equals_orb_rng_and_oracle(seeding):
    R = ref_lib()
    seed = {"SeedRand(1)": 1, "SeedRandOnce(0)": 0, "SeedRand(12345)": 12345}[seeding]
    if seeding.startswith("SeedRandOnce"):
        R.ref_seed_rand_once(seed)   # Initializer.cc:80; glibc maps srand(0) to seed 1
        R.ref_seed_rand(seed)        # SeedRandOnce latches after its first call: reseed explicitly
    else:
        R.ref_seed_rand(seed)
    _, prand = product_rng(seed)
    og = oracle_lib.new_rng(seed)
    O = oracle()
    pattern = pnp_pattern(500, 300) + [(0, 149 - i) for _ in range(300) for i in range(3)] + \
        [(3, 3 + k % 17) for k in range(500)]
    for mn, mx in pattern:
        r = R.ref_random_int(mn, mx)
        assert r == random_int_from(prand, mn, mx)
        assert r == O.ora_rng_random_int(og, mn, mx)
    # the three streams end at the same position
    nxt = R.ref_libc_rand()
    assert nxt == prand() == O.ora_rng_rand(og)


def test_seed_rand_once_latches():
    """SeedRandOnce(seed) seeds only on its first call (Random.cpp:38-45)."""
    R = ref_lib()
    R.ref_seed_rand_once(0)
    R.ref_seed_rand(7)
    R.ref_seed_rand_once(0)   # latched (by this or an earlier call): no reseed
    _, prand = product_rng(7)
    for _ in range(50):
        assert R.ref_libc_rand() == prand()


@pytest.mark.parametrize("N,min_inl,n_it", [(50, 50, 5), (150, 10, 5), (150, 150, 300), (500, 500, 7)])
def test_oracle_pnp_draw_stream_matches_reference(N, min_inl, n_it):
    """The oracle's PnPsolver::iterate (PnPsolver.cc:165-258) consumes exactly the reference's
    RandomInt calls: 4 per pass over the passes it ran, early Refine return included."""
    from pnp_cases import pnp_problem
    R = ref_lib()
    pr = pnp_problem(11 + N, N)
    s = oracle_lib.OraclePnP(pr["p3d"], pr["p2d"], pr["sigma2"], pr["kp_idx"], pr["n_matches"], *pr["K"])
    s.set_ransac(0.99, min_inl, 300, 4, 0.5, 5.991)
    og = oracle_lib.new_rng(1)
    R.ref_seed_rand(1)
    before = 0
    for _ in range(3):
        s.iterate(n_it, og)
        ran = s.iterations - before
        before = s.iterations
        # replay the passes this call ran on the reference stream; compare positions
        for mn, mx in pnp_pattern(N, ran):
            R.ref_random_int(mn, mx)
        a, b = R.ref_libc_rand(), oracle().ora_rng_rand(og)
        assert a == b, (N, min_inl, ran)


@pytest.mark.parametrize("N,min_inl", [(60, 20), (150, 150)])
def test_oracle_sim3_draw_stream_matches_reference(N, min_inl):
    """Sim3Solver::iterate (Sim3Solver.cc:140-207): 3 RandomInt calls per pass, the `&&` loop."""
    from sim3_cases import sim3_problem
    R = ref_lib()
    pr = sim3_problem(21 + N, N)
    s = oracle_lib.OracleSim3(pr["X1"], pr["X2"], pr["s1"], pr["s2"], pr["idx1"], pr["N1"], pr["K1"], pr["K2"],
                              pr["fix"])
    s.set_ransac(0.99, min_inl, 300)
    og = oracle_lib.new_rng(1)
    R.ref_seed_rand(1)
    before = 0
    for _ in range(3):
        s.iterate(5, og)
        ran = s.iterations - before
        before = s.iterations
        for mn, mx in pnp_pattern(N, ran, 3):
            R.ref_random_int(mn, mx)
        assert R.ref_libc_rand() == oracle().ora_rng_rand(og), (N, min_inl, ran)
