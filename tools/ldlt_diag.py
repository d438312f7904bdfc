#!/usr/bin/env python3
"""Compare the tiled LDL^T factorisation (d, L) with the oracle's, tile by tile."""
import ctypes as C
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
import oracle_lib  # noqa: E402
from oracle_lib import ptr  # noqa: E402


def banded(rng, nblk, bw, loops=()):
    n = 6 * nblk
    S = np.zeros((n, n))
    for i in range(nblk):
        for j in range(i, min(nblk, i + bw + 1)):
            S[6 * i:6 * i + 6, 6 * j:6 * j + 6] = rng.normal(size=(6, 6))
    for i, j in loops:
        S[6 * i:6 * i + 6, 6 * j:6 * j + 6] = rng.normal(size=(6, 6))
    S = np.triu(S) + np.triu(S, 1).T
    S += np.diag(np.abs(S).sum(1) + 1.0)
    return S


def main():
    from c_orb_slam_amd._lib import lib
    L = oracle_lib.lib()
    L.ora_ldlt_solve.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p]
    for name, nb, loops in [("banded", 200, ()), ("loop-far", 200, [(1, 198)]), ("loop-mid", 200, [(3, 100)]),
                            ("loop-small", 40, [(1, 38)]), ("loops", 200, [(1, 198), (3, 100)])]:
        rng = np.random.default_rng(1)
        S = banded(rng, nb, 8, loops)
        n = len(S)
        A = S.copy()
        x = np.zeros(n)
        L.ora_ldlt_solve(ptr(A), n, ptr(np.zeros(n)), ptr(x))
        ora_d = np.diag(A).copy()
        ora_L = np.triu(A, 1).T    # oracle stores L^T in the strict upper triangle
        out = np.zeros((n, n))
        assert lib().orbgpu_unit_ldlt_factor(n, ptr(np.ascontiguousarray(S)), ptr(out)) == 0
        g_d = np.diag(out)
        g_L = np.tril(out, -1)
        bad_d = np.flatnonzero(g_d != ora_d)
        diff = g_L != ora_L
        print(f"{name}: n={n} d mismatches {len(bad_d)} first {bad_d[:5]}; L mismatches {diff.sum()}")
        if diff.any():
            r, c = np.nonzero(diff)
            t = sorted(set(zip(r // 64, c // 64)))
            print("   tiles (rowblk, colblk) with L mismatch:", t[:20])
            i = np.argmin(r * n + c)
            print("   first at", r[i], c[i], g_L[r[i], c[i]], ora_L[r[i], c[i]])


if __name__ == "__main__":
    main()
