#!/usr/bin/env python3
"""Spread of the GPU CG paths against each other at the BASELINE sizes.

    python tools/cg_spread.py [--n 4096] [--sigma 0.2374] [--m0 -0.06]

Solves D D^dag x = psi (tol 1e-10, x0 = psi as src/conjugate_gradient.cpp:16)
with the default recompute-Ad pass (fused multiply-adds, link angles from 4M
sites), the same pass without the angles, the stored-Ad pass and the six-launch
reference sequence (per-element arithmetic bitwise the reference's; only the
dots' summation order differs), and prints iterations and ||x - x_six|| /
||x_six|| for each: the reduction-order / rounding band the reference fixture
comparison (tests/test_gpu_large.py) sits in.
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=4096)
    ap.add_argument("--sigma", type=float, default=0.2374)
    ap.add_argument("--m0", type=float, default=-0.06)
    a = ap.parse_args()
    import schwingermodel_amd as sm
    from dist_worker import fill_block
    N, S = a.n, a.n * a.n
    f = fill_block(sm, N, N, 0, N, a.sigma, nthreads=16)
    P = lambda x: ctypes.c_void_p(x.ctypes.data)  # noqa: E731
    L = sm.Lattice(N, N)
    sm.check(sm.lib.sm_upload_gauge(L.ctx, P(f["U"]), P(f["U"][2 * S:])))
    sols = {}
    for name, mode, ang in (("six", 0, 0), ("recompute", 5, 1), ("recompute_noang", 5, 0), ("stored", 4, 0)):
        sm.check(sm.lib.sm_tune_cg(L.ctx, mode, 0))
        sm.check(sm.lib.sm_cg_link_angles(L.ctx, ang, None))
        x = np.empty(4 * S)
        res = sm.CGResult()
        sm.check(sm.lib.sm_cg(L.ctx, P(f["psi"]), P(f["psi"][2 * S:]), P(x), P(x[2 * S:]), a.m0, 1e-10, 20000,
                              ctypes.byref(res)))
        used = ctypes.c_int()
        sm.check(sm.lib.sm_cg_link_angles(L.ctx, -1, ctypes.byref(used)))
        sols[name] = (x, res.iterations, res.converged, used.value)
    L.close()
    x0 = sols["six"][0]
    for name, (x, it, conv, used) in sols.items():
        print(json.dumps({"N": N, "m0": a.m0, "path": name, "iterations": it, "converged": conv,
                          "angles_in_use": used,
                          "x_rel_to_six": float(np.linalg.norm(x - x0) / np.linalg.norm(x0))}), flush=True)


if __name__ == "__main__":
    main()
