#!/usr/bin/env python3
"""Config 5 (8192^2, beta=2 field, m0 = -0.19) against the reference's summary
fixture through every GPU CG path (round 4): the default recompute-Ad pass with
link codes, the same with complex links, the stored-Ad pass, and the
six-launch sequence (the reference's per-element arithmetic, dots in fixed
order). Prints iterations, sampled x and sum-of-squares relative differences,
like tests/test_gpu_large.py.

    python tools/c5_paths.py [--name l8192x8192_b2_m-0p19]
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
    ap.add_argument("--name", default="l8192x8192_b2_m-0p19")
    a = ap.parse_args()
    from test_gpu_large import fill, sample, sumsq
    import schwingermodel_amd as sm
    g = os.path.join(REPO, "tests", "golden")
    meta = json.load(open(os.path.join(g, "manifest.json")))["large"][a.name]
    with np.load(os.path.join(g, meta["file"]), allow_pickle=False) as z:
        ref = {k: z[k].copy() for k in z.files}
    N = meta["Nx"]
    S = N * N
    L = sm.init(N, N)
    U, psi, chi = sm.spinor(S), sm.spinor(S), sm.spinor(S)
    fill(sm, N, meta["sigma"], U, psi, chi)
    ref_sq = meta["fsum_sq"]["ref_cgx"]
    for label, fused, codes in (("recompute, link codes (default)", 5, 1), ("recompute, complex links", 5, 0),
                                ("stored Ad", 4, 0), ("six launches", 0, 0)):
        sm.check(sm.lib.sm_tune_cg(L.ctx, fused, 0))
        sm.check(sm.lib.sm_cg_link_angles(L.ctx, codes, None))
        x = sm.spinor(S)
        conv = sm.conjugate_gradient(U, psi, x, meta["m0"])
        xs, xr = sample(x, ref["sites"]), ref["ref_cgx"]
        print(json.dumps({"path": label, "converged": conv, "iterations": L.last_cg.iterations,
                          "reference_iterations": meta["cg_iters"],
                          "sampled_x_rel": float(np.linalg.norm(xs - xr) / np.linalg.norm(xr)),
                          "sum_x2_rel": abs(sumsq(x) - ref_sq) / ref_sq}), flush=True)
    L.close()


if __name__ == "__main__":
    main()
