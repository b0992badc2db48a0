#!/usr/bin/env python3
"""Per-iteration time of the even-odd CG (sm_eo_cg, tol 0) for fused-Dhat chunk heights.

    python tools/tune_eo.py [--n 1024] [--xchunk 2,4,8,16] [--iters 200] [--modes six,folded,twodir]

Host-pointer API: the timing includes the upload of phi and the download of
x (subtract, or compare variants at equal --iters).
"""
import argparse
import ctypes
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1024)
    ap.add_argument("--xchunk", default="0,2,4,8,16")
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--modes", default="folded",
                    help="comma list: six (six-launch CG), folded (2 passes), twodir (one pass, sm_eotd.hip)")
    a = ap.parse_args()
    import numpy as np
    import schwingermodel_amd as sm
    N = a.n
    S = N * N
    U, phi = np.empty(4 * S), np.empty(4 * S)
    sm.lib.sm_fill_gauge(4321, 0.3246, N, 0, N, 0, N, U.ctypes.data, U[2 * S:].ctypes.data)
    sm.lib.sm_fill_spinor(91011, N, 0, N, 0, N, phi.ctypes.data, phi[2 * S:].ctypes.data)
    x = np.empty(4 * S)
    env = {"six": {}, "folded": {"SM_EO_CG_FOLDED": "1"}, "twodir": {"SM_EO_CG_TD": "1"}}
    for xc, mode in [(int(v), m) for v in a.xchunk.split(",") for m in a.modes.split(",")]:
        xkey = "SM_EOTD_XCHUNK" if mode == "twodir" else "SM_EO_XCHUNK"
        if xc > 0:
            os.environ[xkey] = str(xc)   # read per solve: kept set for the solves
        for k, v in env[mode].items():
            os.environ[k] = v
        L = sm.Lattice(N, N)
        for k in env[mode]:
            os.environ.pop(k, None)
        sm.check(sm.lib.sm_upload_gauge(L.ctx, U.ctypes.data, U[2 * S:].ctypes.data))
        res = sm.CGResult()
        best = None
        for _ in range(3):
            t = time.perf_counter()
            sm.check(sm.lib.sm_eo_cg(L.ctx, phi.ctypes.data, phi[2 * S:].ctypes.data, x.ctypes.data,
                                     x[2 * S:].ctypes.data, -0.10, 0.0, a.iters, ctypes.byref(res)))
            dt = time.perf_counter() - t
            best = dt if best is None else min(best, dt)
        L.close()
        os.environ.pop(xkey, None)
        print(json.dumps({"n": N, "xchunk": xc, "mode": mode, "iters": res.iterations,
                          "ms_per_it": round(1e3 * best / a.iters, 4)}), flush=True)


if __name__ == "__main__":
    main()
