#!/usr/bin/env python3
"""Drift of the link codes' ulp offsets k under the HMC's link update.

The recompute-Ad CG pass reads every link as its smaller component v plus a
flag word holding k, the offset in ulps of the larger component |w| from the
decoder's root sqrt(1 - v^2) (csrc/sm_linkcode.h). The reference's leapfrog
multiplies U by exp(i eps P) every MD step without re-unitarising
(src/hmc.cpp:70-100), so |U| walks away from 1 and |k| grows. This tool runs
sm_quenched_trajectory (HMC::Leapfrog with the gauge force, 10 MD steps) on
the config-3 field (4096^2, sigma 0.2374, beta 5) and, after each of the
requested trajectory counts, downloads U and histograms k computed on the
host with a correctly rounded sqrt(1 - v*v) (the device's root is within one
ulp of it, so each k is exact to +-1), plus the device's own check
(sm_link_code_check: links not encodable at all).

    python tools/link_drift.py [--nx 4096] [--nt 4096] [--at 0,50,500]
One JSON line per count: max |k|, the fraction of links inside each packed
range ([-2, 1] nibbles, 6-bit, 8-bit, 10-bit), and a coarse histogram.
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def offsets(U):
    """k for every link of U (complex128 array), host root."""
    c, s = U.real, U.imag
    cosv = np.abs(s) > np.abs(c)
    v = np.where(cosv, c, s)
    w = np.abs(np.where(cosv, s, c))
    r = np.sqrt(1.0 - v * v)
    return w.view(np.int64) - r.view(np.int64)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nx", type=int, default=4096)
    ap.add_argument("--nt", type=int, default=4096)
    ap.add_argument("--sigma", type=float, default=0.2374)
    ap.add_argument("--at", default="0,50,500")
    a = ap.parse_args()
    import torch
    import schwingermodel_amd as sm
    Nx, Nt = a.nx, a.nt
    V = Nx * Nt
    U = np.empty(4 * V)
    sm.lib.sm_fill_gauge(4321, a.sigma, Nt, 0, Nx, 0, Nt, U.ctypes.data, U[2 * V:].ctypes.data)
    dU = torch.from_numpy(U).cuda()
    L = sm.Lattice(Nx, Nt)
    sm.check(sm.lib.sm_upload_gauge_dev(L.ctx, ctypes.c_void_p(dU.data_ptr())))
    prm = sm.HMCParams(m0=-0.06, beta=5.0, tau=1.0, md_steps=10, cg_tol=1e-10, cg_max_iter=10000, seed=2024,
                       even_odd=0)
    done = 0
    for n in (int(v) for v in a.at.split(",")):
        t = time.perf_counter()
        while done < n:
            sm.check(sm.lib.sm_quenched_trajectory(L.ctx, ctypes.byref(prm), done))
            done += 1
        sm.check(sm.lib.sm_synchronize(L.ctx))
        t_md = time.perf_counter() - t
        err, bad = ctypes.c_double(-1.0), ctypes.c_long(-1)
        sm.check(sm.lib.sm_link_code_check(L.ctx, None, ctypes.byref(err), ctypes.byref(bad)))
        host = np.empty(4 * V)
        sm.check(sm.lib.sm_download_gauge(L.ctx, host.ctypes.data, host[2 * V:].ctypes.data))
        k = offsets(host.view(np.complex128))
        ak = np.abs(k)
        edges = [0, 1, 2, 4, 8, 16, 32, 64, 128, 256, 512, 1024, 8192]
        hist = {f"{lo}-{hi - 1}": int(((ak >= lo) & (ak < hi)).sum()) for lo, hi in zip(edges, edges[1:])}
        print(json.dumps({
            "lattice": f"{Nx}x{Nt}", "trajectories": n, "md_steps": 10 * n, "md_seconds": round(t_md, 3),
            "links": int(k.size), "device_not_encodable": bad.value, "device_max_decode_err": err.value,
            "max_abs_k": int(ak.max()), "rms_k": float(np.sqrt(np.mean(k.astype(np.float64) ** 2))),
            "frac_in_nibble_-2_1": float(((k >= -2) & (k <= 1)).mean()),
            "frac_in_6bit": float(((k >= -32) & (k <= 31)).mean()),
            "frac_in_8bit": float(((k >= -128) & (k <= 127)).mean()),
            "frac_in_10bit": float(((k >= -512) & (k <= 511)).mean()),
            "hist_abs_k": hist, "k_note": "host root (correctly rounded sqrt(1 - v*v)); device k within +-1"}),
            flush=True)
    L.close()


if __name__ == "__main__":
    main()
