#!/usr/bin/env python3
"""CPU prototype (numpy over the oracle's bitwise-reference DD^dag) of CG
recurrences that move fewer bytes per iteration, against the reference's CG
(src/conjugate_gradient.cpp:4-66). Test infrastructure, not product code.

  ref      the reference sequence: r -= alpha Ad, beta = |r_new|^2 / |r_old|^2
  onepass  the GPU one-pass recurrence (sm_cgfused.hip): r_j formed on load,
           beta_j from the pass's own dots (expansion of |r_j - alpha Ad_j|^2)
  rless    onepass without an r vector: r_j = d_j - beta_{j-1} d_{j-1}
           rebuilt from the two stored directions, so a pass reads d_j,
           d_{j-1}, Ad_j and writes d_{j+1}, Ad_{j+1} (no r traffic), and x
           takes two updates every other pass (x + a_{j-1} d_{j-1}) + a_j d_j.

Prints iterations and ||x - x_ref|| / ||x_ref|| per lattice.
    python tools/proto_cg_variants.py [--sizes 64,128,256]
"""
import argparse
import ctypes
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def setup(Nx, Nt, sigma, seed_u=4321, seed_chi=91011):
    import schwingermodel_amd as sm
    S = Nx * Nt
    U = np.empty(4 * S)
    chi = np.empty(4 * S)
    sm.lib.sm_fill_gauge(seed_u, sigma, Nt, 0, Nx, 0, Nt, U.ctypes.data, U[2 * S:].ctypes.data)
    sm.lib.sm_fill_spinor(seed_chi, Nt, 0, Nx, 0, Nt, chi.ctypes.data, chi[2 * S:].ctypes.data)
    return U, chi


def make_A(o, Nx, Nt, U, m0):
    S = Nx * Nt
    tmp = np.empty(4 * S)
    out = np.empty(4 * S)

    def A(v):  # v: complex128 [2S]
        vin = np.ascontiguousarray(v).view(np.float64)
        o.oracle_ddag(Nx, Nt, U.ctypes.data, U[2 * S:].ctypes.data, vin.ctypes.data, vin[2 * S:].ctypes.data,
                      tmp.ctypes.data, tmp[2 * S:].ctypes.data, out.ctypes.data, out[2 * S:].ctypes.data,
                      ctypes.c_double(m0))
        return out.view(np.complex128).copy()
    return A


def dot(a, b):
    return np.sum(a * np.conj(b))


def cg_ref(A, phi, tol, max_iter):
    x = phi.copy()
    r = phi - A(x)
    d = r.copy()
    rn = dot(r, r)
    pn = np.sqrt(dot(phi, phi).real)
    for k in range(max_iter):
        Ad = A(d)
        al = rn / dot(d, Ad)
        x += al * d
        r -= al * Ad
        err = np.sqrt(dot(r, r).real)
        if err < tol * pn:
            return x, k + 1
        be = err * err / rn
        d = d * be + r
        rn = dot(r, r)
    return x, max_iter


def cg_onepass(A, phi, tol, max_iter):
    """j-th pass: r_j = r_{j-1} - a_{j-1} Ad_{j-1}; d_j = b_{j-1} d_{j-1} + r_j; x += a_{j-1} d_{j-1}."""
    x = phi.copy()
    r = phi - A(x)
    d = r.copy()
    pn = np.sqrt(dot(phi, phi).real)
    Ad = A(d)
    rr = dot(r, r).real
    al = rr / dot(d, Ad)
    be = (rr - 2 * (np.conj(al) * dot(r, Ad)).real + abs(al) ** 2 * dot(Ad, Ad).real) / rr
    for k in range(1, max_iter + 1):
        x += al * d
        r = r - al * Ad
        d = d * be + r
        Ad = A(d)
        rr = dot(r, r).real
        if np.sqrt(rr) < tol * pn:
            return x, k
        al = rr / dot(d, Ad)
        be = (rr - 2 * (np.conj(al) * dot(r, Ad)).real + abs(al) ** 2 * dot(Ad, Ad).real) / rr
    return x, max_iter


def cg_rless(A, phi, tol, max_iter):
    """No stored r. Pass j holds d_{j-1}, d_{j-2}, Ad_{j-1}, b_{j-2}, a_{j-1}, b_{j-1}."""
    x = phi.copy()
    r0 = phi - A(x)
    pn = np.sqrt(dot(phi, phi).real)
    d_prev = np.zeros_like(r0)   # d_{-1}: with b_{-1} = 0, r_0 = d_0 - 0
    d = r0.copy()                # d_0
    b_prev = 0.0
    Ad = A(d)
    rr = dot(r0, r0).real
    al = rr / dot(d, Ad)
    be = (rr - 2 * (np.conj(al) * dot(r0, Ad)).real + abs(al) ** 2 * dot(Ad, Ad).real) / rr
    al_prev = 0.0
    for k in range(1, max_iter + 1):
        r_old = d - d_prev * b_prev          # r_{k-1} rebuilt
        r = r_old - al * Ad                  # r_k
        if k % 2 == 0:
            x = (x + al_prev * d_prev) + al * d
        dn = d * be + r                      # d_k
        d_prev, d, b_prev = d, dn, be
        al_prev = al
        Ad = A(d)
        rr = dot(r, r).real
        if np.sqrt(rr) < tol * pn:
            if k % 2 == 1:
                x = x + al_prev * d_prev
            return x, k
        al = rr / dot(d, Ad)
        be = (rr - 2 * (np.conj(al) * dot(r, Ad)).real + abs(al) ** 2 * dot(Ad, Ad).real) / rr
    return x, max_iter


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="64,128,256")
    ap.add_argument("--cases", default="0.4242:0.0,0.3246:-0.10,0.4242:-0.19,0.2374:-0.06")
    a = ap.parse_args()
    o = ctypes.CDLL(os.path.join(REPO, "oracle", "liboracle.so"))
    o.oracle_ddag.argtypes = [ctypes.c_int, ctypes.c_int] + [ctypes.c_void_p] * 8 + [ctypes.c_double]
    for N in [int(s) for s in a.sizes.split(",")]:
        for case in a.cases.split(","):
            sigma, m0 = (float(v) for v in case.split(":"))
            U, chi = setup(N, N, sigma)
            A = make_A(o, N, N, U, m0)
            phi = chi.view(np.complex128).copy()
            xr, kr = cg_ref(A, phi, 1e-10, 10000)
            res = {"N": N, "sigma": sigma, "m0": m0, "ref_iters": kr}
            for name, fn in (("onepass", cg_onepass), ("rless", cg_rless)):
                x, k = fn(A, phi, 1e-10, 10000)
                tr = np.linalg.norm(phi - A(x)) / np.linalg.norm(phi)
                res[name] = {"iters": k, "dx": float(np.linalg.norm(x - xr) / np.linalg.norm(xr)),
                             "true_res": float(tr)}
            print(res, flush=True)


if __name__ == "__main__":
    main()
