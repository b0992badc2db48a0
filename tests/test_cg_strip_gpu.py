"""t-strip blocks of the recompute-Ad CG pass (sm_tune_cg_strip, round 6).

The default pass gives each 64-lane wave its own window of 56 owned
t-columns (4 halo lanes per side feed the four stencil stages' t-hops). The
strip form makes a block's 4 waves march ONE strip of 256 lanes (248 owned
columns): a stage's t-hops between the waves cross through LDS at one
barrier, so only the strip's ends are halo lanes. The arithmetic of every
site is the same; only the dot partials' tile partition changes (and with it
the summation order of the scalars), so a solve must reach the reference's
iteration count and x within the reduction-order band (src/conjugate_gradient.cpp:
28-66), the same bars as every other CG path: against the reference's golden
vectors at 1e-12, and against the stored-Ad two-direction pass on shapes that
exercise the strip geometry -- one strip narrower than Wt, Wt a multiple of
248 and one past it, lattices narrower than one strip, chunks shorter than the
halo, balanced x-chunks, every march schedule, and solves cut off by max_iter
after an even / odd pass.
"""
import ctypes

import numpy as np
import pytest

from conftest import fixture_names, load_fixture, opts_env

pytestmark = pytest.mark.gpu

NAMES = fixture_names()


@pytest.fixture(scope="module")
def sm():
    import schwingermodel_amd
    return schwingermodel_amd


def flat(s):
    return np.concatenate([s.mu0.view(np.float64), s.mu1.view(np.float64)])


def as_spinor(sm, a, S):
    z = a.view(np.complex128)
    return sm.spinor.from_arrays(z[:S].copy(), z[S:].copy())


@pytest.mark.parametrize("name", NAMES)
def test_strip_cg_vs_reference(sm, name):
    meta, a = load_fixture(name)
    Nx, Nt, m0 = meta["Nx"], meta["Nt"], meta["m0"]
    S = Nx * Nt
    L = sm.init(Nx, Nt)
    sm.check(sm.lib.sm_tune_cg(L.ctx, 5, 0))
    sm.check(sm.lib.sm_tune_cg_strip(L.ctx, 1, -1))
    U, psi = as_spinor(sm, a["U"], S), as_spinor(sm, a["psi"], S)
    x = sm.spinor(S)
    assert sm.conjugate_gradient(U, psi, x, m0) == 1
    res = L.last_cg
    ref_it = meta["cg_iters"]
    assert abs(res.iterations - ref_it) <= max(1, ref_it // 100), (res.iterations, ref_it)
    xr = a["ref_cgx"]
    assert np.linalg.norm(flat(x) - xr) / np.linalg.norm(xr) <= 1e-12
    Ax = sm.spinor(S)
    sm.D_D_dagger_phi(U, x, Ax, m0)
    r = np.concatenate([psi.mu0 - Ax.mu0, psi.mu1 - Ax.mu1])
    assert np.linalg.norm(r) / np.linalg.norm(np.concatenate([psi.mu0, psi.mu1])) < 1e-10


@pytest.mark.parametrize("rev", [0, 1, 2])
@pytest.mark.parametrize("Nx,Nt,xchunk,max_iter,bal", [
    (96, 120, 0, 10000, 0),    # one strip wider than the lattice
    (200, 56, 7, 10000, 0),    # chunks longer than the halo, a short last chunk
    (5, 9, 0, 10000, 0),       # a lattice smaller than the halo
    (64, 248, 64, 10000, 0),   # Wt = one strip exactly
    (64, 249, 16, 10000, 1),   # one column into the second strip; balanced chunks
    (40, 500, 3, 10000, 1),    # chunks shorter than the halo rows
    (24, 4096, 0, 10000, 0),   # 17 strips, the headline's width
    (130, 66, 5, 17, 0),       # cut off after an odd pass
    (130, 66, 5, 16, 1),       # cut off after an even pass
])
def test_strip_matches_twodir(sm, Nx, Nt, xchunk, max_iter, bal, rev):
    S = Nx * Nt
    with opts_env(rev=rev, ra_red_max_blocks=0):  # read when the context is created
        L = sm.init(Nx, Nt)
    U, psi = sm.spinor(S), sm.spinor(S)
    P = lambda a: a.ctypes.data  # noqa: E731
    sm.lib.sm_fill_gauge(4321, 0.4242, Nt, 0, Nx, 0, Nt, P(U.mu0), P(U.mu1))
    sm.lib.sm_fill_spinor(5678, Nt, 0, Nx, 0, Nt, P(psi.mu0), P(psi.mu1))
    out = {}
    old = sm.CG.max_iter
    try:
        sm.CG.max_iter = max_iter
        for mode in ("twodir", "strip"):
            if mode == "strip":
                sm.check(sm.lib.sm_tune_cg(L.ctx, 5, xchunk))
                sm.check(sm.lib.sm_tune_cg_strip(L.ctx, 1, bal))
            else:
                sm.check(sm.lib.sm_tune_cg(L.ctx, 4, 0))
            x = sm.spinor(S)
            conv = sm.conjugate_gradient(U, psi, x, -0.12)
            out[mode] = (flat(x), L.last_cg.iterations, conv)
    finally:
        sm.CG.max_iter = old
    (xs, its, cs), (xt, itt, ct) = out["strip"], out["twodir"]
    assert cs == ct == (1 if max_iter == 10000 else 0)
    assert abs(its - itt) <= (1 if max_iter == 10000 else 0), (its, itt)
    rel = np.linalg.norm(xs - xt) / np.linalg.norm(xt)
    assert rel <= (1e-11 if max_iter == 10000 else 1e-13), rel


def test_strip_matches_window_pass_1024(sm):
    """At 1024^2 (the ticketed tail's grid, codes off below 4M sites) and at
    1024 x 4096 with the link codes (packed flags): strip and window passes
    agree in iterations and x."""
    for Nx, Nt in ((1024, 1024), (1024, 4096)):
        S = Nx * Nt
        U, psi = np.empty(4 * S), np.empty(4 * S)
        sm.lib.sm_fill_gauge(4321, 0.2374, Nt, 0, Nx, 0, Nt, U.ctypes.data, U[2 * S:].ctypes.data)
        sm.lib.sm_fill_spinor(5678, Nt, 0, Nx, 0, Nt, psi.ctypes.data, psi[2 * S:].ctypes.data)
        out = {}
        for strip in (0, 1):
            L = sm.Lattice(Nx, Nt)
            try:
                sm.check(sm.lib.sm_upload_gauge(L.ctx, U.ctypes.data, U[2 * S:].ctypes.data))
                sm.check(sm.lib.sm_tune_cg(L.ctx, 5, 0))
                sm.check(sm.lib.sm_tune_cg_strip(L.ctx, strip, -1))
                x = np.empty(4 * S)
                res = sm.CGResult()
                sm.check(sm.lib.sm_cg(L.ctx, psi.ctypes.data, psi[2 * S:].ctypes.data, x.ctypes.data,
                                      x[2 * S:].ctypes.data, -0.06, 1e-10, 10000, ctypes.byref(res)))
                b = ctypes.c_int()
                sm.check(sm.lib.sm_cg_link_bytes(L.ctx, ctypes.byref(b)))
                out[strip] = (res.converged, res.iterations, x, b.value)
            finally:
                L.close()
        assert out[0][0] == out[1][0] == 1
        assert abs(out[0][1] - out[1][1]) <= 1, (out[0][1], out[1][1])
        assert out[0][3] == out[1][3]
        assert np.linalg.norm(out[1][2] - out[0][2]) / np.linalg.norm(out[0][2]) <= 1e-12


def test_strip_refused_on_tshards(sm):
    """t-strip blocks are a one-shard form: a t-shard context (the RCCL
    loopback) refuses them and keeps its window pass."""
    L = sm.Lattice(32, 48, loopback=True)
    try:
        assert sm.lib.sm_tune_cg_strip(L.ctx, 1, -1) == 1
        assert b"one-shard" in sm.lib.sm_last_error()
    finally:
        L.close()
