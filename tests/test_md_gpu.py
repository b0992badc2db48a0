"""GPU parity of the molecular-dynamics layer.

Against the reference's own outputs (tests/golden/md*.npz, produced by the
unmodified src/gauge_conf.cpp + src/hmc.cpp, see make_golden.py):

* bitwise: plaquette field U_01(n), staples, gauge force (Force_G), phi = D chi;
* the global sums (Sp, gauge action, kinetic term) differ only in summation
  order: relative 1e-13;
* anything downstream of a CG solve (Force, Leapfrog, Hamiltonian) inherits the
  solver's reduction-order difference, which the reference itself shows
  between its own decompositions (manifest "decomposition_2x2": up to 1.4e-10
  absolute on the MD force). Tolerances: MD force and (U', P') relative 1e-8,
  Hamiltonians relative 1e-10; CG iteration counts +-1 %.
  The link update's cos/sin come from the device math library, not glibc's
  cexp: equal to ~1 ulp, inside the same tolerance.

Plus properties the reference's algorithm guarantees at any size: leapfrog
reversibility, O(eps^2) energy violation, reproducible trajectories, an
exact restore of U on a Metropolis reject.
"""
import ctypes

import numpy as np
import pytest

from conftest import bits_equal, load_md_fixture, md_fixture_names, ptr

pytestmark = pytest.mark.gpu
NAMES = md_fixture_names()
TOL, MAXIT = 1e-10, 10000


@pytest.fixture(scope="module")
def sm():
    import schwingermodel_amd
    return schwingermodel_amd


def params(sm, meta, seed=1):
    return sm.HMCParams(meta["m0"], meta["beta"], meta["tau"], meta["md_steps"], TOL, MAXIT, seed)


def lattice(sm, meta, a):
    Nx, Nt = meta["Nx"], meta["Nt"]
    S = Nx * Nt
    L = sm.Lattice(Nx, Nt)
    sm.check(sm.lib.sm_upload_gauge(L.ctx, ptr(a["U"][:2 * S]), ptr(a["U"][2 * S:])))
    return L, S


def rel(a, b):
    return float(np.linalg.norm(a - b) / np.linalg.norm(b))


@pytest.mark.parametrize("name", NAMES)
def test_plaquette(sm, name):
    meta, a = load_md_fixture(name)
    L, S = lattice(sm, meta, a)
    sp, act = ctypes.c_double(), ctypes.c_double()
    P = np.empty(2 * S)
    sm.check(sm.lib.sm_plaquette(L.ctx, meta["beta"], ctypes.byref(sp), ctypes.byref(act), ptr(P)))
    assert bits_equal(P, a["ref_plaq"])
    assert abs(sp.value - meta["sp"]) <= 1e-13 * max(1.0, abs(meta["sp"])) + 1e-13 * S
    assert abs(act.value - meta["gauge_action"]) <= 1e-13 * abs(meta["gauge_action"]) + 1e-13 * S
    L.close()


@pytest.mark.parametrize("name", NAMES)
def test_staples_and_gauge_force_bitwise(sm, name):
    meta, a = load_md_fixture(name)
    L, S = lattice(sm, meta, a)
    St = np.empty(4 * S)
    sm.check(sm.lib.sm_staples(L.ctx, ptr(St[:2 * S]), ptr(St[2 * S:])))
    assert bits_equal(St, a["ref_staple"])
    F = np.zeros(2 * S)
    sm.check(sm.lib.sm_gauge_force(L.ctx, meta["beta"], ptr(F[:S]), ptr(F[S:])))
    assert bits_equal(F, a["ref_gforce"])
    L.close()


@pytest.mark.parametrize("name", NAMES)
def test_md_force(sm, name):
    meta, a = load_md_fixture(name)
    L, S = lattice(sm, meta, a)
    # phi = D chi through the operator path: bitwise
    phi = np.empty(4 * S)
    chi = a["chi"]
    sm.check(sm.lib.sm_dirac(L.ctx, ptr(chi[:2 * S]), ptr(chi[2 * S:]), ptr(phi[:2 * S]), ptr(phi[2 * S:]),
                             meta["m0"], 0))
    assert bits_equal(phi, a["ref_phi"])
    F = np.empty(2 * S)
    res = sm.CGResult()
    p = params(sm, meta)
    sm.check(sm.lib.sm_md_force(L.ctx, ctypes.byref(p), ptr(phi[:2 * S]), ptr(phi[2 * S:]), ptr(F[:S]),
                                ptr(F[S:]), ctypes.byref(res)))
    assert res.converged == 1
    ref_it = meta["force_cg_iters"]
    assert abs(res.iterations - ref_it) <= max(1, ref_it // 100)
    assert rel(F, a["ref_mdforce"]) <= 1e-8
    L.close()


@pytest.mark.parametrize("name", NAMES)
def test_leapfrog_and_hamiltonian(sm, name):
    meta, a = load_md_fixture(name)
    L, S = lattice(sm, meta, a)
    p = params(sm, meta)
    phi, P = a["ref_phi"], a["P"].copy()
    h = sm.HamiltonianTerms()
    sm.check(sm.lib.sm_hamiltonian(L.ctx, ctypes.byref(p), ptr(phi[:2 * S]), ptr(phi[2 * S:]), ptr(P[:S]),
                                   ptr(P[S:]), ctypes.byref(h)))
    assert h.cg_converged == 1
    assert abs(h.H - meta["H0"]) <= 1e-10 * abs(meta["H0"])
    assert abs(h.sp - meta["sp"]) <= 1e-13 * S
    assert abs(h.kinetic - 0.5 * float(np.sum(P * P))) <= 1e-12 * h.kinetic
    it, fails = ctypes.c_long(), ctypes.c_int()
    sm.check(sm.lib.sm_leapfrog(L.ctx, ctypes.byref(p), ptr(phi[:2 * S]), ptr(phi[2 * S:]), ptr(P[:S]), ptr(P[S:]),
                                ctypes.byref(it), ctypes.byref(fails)))
    assert fails.value == 0
    ref_it = meta["leapfrog_ddag_calls"] - (meta["md_steps"] - 1)
    assert abs(it.value - ref_it) <= max(1, ref_it // 100), (it.value, ref_it)
    U1 = np.empty(4 * S)
    sm.check(sm.lib.sm_download_gauge(L.ctx, ptr(U1[:2 * S]), ptr(U1[2 * S:])))
    assert rel(U1, a["ref_U1"]) <= 1e-8
    assert rel(P, a["ref_P1"]) <= 1e-8
    sm.check(sm.lib.sm_hamiltonian(L.ctx, ctypes.byref(p), ptr(phi[:2 * S]), ptr(phi[2 * S:]), ptr(P[:S]),
                                   ptr(P[S:]), ctypes.byref(h)))
    assert abs(h.H - meta["H1"]) <= 1e-10 * abs(meta["H1"])
    L.close()


def synthetic(sm, N, sigma, seed=4321):
    S = N * N
    U, chi = np.empty(4 * S), np.empty(4 * S)
    sm.lib.sm_fill_gauge(seed, sigma, N, 0, N, 0, N, ptr(U[:2 * S]), ptr(U[2 * S:]))
    sm.lib.sm_fill_spinor(91011, N, 0, N, 0, N, ptr(chi[:2 * S]), ptr(chi[2 * S:]))
    P = np.random.default_rng(5).standard_normal(2 * S)
    return U, chi, P


@pytest.mark.parametrize("N", [16, 128])
def test_leapfrog_reversible(sm, N):
    """(U, P) -> leapfrog -> (U', P'); (U', -P') -> leapfrog -> (U, -P) up to CG tolerance."""
    S = N * N
    U, chi, P = synthetic(sm, N, 0.3246)
    L = sm.Lattice(N, N)
    sm.check(sm.lib.sm_upload_gauge(L.ctx, ptr(U[:2 * S]), ptr(U[2 * S:])))
    p = sm.HMCParams(0.1, 3.0, 0.5, 6, 1e-12, MAXIT, 1)
    phi = np.empty(4 * S)
    sm.check(sm.lib.sm_dirac(L.ctx, ptr(chi[:2 * S]), ptr(chi[2 * S:]), ptr(phi[:2 * S]), ptr(phi[2 * S:]), 0.1, 0))
    P1 = P.copy()
    it, f = ctypes.c_long(), ctypes.c_int()
    sm.check(sm.lib.sm_leapfrog(L.ctx, ctypes.byref(p), ptr(phi[:2 * S]), ptr(phi[2 * S:]), ptr(P1[:S]), ptr(P1[S:]),
                                ctypes.byref(it), ctypes.byref(f)))
    P2 = -P1
    sm.check(sm.lib.sm_leapfrog(L.ctx, ctypes.byref(p), ptr(phi[:2 * S]), ptr(phi[2 * S:]), ptr(P2[:S]), ptr(P2[S:]),
                                ctypes.byref(it), ctypes.byref(f)))
    U2 = np.empty(4 * S)
    sm.check(sm.lib.sm_download_gauge(L.ctx, ptr(U2[:2 * S]), ptr(U2[2 * S:])))
    assert np.abs(U2 - U).max() < 1e-9
    assert np.abs(P2 + P).max() < 1e-8
    L.close()


def test_energy_violation_is_second_order(sm):
    """|dH| of the leapfrog falls ~4x when the step halves (O(eps^2) integrator)."""
    N = 32
    S = N * N
    U, chi, P = synthetic(sm, N, 0.3246)
    L = sm.Lattice(N, N)
    out = []
    for steps in (9, 17):  # eps ratio (steps-1)*eps fixed by tau: eps = tau/steps
        sm.check(sm.lib.sm_upload_gauge(L.ctx, ptr(U[:2 * S]), ptr(U[2 * S:])))
        p = sm.HMCParams(0.1, 3.0, 1.0, steps, 1e-12, MAXIT, 1)
        phi = np.empty(4 * S)
        sm.check(sm.lib.sm_dirac(L.ctx, ptr(chi[:2 * S]), ptr(chi[2 * S:]), ptr(phi[:2 * S]), ptr(phi[2 * S:]),
                                 0.1, 0))
        h0, h1 = sm.HamiltonianTerms(), sm.HamiltonianTerms()
        P1 = P.copy()
        sm.check(sm.lib.sm_hamiltonian(L.ctx, ctypes.byref(p), ptr(phi[:2 * S]), ptr(phi[2 * S:]), ptr(P1[:S]),
                                       ptr(P1[S:]), ctypes.byref(h0)))
        it, f = ctypes.c_long(), ctypes.c_int()
        sm.check(sm.lib.sm_leapfrog(L.ctx, ctypes.byref(p), ptr(phi[:2 * S]), ptr(phi[2 * S:]), ptr(P1[:S]),
                                    ptr(P1[S:]), ctypes.byref(it), ctypes.byref(f)))
        sm.check(sm.lib.sm_hamiltonian(L.ctx, ctypes.byref(p), ptr(phi[:2 * S]), ptr(phi[2 * S:]), ptr(P1[:S]),
                                       ptr(P1[S:]), ctypes.byref(h1)))
        out.append(abs(h1.H - h0.H))
    assert out[1] < out[0] / 2.5, out
    L.close()


def test_trajectory_accept_reject_and_reproducibility(sm):
    N = 16
    S = N * N
    U, _, _ = synthetic(sm, N, 0.4242)
    runs = []
    for _ in range(2):
        L = sm.Lattice(N, N)
        sm.check(sm.lib.sm_upload_gauge(L.ctx, ptr(U[:2 * S]), ptr(U[2 * S:])))
        p = sm.HMCParams(0.0, 2.0, 1.0, 6, TOL, MAXIT, 2024)
        log = []
        for traj in range(8):
            before = np.empty(4 * S)
            sm.check(sm.lib.sm_download_gauge(L.ctx, ptr(before[:2 * S]), ptr(before[2 * S:])))
            r = sm.HMCResult()
            sm.check(sm.lib.sm_hmc_trajectory(L.ctx, ctypes.byref(p), traj, ctypes.byref(r)))
            after = np.empty(4 * S)
            sm.check(sm.lib.sm_download_gauge(L.ctx, ptr(after[:2 * S]), ptr(after[2 * S:])))
            assert r.accepted == (r.r <= np.exp(-r.dH))
            assert r.cg_failures == 0
            assert bits_equal(after, before) == (not r.accepted)
            sp, act = ctypes.c_double(), ctypes.c_double()
            sm.check(sm.lib.sm_plaquette(L.ctx, 2.0, ctypes.byref(sp), ctypes.byref(act), None))
            assert sp.value == r.sp and act.value == r.gauge_action
            log.append((r.dH, r.accepted, r.cg_iterations, after.tobytes()))
        runs.append(log)
        L.close()
    assert runs[0] == runs[1]  # bitwise reproducible


def test_device_gauge_draw_matches_host_generator(sm):
    N = 64
    S = N * N
    L = sm.Lattice(N, N)
    for sigma in (0.4242, -1.0, 0.0):
        host = np.empty(4 * S)
        sm.lib.sm_fill_gauge(77, sigma, N, 0, N, 0, N, ptr(host[:2 * S]), ptr(host[2 * S:]))
        sm.check(sm.lib.sm_fill_gauge_dev(L.ctx, 77, sigma))
        dev = np.empty(4 * S)
        sm.check(sm.lib.sm_download_gauge(L.ctx, ptr(dev[:2 * S]), ptr(dev[2 * S:])))
        ulps = np.abs(dev.view(np.int64) - host.view(np.int64))
        assert np.abs(dev - host).max() <= 4e-16, sigma
        assert (ulps == 0).mean() > 0.9, sigma
    L.close()
