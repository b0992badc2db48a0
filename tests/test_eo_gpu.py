"""Even-odd preconditioned HMC action on the device.

Dhat = m - (1/m) D_eo D_oe (m = m0 + 2) on the even sites. The action
phi_e^dag (Dhat Dhat^dag)^{-1} phi_e samples the same gauge distribution as
the reference's phi^dag (D D^dag)^{-1} phi (det D = m^{V/2} det Dhat), so:

* Dhat / Dhat^dag equal their definition composed from the bitwise full-D
  applies (1e-14 relative: the same bracket, a different final scaling);
* the even-odd CG solves Dhat Dhat^dag x = phi_e to the tolerance, in fewer
  iterations than the full D D^dag solve;
* the MD force is minus the derivative of the Hamiltonian (central finite
  differences on single links, for BOTH actions: sign and normalisation);
* the leapfrog's energy violation is O(eps^2);
* the HMC chain's <plaquette> agrees with the unmodified reference program's
  recorded run within the combined jackknife errors (manifest "hmc_stat").
"""
import ctypes
import json
import math
import os

import numpy as np
import pytest

from conftest import GOLDEN, load_fixture, opts_env, ptr

pytestmark = pytest.mark.gpu
MAXIT = 10000


@pytest.fixture(scope="module")
def sm():
    import schwingermodel_amd
    return schwingermodel_amd


def parity_mask(Nx, Nt):
    x, t = np.meshgrid(np.arange(Nx), np.arange(Nt), indexing="ij")
    return ((x + t) % 2).reshape(-1)


def even_only(f, Nx, Nt):
    """Two-plane interleaved field with its odd sites zeroed."""
    S = Nx * Nt
    odd = parity_mask(Nx, Nt) == 1
    g = f.copy().reshape(2, S, 2)
    g[:, odd, :] = 0.0
    return g.reshape(-1)


def apply_D(sm, L, f, S, m0, dag):
    out = np.empty(4 * S)
    sm.check(sm.lib.sm_dirac(L.ctx, ptr(f[:2 * S]), ptr(f[2 * S:]), ptr(out[:2 * S]), ptr(out[2 * S:]), m0, dag))
    return out


@pytest.mark.parametrize("name", ["l32x48_b3_m-0p10", "l64x64_b5_m-0p06", "l16x16_b2_m-0p19"])
@pytest.mark.parametrize("dag", [0, 1])
def test_dhat_matches_definition(sm, name, dag):
    meta, a = load_fixture(name)
    Nx, Nt, m0 = meta["Nx"], meta["Nt"], meta["m0"]
    S, m = Nx * Nt, m0 + 2
    L = sm.Lattice(Nx, Nt)
    sm.check(sm.lib.sm_upload_gauge(L.ctx, ptr(a["U"][:2 * S]), ptr(a["U"][2 * S:])))
    v = even_only(a["psi"], Nx, Nt)
    w = apply_D(sm, L, v, S, m0, dag)                         # (m v_e, D_oe v_e)
    wo = w - even_only(w, Nx, Nt)                             # odd part
    z = apply_D(sm, L, wo, S, m0, dag)                        # (D_eo w_o, m w_o)
    expect = m * v - (1.0 / m) * even_only(z, Nx, Nt)
    got = np.empty(4 * S)
    sm.check(sm.lib.sm_eo_dhat(L.ctx, dag, ptr(v[:2 * S]), ptr(v[2 * S:]), ptr(got[:2 * S]), ptr(got[2 * S:]), m0))
    L.close()
    assert np.all(got - even_only(got, Nx, Nt) == 0.0)       # odd sites untouched (zero)
    assert np.linalg.norm(got - expect) <= 1e-14 * np.linalg.norm(expect)


@pytest.mark.parametrize("name", ["l32x48_b3_m-0p10", "l64x64_b5_m-0p06", "l8x8_hot_m0p2", "l40x24_hot_m0p2"])
@pytest.mark.parametrize("dag", [0, 1])
def test_fused_dhat_bitwise_equals_two_hops(sm, name, dag):
    """The fused marching Dhat kernel (one pass, odd intermediate in registers)
    performs exactly the two eo_hop launches' arithmetic."""
    meta, a = load_fixture(name)
    Nx, Nt, m0 = meta["Nx"], meta["Nt"], meta["m0"]
    S = Nx * Nt
    v = even_only(a["psi"], Nx, Nt)
    outs = []
    for fused in ("1", "0"):
        with opts_env(eo_fused=fused):  # read when the context is created
            L = sm.Lattice(Nx, Nt)
        sm.check(sm.lib.sm_upload_gauge(L.ctx, ptr(a["U"][:2 * S]), ptr(a["U"][2 * S:])))
        o = np.empty(4 * S)
        sm.check(sm.lib.sm_eo_dhat(L.ctx, dag, ptr(v[:2 * S]), ptr(v[2 * S:]), ptr(o[:2 * S]), ptr(o[2 * S:]), m0))
        L.close()
        outs.append(o)
    assert np.array_equal(outs[0].view(np.uint64), outs[1].view(np.uint64))


@pytest.mark.parametrize("name", ["l64x64_b5_m-0p06", "l32x48_b3_m-0p10"])
def test_eo_cg_solves_and_converges_faster(sm, name):
    meta, a = load_fixture(name)
    Nx, Nt, m0 = meta["Nx"], meta["Nt"], meta["m0"]
    S = Nx * Nt
    L = sm.Lattice(Nx, Nt)
    sm.check(sm.lib.sm_upload_gauge(L.ctx, ptr(a["U"][:2 * S]), ptr(a["U"][2 * S:])))
    phi = even_only(a["psi"], Nx, Nt)
    x = np.empty(4 * S)
    res = sm.CGResult()
    sm.check(sm.lib.sm_eo_cg(L.ctx, ptr(phi[:2 * S]), ptr(phi[2 * S:]), ptr(x[:2 * S]), ptr(x[2 * S:]), m0, 1e-10,
                             MAXIT, ctypes.byref(res)))
    assert res.converged == 1
    # true residual |phi_e - Dhat Dhat^dag x| / |phi_e|
    y, z = np.empty(4 * S), np.empty(4 * S)
    sm.check(sm.lib.sm_eo_dhat(L.ctx, 1, ptr(x[:2 * S]), ptr(x[2 * S:]), ptr(y[:2 * S]), ptr(y[2 * S:]), m0))
    sm.check(sm.lib.sm_eo_dhat(L.ctx, 0, ptr(y[:2 * S]), ptr(y[2 * S:]), ptr(z[:2 * S]), ptr(z[2 * S:]), m0))
    L.close()
    assert np.linalg.norm(phi - z) / np.linalg.norm(phi) < 1e-10
    assert res.iterations < 0.6 * meta["cg_iters"], (res.iterations, meta["cg_iters"])


def _gen_eo_case(sm, Nx, Nt):
    S = Nx * Nt
    a = {"U": np.empty(4 * S), "psi": np.empty(4 * S)}
    sm.lib.sm_fill_gauge(4321, 0.3246, Nt, 0, Nx, 0, Nt, ptr(a["U"][:2 * S]), ptr(a["U"][2 * S:]))
    sm.lib.sm_fill_spinor(5678, Nt, 0, Nx, 0, Nt, ptr(a["psi"][:2 * S]), ptr(a["psi"][2 * S:]))
    return {"Nx": Nx, "Nt": Nt, "m0": -0.1}, a


@pytest.mark.parametrize("variant", ["eo_cg_folded", "eo_cg_td"], ids=["folded", "twodir"])
@pytest.mark.parametrize("name", ["l64x64_b5_m-0p06", "l32x48_b3_m-0p10", "l16x16_b2_m-0p19", "gen:256x120",
                                  "gen:8x12"])
def test_folded_eo_cg_matches_six_kernel_eo_cg(sm, name, variant):
    """The folded even-odd CG (2 passes + scalars per iteration, the one-pass
    recurrence) and the one-pass two-direction kernel (sm_eotd.hip: four
    checkerboard hops in registers, <d, Ad> as |Dhat^dag d|^2) against the
    six-launch even-odd CG with the reference's recurrence: same stop rule,
    iterations +-1 %, solution to 1e-10 (their beta differs from the
    reference's by rounding only)."""
    if name.startswith("gen:"):
        Nx, Nt = (int(v) for v in name[4:].split("x"))
        meta, a = _gen_eo_case(sm, Nx, Nt)
    else:
        meta, a = load_fixture(name)
    Nx, Nt, m0 = meta["Nx"], meta["Nt"], meta["m0"]
    S = Nx * Nt
    phi = even_only(a["psi"], Nx, Nt)
    out = {}
    for folded in ("1", "0"):
        with opts_env(**{variant: folded}):  # read when the context is created
            L = sm.Lattice(Nx, Nt)
        sm.check(sm.lib.sm_upload_gauge(L.ctx, ptr(a["U"][:2 * S]), ptr(a["U"][2 * S:])))
        x = np.empty(4 * S)
        res = sm.CGResult()
        sm.check(sm.lib.sm_eo_cg(L.ctx, ptr(phi[:2 * S]), ptr(phi[2 * S:]), ptr(x[:2 * S]), ptr(x[2 * S:]), m0,
                                 1e-10, MAXIT, ctypes.byref(res)))
        L.close()
        assert res.converged == 1
        out[folded] = (x, res.iterations)
    (xf, itf), (xs, its) = out["1"], out["0"]
    assert abs(itf - its) <= max(1, its // 100), (itf, its)
    assert np.linalg.norm(xf - xs) <= 1e-10 * np.linalg.norm(xs)
    assert np.all(xf - even_only(xf, Nx, Nt) == 0.0)


def fd_force_check(sm, even_odd, N=12, links=((5, 0), (17, 1), (70, 0), (101, 1))):
    """F(n, mu) = -dH/domega for U_mu(n) -> U_mu(n) e^{i omega} (P = 0, fixed phi)."""
    S = N * N
    U = np.empty(4 * S)
    chi = np.empty(4 * S)
    sm.lib.sm_fill_gauge(4321, 0.4242, N, 0, N, 0, N, ptr(U[:2 * S]), ptr(U[2 * S:]))
    sm.lib.sm_fill_spinor(91011, N, 0, N, 0, N, ptr(chi[:2 * S]), ptr(chi[2 * S:]))
    p = sm.HMCParams(0.1, 2.0, 1.0, 4, 1e-13, MAXIT, 1, even_odd)
    L = sm.Lattice(N, N)
    sm.check(sm.lib.sm_upload_gauge(L.ctx, ptr(U[:2 * S]), ptr(U[2 * S:])))
    phi = apply_D(sm, L, chi, S, 0.1, 0)     # any fixed pseudofermion field works for the check
    if even_odd:
        phi = even_only(phi, N, N)
    F = np.empty(2 * S)
    res = sm.CGResult()
    sm.check(sm.lib.sm_md_force(L.ctx, ctypes.byref(p), ptr(phi[:2 * S]), ptr(phi[2 * S:]), ptr(F[:S]), ptr(F[S:]),
                                ctypes.byref(res)))
    P0 = np.zeros(2 * S)
    eps = 1e-4
    for n, mu in links:
        Hs = []
        for sgn in (1, -1):
            Up = U.copy()
            z = complex(Up[2 * S * mu + 2 * n], Up[2 * S * mu + 2 * n + 1]) * np.exp(1j * sgn * eps)
            Up[2 * S * mu + 2 * n], Up[2 * S * mu + 2 * n + 1] = z.real, z.imag
            sm.check(sm.lib.sm_upload_gauge(L.ctx, ptr(Up[:2 * S]), ptr(Up[2 * S:])))
            h = sm.HamiltonianTerms()
            sm.check(sm.lib.sm_hamiltonian(L.ctx, ctypes.byref(p), ptr(phi[:2 * S]), ptr(phi[2 * S:]),
                                           ptr(P0[:S]), ptr(P0[S:]), ctypes.byref(h)))
            Hs.append(h.H)
        dHdw = (Hs[0] - Hs[1]) / (2 * eps)
        f = F[mu * S + n]
        assert abs(f + dHdw) <= 1e-5 * max(1.0, abs(f)), (even_odd, n, mu, f, -dHdw)
    L.close()


def test_force_is_minus_dH_reference_action(sm):
    fd_force_check(sm, 0)


def test_force_is_minus_dH_even_odd_action(sm):
    fd_force_check(sm, 1)


def test_even_odd_energy_violation_is_second_order(sm):
    N = 32
    S = N * N
    U, chi = np.empty(4 * S), np.empty(4 * S)
    sm.lib.sm_fill_gauge(4321, 0.3246, N, 0, N, 0, N, ptr(U[:2 * S]), ptr(U[2 * S:]))
    sm.lib.sm_fill_spinor(91011, N, 0, N, 0, N, ptr(chi[:2 * S]), ptr(chi[2 * S:]))
    P = np.random.default_rng(5).standard_normal(2 * S)
    L = sm.Lattice(N, N)
    phi = None
    out = []
    for steps in (9, 17):
        sm.check(sm.lib.sm_upload_gauge(L.ctx, ptr(U[:2 * S]), ptr(U[2 * S:])))
        p = sm.HMCParams(0.1, 3.0, 1.0, steps, 1e-12, MAXIT, 1, 1)
        if phi is None:
            phi = even_only(apply_D(sm, L, chi, S, 0.1, 0), N, N)
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
    L.close()
    assert out[1] < out[0] / 2.5, out


def test_even_odd_hmc_matches_reference_statistics(sm):
    with open(os.path.join(GOLDEN, "manifest.json")) as f:
        ref = json.load(f)["hmc_stat"]
    N, Nt = ref["Nx"], ref["Nt"]
    V = N * Nt
    L = sm.Lattice(N, Nt)
    p = sm.HMCParams(ref["m0"], ref["beta"], ref["tau"], ref["md_steps"], 1e-10, MAXIT, 777, 1)
    s = sm.HMCSummary()
    n = ref["Nmeas"]
    sp = np.empty(n)
    sm.check(sm.lib.sm_hmc_run(L.ctx, ctypes.byref(p), 1, 0, ref["Ntherm"], n, ref["Nsteps"], None, ctypes.byref(s),
                               ptr(sp), None))
    L.close()
    assert s.cg_failures == 0
    sig = math.hypot(s.dEp, ref["dEp"])
    assert abs(s.Ep - ref["Ep"]) <= 4 * sig + 1e-3, (s.Ep, s.dEp, ref["Ep"], ref["dEp"])
    assert s.acceptance >= ref["acceptance"] - 0.15
