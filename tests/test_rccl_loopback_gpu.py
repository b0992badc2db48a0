"""The RCCL data path on ONE GPU: sm_create_loopback.

A loopback context is one shard (the whole lattice) driven through the
t-shard code path: every halo is packed and sent with ncclSend/ncclRecv to
the context itself over a one-rank communicator, every scalar sum goes
through ncclAllReduce, the edge t-blocks run on the comm stream concurrently
with the interior launch, and the ghost links are exchanged on each gauge
upload -- exactly the calls a multi-GPU run makes, minus the wire. The
self-sent faces are the shard's own periodic wrap, so the results must equal
the plain one-shard context (sm_create):

* D, D^dag, D D^dag, the force and the gauge force: bitwise, and against the
  reference's golden vectors for the fixture;
* CG on every path (recompute-Ad, stored-Ad, six-launch): the same iteration
  count, x to 1e-13 (the t-shard scalar step sums the same partials in the
  same order, so this is normally bitwise);
* an HMC trajectory (momenta, leapfrog, Metropolis) and the even-odd CG.

Two processes cannot share one GPU under RCCL (probed: "invalid usage"), so
this is the strongest RCCL check one MI355X allows; the multi-rank protocol
itself is covered by the host-staged transport (test_dist_gpu.py) and, for
the N > 1 bench, by the driver's 8-GPU run.
"""
import ctypes

import numpy as np
import pytest

from conftest import bits_equal, load_fixture, ptr

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def sm():
    import schwingermodel_amd
    return schwingermodel_amd


def fields(sm, Nx, Nt, sigma, fixture=None):
    S = Nx * Nt
    if fixture is not None:
        meta, a = load_fixture(fixture)
        return a["U"].copy(), a["psi"].copy(), a["chi"].copy(), a
    U, psi, chi = np.empty(4 * S), np.empty(4 * S), np.empty(4 * S)
    sm.lib.sm_fill_gauge(4321, sigma, Nt, 0, Nx, 0, Nt, ptr(U[:2 * S]), ptr(U[2 * S:]))
    sm.lib.sm_fill_spinor(5678, Nt, 0, Nx, 0, Nt, ptr(psi[:2 * S]), ptr(psi[2 * S:]))
    sm.lib.sm_fill_spinor(91011, Nt, 0, Nx, 0, Nt, ptr(chi[:2 * S]), ptr(chi[2 * S:]))
    return U, psi, chi, None


def run_all(sm, L, U, psi, chi, m0, S):
    """Every operator of the path on context L; returns a dict of results."""
    c = L.ctx
    h = lambda a: (ptr(a[:2 * S]), ptr(a[2 * S:]))  # noqa: E731
    out = {}
    sm.check(sm.lib.sm_upload_gauge(c, *h(U)))
    for k, dag in (("Dpsi", 0), ("Ddagchi", 1)):
        o = np.empty(4 * S)
        sm.check(sm.lib.sm_dirac(c, *h(psi if dag == 0 else chi), *h(o), m0, dag))
        out[k] = o
    o = np.empty(4 * S)
    sm.check(sm.lib.sm_ddag(c, *h(psi), *h(o), m0))
    out["DDdagpsi"] = o
    F = np.empty(2 * S)
    sm.check(sm.lib.sm_force(c, *h(psi), *h(chi), ptr(F[:S]), ptr(F[S:])))
    out["force"] = F
    Fg = np.zeros(2 * S)
    sm.check(sm.lib.sm_gauge_force(c, 3.0, ptr(Fg[:S]), ptr(Fg[S:])))
    out["gauge_force"] = Fg
    d = np.zeros(2)
    sm.check(sm.lib.sm_dot(c, *h(chi), *h(out["Dpsi"]), ptr(d)))
    out["dot"] = d
    for mode in (5, 4, 0):
        sm.check(sm.lib.sm_tune_cg(c, mode, 0))
        x = np.empty(4 * S)
        res = sm.CGResult()
        sm.check(sm.lib.sm_cg(c, *h(psi), *h(x), m0, 1e-10, 10000, ctypes.byref(res)))
        out[f"cg{mode}"] = (x, res.iterations, res.converged)
    return out


CASES = [
    # (lattice, sigma, m0, fixture): the fixture is checked against the reference too
    ((32, 48), 0.0, -0.10, "l32x48_b3_m-0p10"),
    # several t-blocks: interior / edge split with the edge launch on the comm stream
    ((96, 1024), 0.3246, -0.08, None),
    # 4096 columns: the headline shape's recompute-Ad geometry (4-deep faces)
    ((64, 4096), 0.2374, -0.06, None),
]


def test_loopback_comm_info(sm):
    """sm_comm_info reads the world from the communicator itself: the loopback
    is RCCL with ncclCommCount 1 and rank 0; a one-shard context has no
    transport (bench.py reports these as rccl_ranks)."""
    loop = sm.Lattice(32, 48, loopback=True)
    try:
        assert loop.comm_info() == ("rccl", 1, 0)
        ip = ctypes.c_int(-1)
        sm.check(sm.lib.sm_cg_sums_in_pass(loop.ctx, ctypes.byref(ip)))
        assert ip.value == 1  # the CG pass's sums in-pass (peer header), the halos over RCCL
    finally:
        loop.close()
    one = sm.Lattice(32, 48)
    try:
        assert one.comm_info() == ("none", 1, 0)
    finally:
        one.close()


@pytest.mark.parametrize("shape,sigma,m0,fixture", CASES, ids=["32x48_fixture", "96x1024", "64x4096"])
def test_loopback_equals_one_shard(sm, shape, sigma, m0, fixture):
    Nx, Nt = shape
    S = Nx * Nt
    U, psi, chi, gold = fields(sm, Nx, Nt, sigma, fixture)
    one = sm.Lattice(Nx, Nt)
    ref = run_all(sm, one, U, psi, chi, m0, S)
    one.close()
    loop = sm.Lattice(Nx, Nt, loopback=True)
    got = run_all(sm, loop, U, psi, chi, m0, S)
    loop.close()
    for k in ("Dpsi", "Ddagchi", "DDdagpsi", "force", "gauge_force"):
        assert bits_equal(got[k], ref[k]), k
    if gold is not None:
        for k in ("Dpsi", "Ddagchi", "DDdagpsi", "force"):
            assert bits_equal(got[k], gold["ref_" + k]), k
    assert np.allclose(got["dot"], ref["dot"], rtol=1e-14, atol=0)
    for mode in (5, 4, 0):
        (x, it, conv), (xr, itr, convr) = got[f"cg{mode}"], ref[f"cg{mode}"]
        assert conv == 1 and convr == 1 and it == itr, (mode, it, itr)
        rel = np.linalg.norm(x - xr) / np.linalg.norm(xr)
        assert rel <= 1e-13, (mode, rel)
        if gold is not None:
            assert np.linalg.norm(x - gold["ref_cgx"]) / np.linalg.norm(gold["ref_cgx"]) <= 1e-12


def test_loopback_hmc_trajectory_and_even_odd(sm):
    """An HMC trajectory (ghost links re-exchanged after every link update,
    Metropolis, reject restore) and the even-odd CG (4-deep checkerboard faces)
    through the RCCL loopback equal the one-shard context."""
    Nx, Nt = 64, 64
    S = Nx * Nt
    U, psi, chi, _ = fields(sm, Nx, Nt, 0.4242)
    res = {}
    for name, kw in (("one", {}), ("loop", {"loopback": True})):
        L = sm.Lattice(Nx, Nt, **kw)
        sm.check(sm.lib.sm_upload_gauge(L.ctx, ptr(U[:2 * S]), ptr(U[2 * S:])))
        x = np.empty(4 * S)
        cg = sm.CGResult()
        sm.check(sm.lib.sm_eo_cg(L.ctx, ptr(psi[:2 * S]), ptr(psi[2 * S:]), ptr(x[:2 * S]), ptr(x[2 * S:]),
                                 -0.05, 1e-10, 10000, ctypes.byref(cg)))
        prm = sm.HMCParams(0.0, 2.0, 0.5, 5, 1e-10, 10000, 7)
        trajs = []
        for t in range(3):
            r = sm.HMCResult()
            sm.check(sm.lib.sm_hmc_trajectory(L.ctx, ctypes.byref(prm), t, ctypes.byref(r)))
            trajs.append((r.dH, r.accepted, r.cg_iterations, r.cg_failures))
        Uo = np.empty(4 * S)
        sm.check(sm.lib.sm_download_gauge(L.ctx, ptr(Uo[:2 * S]), ptr(Uo[2 * S:])))
        res[name] = (x, cg.iterations, cg.converged, trajs, Uo)
        L.close()
    x1, it1, c1, tr1, U1 = res["one"]
    x2, it2, c2, tr2, U2 = res["loop"]
    assert c1 == c2 == 1 and it1 == it2
    assert np.linalg.norm(x2 - x1) / np.linalg.norm(x1) <= 1e-13
    for a, b in zip(tr1, tr2):
        assert a[1:] == b[1:], (a, b)
        assert abs(a[0] - b[0]) <= 1e-9 * max(1.0, abs(a[0])), (a, b)
    assert np.linalg.norm(U2 - U1) / np.linalg.norm(U1) <= 1e-12


def test_loopback_cg_after_nan_solve(sm):
    """A solve that leaves NaN in every face slot (phi = NaN) must not poison
    the next one: pass 0 of the recompute-Ad CG weights d_{-2} by zero, so its
    faces must be d_0's, not the previous solve's (regression: a stale NaN
    times beta2 = 0 made the next solve run to max_iter)."""
    Nx, Nt = 64, 4096
    S = Nx * Nt
    U, psi, _, _ = fields(sm, Nx, Nt, 0.2374)
    h = lambda a: (ptr(a[:2 * S]), ptr(a[2 * S:]))  # noqa: E731
    its = {}
    for name, kw in (("one", {}), ("loop", {"loopback": True})):
        L = sm.Lattice(Nx, Nt, **kw)
        sm.check(sm.lib.sm_upload_gauge(L.ctx, *h(U)))
        sm.check(sm.lib.sm_tune_cg(L.ctx, 5, 0))
        bad = np.full(4 * S, np.nan)
        x = np.empty(4 * S)
        res = sm.CGResult()
        sm.lib.sm_cg(L.ctx, *h(bad), *h(x), -0.06, 1e-10, 6, ctypes.byref(res))  # does not converge
        assert res.converged == 0
        sm.check(sm.lib.sm_cg(L.ctx, *h(psi), *h(x), -0.06, 1e-10, 10000, ctypes.byref(res)))
        its[name] = (res.converged, res.iterations, x.copy())
        L.close()
    assert its["loop"][0] == its["one"][0] == 1 and its["loop"][1] == its["one"][1], (its["loop"][:2], its["one"][:2])
    assert np.linalg.norm(its["loop"][2] - its["one"][2]) / np.linalg.norm(its["one"][2]) <= 1e-13


@pytest.mark.parametrize("split", [0, 1])
@pytest.mark.parametrize("shape,sigma", [((32, 48), 0.41), ((96, 1024), 0.3246), ((64, 4096), 0.2374),
                                         ((8, 2), 0.5), ((24, 3), 0.5)],
                         ids=["32x48", "96x1024", "64x4096", "8x2", "24x3"])
def test_loopback_apply_modes_bitwise(sm, shape, sigma, split):
    """Both t-shard Dirac apply schedules (faces first; interior / edge
    t-blocks around the faces -- sm_capi.cpp apply) give D, D^dag, D D^dag
    bitwise equal to the one-shard context, on shapes down to two and three
    t-columns."""
    from conftest import opts_env
    Nx, Nt = shape
    S = Nx * Nt
    U, psi, chi, _ = fields(sm, Nx, Nt, sigma)
    h = lambda a: (ptr(a[:2 * S]), ptr(a[2 * S:]))  # noqa: E731

    def ops(L):
        sm.check(sm.lib.sm_upload_gauge(L.ctx, *h(U)))
        out = []
        for dag, src in ((0, psi), (1, chi)):
            o = np.empty(4 * S)
            sm.check(sm.lib.sm_dirac(L.ctx, *h(src), *h(o), -0.07, dag))
            out.append(o)
        o = np.empty(4 * S)
        sm.check(sm.lib.sm_ddag(L.ctx, *h(psi), *h(o), -0.07))
        out.append(o)
        return out

    one = sm.Lattice(Nx, Nt)
    ref = ops(one)
    one.close()
    with opts_env(apply_split=split):
        loop = sm.Lattice(Nx, Nt, loopback=True)
    got = ops(loop)
    loop.close()
    for k, (g, r) in enumerate(zip(got, ref)):
        assert bits_equal(g, r), (split, k)


@pytest.mark.parametrize("shape", [(4096, 1024), (4096, 512)], ids=["4096x1024_edge32", "4096x512_edge8"])
def test_loopback_cg_edge_rows_rule(sm, shape):
    """The t-shard CG pass's edge launch marches 8-row chunks where even those
    let its tiles join the interior ones in one residency round (4096 x 512),
    32 where only those do (4096 x 1024) and 16 elsewhere (sm_capi.cpp
    cg_ra_pass): the loopback solve equals the
    one-shard solve (iterations within one, x to 1e-12) either way, and forcing the
    other chunk length (test option edge_xchunk) changes only the partial
    sums' partition."""
    from conftest import opts_env
    Nx, Nt = shape
    S = Nx * Nt
    U, psi, _, _ = fields(sm, Nx, Nt, 0.2374)
    h = lambda a: (ptr(a[:2 * S]), ptr(a[2 * S:]))  # noqa: E731
    out = {}
    other = 16
    for name, kw, opts in (("one", {}, {}), ("loop", {"loopback": True}, {}),
                           ("loop_other", {"loopback": True}, {"edge_xchunk": other})):
        with opts_env(**opts):
            L = sm.Lattice(Nx, Nt, **kw)
        sm.check(sm.lib.sm_upload_gauge(L.ctx, *h(U)))
        sm.check(sm.lib.sm_tune_cg(L.ctx, 5, 0))
        x = np.empty(4 * S)
        res = sm.CGResult()
        sm.check(sm.lib.sm_cg(L.ctx, *h(psi), *h(x), -0.06, 1e-10, 20000, ctypes.byref(res)))
        out[name] = (res.converged, res.iterations, x)
        L.close()
    c0, it0, x0 = out["one"]
    assert c0 == 1
    for k in ("loop", "loop_other"):
        c, it, x = out[k]
        assert c == 1 and abs(it - it0) <= 1, (k, it, it0)
        assert np.linalg.norm(x - x0) / np.linalg.norm(x0) <= 1e-12, k
