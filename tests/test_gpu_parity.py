"""GPU parity: the HIP path against the reference's golden vectors and the oracle.

Bar (SURVEY.md §8c / BASELINE.md): D, D^dag, D D^dag and the force are
BIT-IDENTICAL to the reference; CG reaches the same stop criterion with the
same iteration count (+-1 %), ||x - x_ref|| / ||x_ref|| <= 1e-12 and a true
relative residual < 1e-10.
"""
import ctypes

import numpy as np
import pytest

from conftest import bits_equal, fixture_names, load_fixture, opts_env, planes, ptr

pytestmark = pytest.mark.gpu

NAMES = fixture_names()
CG_REL_TOL = 1e-12


@pytest.fixture(scope="module")
def sm():
    import schwingermodel_amd as sm
    return sm


def as_spinor(sm, flat, S):
    p0, p1 = planes(flat, S)
    return sm.spinor.from_arrays(p0.view(np.complex128).copy(), p1.view(np.complex128).copy())


def flat(s):
    return np.concatenate([s.mu0.view(np.float64), s.mu1.view(np.float64)])


@pytest.mark.parametrize("name", NAMES)
def test_operators_bitwise_vs_reference(sm, name):
    meta, a = load_fixture(name)
    Nx, Nt, m0 = meta["Nx"], meta["Nt"], meta["m0"]
    S = Nx * Nt
    sm.init(Nx, Nt)
    U, psi, chi = (as_spinor(sm, a[k], S) for k in ("U", "psi", "chi"))
    out = sm.spinor(S)
    sm.D_phi(U, psi, out, m0)
    assert bits_equal(flat(out), a["ref_Dpsi"]), np.abs(flat(out) - a["ref_Dpsi"]).max()
    sm.D_dagger_phi(U, chi, out, m0)
    assert bits_equal(flat(out), a["ref_Ddagchi"])
    sm.D_D_dagger_phi(U, psi, out, m0)
    assert bits_equal(flat(out), a["ref_DDdagpsi"])
    F = sm.phi_dag_partialD_phi(U, psi, chi)
    assert bits_equal(np.concatenate([F.mu0, F.mu1]), a["ref_force"])


@pytest.mark.parametrize("fused", [5, 4, 0], ids=["recompute", "twodir", "sixkernel"])
@pytest.mark.parametrize("name", NAMES)
def test_cg_vs_reference(sm, name, fused):
    """Every CG path: the two-direction iteration that recomputes Ad in-kernel,
    the two-direction one-pass iteration that stores Ad (no r vector) and the
    reference's six-launch sequence."""
    meta, a = load_fixture(name)
    Nx, Nt, m0 = meta["Nx"], meta["Nt"], meta["m0"]
    S = Nx * Nt
    L = sm.init(Nx, Nt)
    sm.check(sm.lib.sm_tune_cg(L.ctx, fused, 0))
    U, psi = as_spinor(sm, a["U"], S), as_spinor(sm, a["psi"], S)
    x = sm.spinor(S)
    assert sm.conjugate_gradient(U, psi, x, m0) == 1
    res = L.last_cg
    ref_it = meta["cg_iters"]
    assert abs(res.iterations - ref_it) <= max(1, ref_it // 100), (res.iterations, ref_it)
    xr = a["ref_cgx"]
    rel = np.linalg.norm(flat(x) - xr) / np.linalg.norm(xr)
    assert rel <= CG_REL_TOL, rel
    # independent true residual through the reference's own D D^dag output path
    Ax = sm.spinor(S)
    sm.D_D_dagger_phi(U, x, Ax, m0)
    r = np.concatenate([psi.mu0 - Ax.mu0, psi.mu1 - Ax.mu1])
    p = np.concatenate([psi.mu0, psi.mu1])
    assert np.linalg.norm(r) / np.linalg.norm(p) < 1e-10
    assert res.residual < 1e-10 * res.phi_norm


@pytest.mark.parametrize("name", ["l64x64_b2_m0", "l32x48_hot_m0"])
def test_dot_matches_reference(sm, name):
    meta, a = load_fixture(name)
    S = meta["Nx"] * meta["Nt"]
    sm.init(meta["Nx"], meta["Nt"])
    chi, Dpsi = as_spinor(sm, a["chi"], S), as_spinor(sm, a["ref_Dpsi"], S)
    z = sm.dot(chi, Dpsi)
    zr = complex(*meta["dot_chi_Dpsi"])
    assert abs(z - zr) <= 1e-13 * abs(zr)


@pytest.mark.parametrize("Nx,Nt", [(64, 64), (256, 192), (130, 66)])  # redundant-scalar and scalar-kernel grids
@pytest.mark.parametrize("stop", [16, 17, 1, 2])
def test_twodir_pending_x_matches_sixkernel(sm, Nx, Nt, stop):
    """The two-direction forms (Ad stored: 4; Ad recomputed: 5) update x on
    even passes only: stopping after an odd or even number of iterations
    (max_iter) must give the x of the reference's six-launch sequence, which
    updates x every iteration."""
    S = Nx * Nt
    L = sm.init(Nx, Nt)
    U, psi = sm.spinor(S), sm.spinor(S)
    P = lambda a: a.ctypes.data  # noqa: E731
    sm.lib.sm_fill_gauge(4321, 0.3246, Nt, 0, Nx, 0, Nt, P(U.mu0), P(U.mu1))
    sm.lib.sm_fill_spinor(5678, Nt, 0, Nx, 0, Nt, P(psi.mu0), P(psi.mu1))
    xs = {}
    old = sm.CG.max_iter
    try:
        sm.CG.max_iter = stop
        for fused in (0, 4, 5):
            sm.check(sm.lib.sm_tune_cg(L.ctx, fused, 0))
            x = sm.spinor(S)
            assert sm.conjugate_gradient(U, psi, x, -0.10) == 0
            assert L.last_cg.iterations == stop
            xs[fused] = flat(x)
    finally:
        sm.CG.max_iter = old
    for fused in (4, 5):
        rel = np.linalg.norm(xs[fused] - xs[0]) / np.linalg.norm(xs[0])
        assert rel <= 1e-13, (fused, rel)


class _Hip:
    """hipMalloc / hipMemcpy through the HIP runtime libsm_hip.so itself links
    (no torch in this process: a second HIP runtime initialised after ours
    finds no GPU)."""

    def __init__(self):
        self.rt = ctypes.CDLL("libamdhip64.so.7")
        self.rt.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
        self.rt.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
        self.rt.hipFree.argtypes = [ctypes.c_void_p]
        self.rt.hipDeviceSynchronize.argtypes = []

    def upload(self, a):
        p = ctypes.c_void_p()
        assert self.rt.hipMalloc(ctypes.byref(p), a.nbytes) == 0
        assert self.rt.hipMemcpy(p, a.ctypes.data, a.nbytes, 1) == 0  # hipMemcpyHostToDevice
        return p

    def download(self, p, a):
        assert self.rt.hipDeviceSynchronize() == 0
        assert self.rt.hipMemcpy(a.ctypes.data, p, a.nbytes, 2) == 0  # hipMemcpyDeviceToHost
        return a


@pytest.mark.parametrize("passes", [17, 18])
def test_twodir_stepwise_finish_matches_sixkernel(sm, passes):
    """sm_cg_begin / sm_cg_iterate / sm_cg_finish without convergence (tol 0):
    after an odd or even number of passes the two-direction x (pending update
    added by sm_cg_finish) equals the x of the six-launch sequence after as
    many iterations (one-pass pass 0 only forms Ad_0)."""
    Nx, Nt = 128, 96
    S = Nx * Nt
    L = sm.init(Nx, Nt)
    U, psi = sm.spinor(S), sm.spinor(S)
    P = lambda a: a.ctypes.data  # noqa: E731
    sm.lib.sm_fill_gauge(4321, 0.3246, Nt, 0, Nx, 0, Nt, P(U.mu0), P(U.mu1))
    sm.lib.sm_fill_spinor(5678, Nt, 0, Nx, 0, Nt, P(psi.mu0), P(psi.mu1))
    hip = _Hip()
    dU = hip.upload(np.concatenate([U.mu0, U.mu1]))
    dphi = hip.upload(np.concatenate([psi.mu0, psi.mu1]))
    dx = hip.upload(np.zeros(2 * S, dtype=np.complex128))
    sm.check(sm.lib.sm_upload_gauge_dev(L.ctx, dU))
    xs = {}
    try:
        for fused in (0, 4, 5):
            sm.check(sm.lib.sm_tune_cg(L.ctx, fused, 0))
            sm.check(sm.lib.sm_cg_begin(L.ctx, dphi, dx, -0.10, 0.0))
            sm.check(sm.lib.sm_cg_iterate(L.ctx, passes - 1 if fused == 0 else passes))
            res = sm.CGResult()
            sm.check(sm.lib.sm_cg_finish(L.ctx, ctypes.byref(res)))
            assert res.iterations == passes - 1 and res.converged == 0
            xs[fused] = hip.download(dx, np.empty(2 * S, dtype=np.complex128))
    finally:
        for p in (dU, dphi, dx):
            hip.rt.hipFree(p)
    for fused in (4, 5):
        rel = np.linalg.norm(xs[fused] - xs[0]) / np.linalg.norm(xs[0])
        assert rel <= 1e-13, (fused, rel)


@pytest.mark.parametrize("fold,red", [("2", "512"), ("2", "0"), ("1", "512"), ("0", "512")])
@pytest.mark.parametrize("Nx,Nt,xchunk", [(96, 120, 0), (200, 56, 7), (5, 9, 0), (64, 64, 64)])
def test_recompute_matches_twodir(sm, Nx, Nt, xchunk, fold, red):
    """The recompute-Ad pass (fused multiply-add, folded and exact bracket
    arithmetic; in-kernel redundant scalars or the scalar kernel) against the
    two-direction pass that stores Ad: the same iteration count to 1e-10 and
    x within the reduction-order band, including chunks shorter than the
    4-row halo, Nt not a multiple of the 56-column wave and a lattice smaller
    than one wave's halo."""
    S = Nx * Nt
    with opts_env(fold=fold, ra_red_max_blocks=red):  # read when the context is created
        L = sm.init(Nx, Nt)
    U, psi = sm.spinor(S), sm.spinor(S)
    P = lambda a: a.ctypes.data  # noqa: E731
    sm.lib.sm_fill_gauge(4321, 0.4242, Nt, 0, Nx, 0, Nt, P(U.mu0), P(U.mu1))
    sm.lib.sm_fill_spinor(5678, Nt, 0, Nx, 0, Nt, P(psi.mu0), P(psi.mu1))
    out = {}
    for fused in (4, 5):
        sm.check(sm.lib.sm_tune_cg(L.ctx, fused, xchunk if fused == 5 else 0))
        x = sm.spinor(S)
        assert sm.conjugate_gradient(U, psi, x, -0.12) == 1
        out[fused] = (flat(x), L.last_cg.iterations)
    assert abs(out[5][1] - out[4][1]) <= 1, (out[5][1], out[4][1])
    rel = np.linalg.norm(out[5][0] - out[4][0]) / np.linalg.norm(out[4][0])
    assert rel <= 1e-11, rel


@pytest.mark.parametrize("rev", [0, 1, 2])
@pytest.mark.parametrize("Nx,Nt,xchunk,max_iter", [(96, 120, 0, 10000), (200, 56, 7, 10000), (5, 9, 0, 10000),
                                                  (64, 64, 64, 10000), (130, 66, 5, 17), (130, 66, 5, 16)])
def test_march_schedules_match_twodir(sm, Nx, Nt, xchunk, max_iter, rev):
    """The recompute-Ad pass under each march schedule (test option rev:
    0 all forward, 1 odd passes backwards over reversed tiles, 2 x-adjacent
    chunks in opposite directions as well; the ticketed-tail grids take it, so
    the redundant-scalar path is switched off) against the stored-Ad
    two-direction pass: same iteration count, x in the reduction-order band,
    including chunks shorter than the 4-row halo, a last chunk shorter than
    the others, odd chunk counts, a lattice smaller than one wave's halo, and
    solves cut off by max_iter after an even / odd pass (the pending x rows
    of a backward pass)."""
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
        for fused in (4, 5):
            sm.check(sm.lib.sm_tune_cg(L.ctx, fused, xchunk if fused == 5 else 0))
            x = sm.spinor(S)
            conv = sm.conjugate_gradient(U, psi, x, -0.12)
            out[fused] = (flat(x), L.last_cg.iterations, conv)
    finally:
        sm.CG.max_iter = old
    assert out[5][2] == out[4][2] == (1 if max_iter == 10000 else 0)
    assert abs(out[5][1] - out[4][1]) <= (1 if max_iter == 10000 else 0), (out[5][1], out[4][1])
    rel = np.linalg.norm(out[5][0] - out[4][0]) / np.linalg.norm(out[4][0])
    assert rel <= (1e-11 if max_iter == 10000 else 1e-13), rel


def test_cg_nonconvergence_semantics(sm, capsys):
    meta, a = load_fixture("l64x64_b5_m-0p06")
    S = 64 * 64
    L = sm.init(64, 64)
    U, psi = as_spinor(sm, a["U"], S), as_spinor(sm, a["psi"], S)
    x = sm.spinor(S)
    old = sm.CG.max_iter
    try:
        sm.CG.max_iter = 17
        assert sm.conjugate_gradient(U, psi, x, meta["m0"]) == 0
    finally:
        sm.CG.max_iter = old
    assert L.last_cg.iterations == 17 and L.last_cg.converged == 0
    assert "did not converge in 17 iterations" in capsys.readouterr().out


def test_oracle_parity_random_sizes(sm, oracle):
    """Bitwise vs the oracle on fresh seeded inputs (sizes not in the fixtures)."""
    for Nx, Nt, sigma, m0 in ((24, 72, 0.3, -0.05), (130, 66, -1.0, 0.1), (7, 5, 0.5, 0.0)):
        S = Nx * Nt
        sm.init(Nx, Nt)
        U, psi = sm.spinor(S), sm.spinor(S)
        sm.lib.sm_fill_gauge(11, sigma, Nt, 0, Nx, 0, Nt, ptr(U.mu0), ptr(U.mu1))
        sm.lib.sm_fill_spinor(12, Nt, 0, Nx, 0, Nt, ptr(psi.mu0), ptr(psi.mu1))
        for dag in (0, 1):
            out, ref = sm.spinor(S), sm.spinor(S)
            (sm.D_dagger_phi if dag else sm.D_phi)(U, psi, out, m0)
            oracle.oracle_dirac(Nx, Nt, ptr(U.mu0), ptr(U.mu1), ptr(psi.mu0), ptr(psi.mu1),
                                ptr(ref.mu0), ptr(ref.mu1), m0, dag)
            assert bits_equal(flat(out), flat(ref)), (Nx, Nt, dag)


@pytest.mark.parametrize("Nx,Nt", [(1024, 1024), (4096, 4096)])
def test_large_lattice_properties(sm, oracle, Nx, Nt):
    """Full-size checks: bitwise vs the threaded oracle on the same inputs
    (1024^2) and the size-independent adjointness <chi, D psi> = <D^dag chi, psi>."""
    S = Nx * Nt
    L = sm.init(Nx, Nt)
    U, psi, chi = sm.spinor(S), sm.spinor(S), sm.spinor(S)
    sm.lib.sm_fill_gauge(4321, 0.2374, Nt, 0, Nx, 0, Nt, ptr(U.mu0), ptr(U.mu1))
    sm.lib.sm_fill_spinor(5678, Nt, 0, Nx, 0, Nt, ptr(psi.mu0), ptr(psi.mu1))
    sm.lib.sm_fill_spinor(91011, Nt, 0, Nx, 0, Nt, ptr(chi.mu0), ptr(chi.mu1))
    m0 = -0.06
    Dpsi, Ddchi = sm.spinor(S), sm.spinor(S)
    sm.D_phi(U, psi, Dpsi, m0)
    sm.D_dagger_phi(U, chi, Ddchi, m0)
    z1, z2 = sm.dot(chi, Dpsi), sm.dot(Ddchi, psi)
    assert abs(z1 - z2) <= 1e-12 * abs(z1)
    if Nx <= 1024:
        ref = sm.spinor(S)
        oracle.oracle_dirac_mt(Nx, Nt, ptr(U.mu0), ptr(U.mu1), ptr(psi.mu0), ptr(psi.mu1),
                               ptr(ref.mu0), ptr(ref.mu1), m0, 0, 8)
        assert bits_equal(flat(Dpsi), flat(ref))
    L.close()


def _angles_in_use(sm, L):
    u = ctypes.c_int(-1)
    sm.check(sm.lib.sm_cg_link_angles(L.ctx, -1, ctypes.byref(u)))
    return u.value


@pytest.mark.parametrize("name", NAMES)
def test_link_angles_vs_complex_links(sm, name):
    """The recompute-Ad pass reading each link as its exact code (10 instead
    of 16 B per link, the default; sm_linkcode.h) against the same pass
    reading the complex links: the decoder rebuilds every link bitwise, so the
    two solves are the same arithmetic -- same iteration count, x bitwise
    equal -- and both meet the reference's solution to 1e-12
    (test_cg_vs_reference runs the default)."""
    meta, a = load_fixture(name)
    Nx, Nt, m0 = meta["Nx"], meta["Nt"], meta["m0"]
    S = Nx * Nt
    L = sm.init(Nx, Nt)
    sm.check(sm.lib.sm_tune_cg(L.ctx, 5, 0))
    U, psi = as_spinor(sm, a["U"], S), as_spinor(sm, a["psi"], S)
    out = {}
    try:
        for on in (0, 1):
            sm.check(sm.lib.sm_cg_link_angles(L.ctx, on, None))
            x = sm.spinor(S)
            assert sm.conjugate_gradient(U, psi, x, m0) == 1
            assert _angles_in_use(sm, L) == on
            out[on] = (flat(x), L.last_cg.iterations)
    finally:
        sm.check(sm.lib.sm_cg_link_angles(L.ctx, 1, None))
    assert out[1][1] == out[0][1], (out[1][1], out[0][1])
    assert bits_equal(out[1][0], out[0][0])
    xr = a["ref_cgx"]
    assert np.linalg.norm(out[1][0] - xr) / np.linalg.norm(xr) <= CG_REL_TOL


def test_link_angles_follow_gauge_updates(sm):
    """Link codes are rebuilt after every change of U (upload, MD update),
    never reused stale (each solve is bitwise its complex-link twin), and a
    field with a link too far off the unit circle for a 14-bit ulp offset
    keeps the complex-link pass (again bitwise the codes-off solve)."""
    Nx, Nt = 96, 64
    S = Nx * Nt
    L = sm.init(Nx, Nt)
    sm.check(sm.lib.sm_tune_cg(L.ctx, 5, 0))  # the recompute-Ad pass (default from 256^2 sites)
    P = lambda a: a.ctypes.data  # noqa: E731
    U1, U2, psi = sm.spinor(S), sm.spinor(S), sm.spinor(S)
    sm.lib.sm_fill_gauge(11, 0.4, Nt, 0, Nx, 0, Nt, P(U1.mu0), P(U1.mu1))
    sm.lib.sm_fill_gauge(12, 0.9, Nt, 0, Nx, 0, Nt, P(U2.mu0), P(U2.mu1))
    sm.lib.sm_fill_spinor(13, Nt, 0, Nx, 0, Nt, P(psi.mu0), P(psi.mu1))

    def solve(U, on):
        sm.check(sm.lib.sm_cg_link_angles(L.ctx, on, None))
        x = sm.spinor(S)
        assert sm.conjugate_gradient(U, psi, x, -0.1) == 1
        return flat(x), _angles_in_use(sm, L)

    try:
        x1, u1 = solve(U1, 1)
        x2, u2 = solve(U2, 1)       # new U: codes rebuilt
        x2c, _ = solve(U2, 0)
        x1c, _ = solve(U1, 0)
        assert u1 == 1 and u2 == 1
        assert bits_equal(x2, x2c) and bits_equal(x1, x1c)
        assert np.linalg.norm(x1 - x2) / np.linalg.norm(x1) > 1e-3  # the solves did see different fields
        bad = U2.copy()
        bad.mu1[17] *= 1.0 + 1e-9  # one link off the unit circle by ~4e6 ulps
        xb, ub = solve(bad, 1)
        xbc, _ = solve(bad, 0)
        assert ub == 0
        assert bits_equal(xb, xbc)
    finally:
        sm.check(sm.lib.sm_cg_link_angles(L.ctx, 1, None))


def _code_check(sm, L, out=None):
    err, bad = ctypes.c_double(-1.0), ctypes.c_long(-1)
    sm.check(sm.lib.sm_link_code_check(L.ctx, out, ctypes.byref(err), ctypes.byref(bad)))
    return err.value, bad.value


def test_link_codes_decode_on_device_config3(sm):
    """The codes of the bench field (config 3: 4096^2, beta = 5 Gaussian theta,
    the counter-based generator on the device), encoded and decoded ON THE
    DEVICE with the CG pass's own functions (v_rsq_f64 seed): every link is
    rebuilt bitwise (largest error exactly 0, no link flagged)."""
    Nx = Nt = 4096
    L = sm.init(Nx, Nt)
    try:
        sm.check(sm.lib.sm_fill_gauge_dev(L.ctx, 4321, 0.2374))
        err, bad = _code_check(sm, L)
        print(f"config-3 field: largest |rebuilt - stored| component {err:.3e}, links not rebuilt bitwise: {bad}")
        assert bad == 0 and err == 0.0, (err, bad)
    finally:
        L.close()


def test_link_codes_device_decode_matches_stored_links(sm):
    """The rebuilt links themselves, downloaded: on a generated field, on a
    field with every link pushed off the unit circle by a few ulp and on one
    with a link 1e-15 off, every link comes back bitwise; a link 1e-9 off (an
    ulp offset beyond 14 bits) is the only one flagged, and the solve then
    reads the complex links. Whichever form the solve reads, its x is bitwise
    the complex-link solve's."""
    Nx, Nt = 96, 64
    S = Nx * Nt
    L = sm.init(Nx, Nt)
    sm.check(sm.lib.sm_tune_cg(L.ctx, 5, 0))
    P = lambda a: a.ctypes.data  # noqa: E731
    U, psi = sm.spinor(S), sm.spinor(S)
    sm.lib.sm_fill_gauge(11, 0.4, Nt, 0, Nx, 0, Nt, P(U.mu0), P(U.mu1))
    sm.lib.sm_fill_spinor(13, Nt, 0, Nx, 0, Nt, P(psi.mu0), P(psi.mu1))
    hip = _Hip()
    rng = np.random.default_rng(7)
    drift = U.copy()
    f = 1.0 + rng.integers(-6, 7, 2 * S) * 2.0 ** -53  # |U|^2 - 1 up to ~1.3e-15
    drift.mu0 *= f[:S]
    drift.mu1 *= f[S:]
    near = U.copy()
    near.mu0[123] *= 1.0 + 1e-15
    far = U.copy()
    far.mu0[123] *= 1.0 + 1e-9
    try:
        # link bytes per site the pass reads: packed flag nibbles (fresh field,
        # every ulp offset in [-2, 1]), 16-bit flag words (offsets beyond), or
        # the complex links (a link not encodable)
        for field, nbad, lbytes in ((U, 0, 17), (drift, 0, 20), (near, 0, 20), (far, 1, 32)):
            host = np.concatenate([field.mu0, field.mu1])
            dU = hip.upload(host)
            dout = hip.upload(np.zeros(2 * S, dtype=np.complex128))
            sm.check(sm.lib.sm_upload_gauge_dev(L.ctx, dU))
            err, bad = _code_check(sm, L, dout)
            back = hip.download(dout, np.empty(2 * S, dtype=np.complex128))
            same = back.view(np.uint64).reshape(-1, 2) == host.view(np.uint64).reshape(-1, 2)
            assert bad == nbad == int((~same.all(axis=1)).sum()), (bad, nbad)
            comp = np.maximum(np.abs(back.real - host.real), np.abs(back.imag - host.imag))
            assert err == comp.max(), (err, comp.max())
            xs = {}
            for on in (1, 0):
                sm.check(sm.lib.sm_cg_link_codes(L.ctx, on, None))
                x = sm.spinor(S)
                assert sm.conjugate_gradient(field, psi, x, -0.1) == 1
                u = ctypes.c_int(-1)
                sm.check(sm.lib.sm_cg_link_codes(L.ctx, -1, ctypes.byref(u)))
                xs[on] = (flat(x), u.value)
            assert xs[1][1] == (1 if bad == 0 else 0), (bad, xs[1][1])
            assert bits_equal(xs[1][0], xs[0][0])
            sm.check(sm.lib.sm_cg_link_codes(L.ctx, 1, None))
            x = sm.spinor(S)
            assert sm.conjugate_gradient(field, psi, x, -0.1) == 1
            b = ctypes.c_int(-1)
            sm.check(sm.lib.sm_cg_link_bytes(L.ctx, ctypes.byref(b)))
            assert b.value == lbytes, (b.value, lbytes)
    finally:
        sm.check(sm.lib.sm_cg_link_codes(L.ctx, 1, None))


def test_link_bytes_recorded_at_launch(sm):
    """sm_cg_link_bytes reports what the last CG pass launched read (ADVICE
    r05): 0 before any pass, the packed codes' 17 after a solve on a fresh
    field, STILL 17 after a gauge upload that no solve has used yet (a field
    with one link off the circle, which the next solve reads as complex links),
    then 32 after that solve, and 32 for the stored-Ad pass."""
    Nx, Nt = 256, 256
    S = Nx * Nt
    L = sm.init(Nx, Nt)
    U, psi = sm.spinor(S), sm.spinor(S)
    P = lambda a: a.ctypes.data  # noqa: E731
    sm.lib.sm_fill_gauge(4321, 0.2374, Nt, 0, Nx, 0, Nt, P(U.mu0), P(U.mu1))
    sm.lib.sm_fill_spinor(5678, Nt, 0, Nx, 0, Nt, P(psi.mu0), P(psi.mu1))

    def link_bytes():
        b = ctypes.c_int(-1)
        sm.check(sm.lib.sm_cg_link_bytes(L.ctx, ctypes.byref(b)))
        return b.value

    assert link_bytes() == 0
    sm.check(sm.lib.sm_tune_cg(L.ctx, 5, 0))
    sm.check(sm.lib.sm_cg_link_codes(L.ctx, 1, None))
    try:
        x = sm.spinor(S)
        assert sm.conjugate_gradient(U, psi, x, -0.1) == 1
        assert link_bytes() == 17
        far = U.copy()
        far.mu0[77] *= 1.0 + 1e-9
        L.upload_gauge(far)
        assert link_bytes() == 17  # no pass has read the new field yet
        x = sm.spinor(S)
        assert sm.conjugate_gradient(far, psi, x, -0.1) == 1
        assert link_bytes() == 32
        sm.check(sm.lib.sm_tune_cg(L.ctx, 4, 0))
        x = sm.spinor(S)
        assert sm.conjugate_gradient(U, psi, x, -0.1) == 1
        assert link_bytes() == 32
    finally:
        sm.check(sm.lib.sm_cg_link_codes(L.ctx, 1, None))


@pytest.mark.parametrize("drift", [False, True], ids=["packed_flags", "flag_words"])
def test_link_codes_tshard_path_bitwise(sm, drift):
    """The t-shard form of the code pass (faces of codes and flags through
    the RCCL loopback context, sm_create_loopback) in both flag formats: a
    fresh field (flag nibbles, 17 B/site of links) and one with every link a
    few ulp off the circle (16-bit flag words, 20 B/site). Codes on and off
    give bitwise the same x, and the same x as the one-shard context."""
    Nx, Nt = 64, 512
    S = Nx * Nt
    P = lambda a: a.ctypes.data  # noqa: E731
    U, psi = sm.spinor(S), sm.spinor(S)
    sm.lib.sm_fill_gauge(4321, 0.3246, Nt, 0, Nx, 0, Nt, P(U.mu0), P(U.mu1))
    sm.lib.sm_fill_spinor(13, Nt, 0, Nx, 0, Nt, P(psi.mu0), P(psi.mu1))
    if drift:
        f = 1.0 + np.random.default_rng(3).integers(-6, 7, 2 * S) * 2.0 ** -53
        U.mu0 *= f[:S]
        U.mu1 *= f[S:]
    out = {}
    for loop in (True, False):
        L = sm.init(Nx, Nt, loopback=loop)  # the context the reference-shaped calls use
        try:
            sm.check(sm.lib.sm_tune_cg(L.ctx, 5, 0))
            for on in (1, 0):
                sm.check(sm.lib.sm_cg_link_codes(L.ctx, on, None))
                x = sm.spinor(S)
                assert sm.conjugate_gradient(U, psi, x, -0.05) == 1
                b = ctypes.c_int(-1)
                sm.check(sm.lib.sm_cg_link_bytes(L.ctx, ctypes.byref(b)))
                out[(loop, on)] = (flat(x), b.value)
        finally:
            L.close()
    assert out[(True, 1)][1] == out[(False, 1)][1] == (20 if drift else 17), out
    assert out[(True, 0)][1] == 32
    assert bits_equal(out[(True, 1)][0], out[(True, 0)][0])
    assert bits_equal(out[(False, 1)][0], out[(False, 0)][0])
    assert np.linalg.norm(out[(True, 1)][0] - out[(False, 1)][0]) / np.linalg.norm(out[(False, 1)][0]) <= 1e-12


def test_link_codes_after_hmc_trajectories(sm):
    """links after HMC updates (U <- U exp(i eps P),
    src/hmc.cpp:69-99, never re-unitarised, so |U| drifts by rounding). After
    10, 20, ... 50 trajectories (sm_hmc_trajectory, 10 MD steps each) every
    link is still rebuilt bitwise, the solve uses the codes, and its x is
    bitwise the complex-link solve's. (Round 4's codes, accepted within
    2^-51, had dropped out after 20 trajectories.)"""
    Nx, Nt = 64, 64
    S = Nx * Nt
    L = sm.init(Nx, Nt)
    sm.check(sm.lib.sm_tune_cg(L.ctx, 5, 0))
    prm = sm.HMCParams(m0=0.0, beta=2.0, tau=1.0, md_steps=10, cg_tol=1e-10, cg_max_iter=10000, seed=99,
                       even_odd=0)
    P = lambda a: a.ctypes.data  # noqa: E731
    U, psi = sm.spinor(S), sm.spinor(S)
    sm.lib.sm_fill_gauge(4321, 0.4242, Nt, 0, Nx, 0, Nt, P(U.mu0), P(U.mu1))
    sm.lib.sm_fill_spinor(13, Nt, 0, Nx, 0, Nt, P(psi.mu0), P(psi.mu1))
    sm.check(sm.lib.sm_upload_gauge(L.ctx, P(U.mu0), P(U.mu1)))
    seen = []
    try:
        for block in range(5):
            for t in range(10):
                res = sm.HMCResult()
                sm.check(sm.lib.sm_hmc_trajectory(L.ctx, ctypes.byref(prm), 10 * block + t, ctypes.byref(res)))
            err, bad = _code_check(sm, L)
            cur = sm.spinor(S)
            sm.check(sm.lib.sm_download_gauge(L.ctx, P(cur.mu0), P(cur.mu1)))
            mod = np.abs(np.concatenate([cur.mu0, cur.mu1])) ** 2 - 1.0
            xs = {}
            for on in (1, 0):
                sm.check(sm.lib.sm_cg_link_codes(L.ctx, on, None))
                x = sm.spinor(S)
                assert sm.conjugate_gradient(cur, psi, x, 0.0) == 1
                u = ctypes.c_int(-1)
                sm.check(sm.lib.sm_cg_link_codes(L.ctx, -1, ctypes.byref(u)))
                xs[on] = (flat(x), u.value)
            seen.append((10 * (block + 1), float(np.abs(mod).max()), bad))
            assert bad == 0 and err == 0.0, seen
            assert xs[1][1] == 1, seen
            assert bits_equal(xs[1][0], xs[0][0])
    finally:
        sm.check(sm.lib.sm_cg_link_codes(L.ctx, 1, None))
    print("after (trajectories, max | |U|^2 - 1 |, links not encodable):", seen)


@pytest.mark.parametrize("wpb,xchunk", [(1, 0), (2, 0), (1, 5), (2, 64), (4, 40), (1, 300)])
def test_recompute_launch_geometries_agree(sm, wpb, xchunk):
    """The recompute-Ad pass under every launch geometry sm_tune_cg_geometry
    offers (one-, two- and four-wave blocks; chunks shorter than the halo,
    longer than the lattice) solves to the same iteration count and x as the
    stored-Ad pass (the reduction-order band). 200 x 150 sites: 3 waves of 56
    columns, the last one partial."""
    Nx, Nt = 200, 150
    S = Nx * Nt
    L = sm.init(Nx, Nt)
    U, psi = sm.spinor(S), sm.spinor(S)
    P = lambda a: a.ctypes.data  # noqa: E731
    sm.lib.sm_fill_gauge(4321, 0.4242, Nt, 0, Nx, 0, Nt, P(U.mu0), P(U.mu1))
    sm.lib.sm_fill_spinor(5678, Nt, 0, Nx, 0, Nt, P(psi.mu0), P(psi.mu1))
    out = {}
    for fused in (4, 5):
        sm.check(sm.lib.sm_tune_cg(L.ctx, fused, 0))
        if fused == 5:
            sm.check(sm.lib.sm_tune_cg_geometry(L.ctx, wpb, xchunk))
        x = sm.spinor(S)
        assert sm.conjugate_gradient(U, psi, x, -0.12) == 1
        out[fused] = (flat(x), L.last_cg.iterations)
    assert abs(out[5][1] - out[4][1]) <= 1, (out[5][1], out[4][1])
    rel = np.linalg.norm(out[5][0] - out[4][0]) / np.linalg.norm(out[4][0])
    assert rel <= 1e-11, rel
    assert sm.lib.sm_tune_cg_geometry(L.ctx, 3, 0) != 0  # 1, 2 or 4 waves only
