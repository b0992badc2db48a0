"""Pin the CPU oracle (oracle/sm_oracle.c) to the reference's own outputs.

The golden vectors were produced by the unmodified reference sources
(tests/golden/make_golden.py); the oracle must reproduce every one BIT FOR BIT,
including the CG iterate sequence (iteration count and solution).
"""
import ctypes

import numpy as np
import pytest

from conftest import bits_equal, fixture_names, load_fixture, planes, ptr

NAMES = fixture_names()


@pytest.mark.parametrize("name", NAMES)
def test_dirac_bitwise(oracle, name):
    meta, a = load_fixture(name)
    Nx, Nt, m0 = meta["Nx"], meta["Nt"], meta["m0"]
    S = Nx * Nt
    U0, U1 = planes(a["U"], S)
    for inp, ref, dag in ((a["psi"], a["ref_Dpsi"], 0), (a["chi"], a["ref_Ddagchi"], 1)):
        out = np.empty(4 * S)
        i0, i1 = planes(inp, S)
        o0, o1 = planes(out, S)
        oracle.oracle_dirac(Nx, Nt, ptr(U0), ptr(U1), ptr(i0), ptr(i1), ptr(o0), ptr(o1), m0, dag)
        assert bits_equal(out, ref), (name, dag, np.abs(out - ref).max())


@pytest.mark.parametrize("name", NAMES)
def test_ddag_bitwise(oracle, name):
    meta, a = load_fixture(name)
    Nx, Nt, m0 = meta["Nx"], meta["Nt"], meta["m0"]
    S = Nx * Nt
    U0, U1 = planes(a["U"], S)
    tmp, out = np.empty(4 * S), np.empty(4 * S)
    i0, i1 = planes(a["psi"], S)
    t0, t1 = planes(tmp, S)
    o0, o1 = planes(out, S)
    oracle.oracle_ddag(Nx, Nt, ptr(U0), ptr(U1), ptr(i0), ptr(i1), ptr(t0), ptr(t1), ptr(o0), ptr(o1), m0)
    assert bits_equal(out, a["ref_DDdagpsi"])


@pytest.mark.parametrize("name", NAMES)
def test_force_bitwise(oracle, name):
    meta, a = load_fixture(name)
    Nx, Nt = meta["Nx"], meta["Nt"]
    S = Nx * Nt
    U0, U1 = planes(a["U"], S)
    l0, l1 = planes(a["psi"], S)
    r0, r1 = planes(a["chi"], S)
    F = np.empty(2 * S)
    oracle.oracle_force(Nx, Nt, ptr(U0), ptr(U1), ptr(l0), ptr(l1), ptr(r0), ptr(r1), ptr(F[:S]), ptr(F[S:]))
    assert bits_equal(F, a["ref_force"])


@pytest.mark.parametrize("name", NAMES)
def test_cg_bitwise(oracle, name):
    meta, a = load_fixture(name)
    Nx, Nt, m0 = meta["Nx"], meta["Nt"], meta["m0"]
    S = Nx * Nt
    U0, U1 = planes(a["U"], S)
    p0, p1 = planes(a["psi"], S)
    x = np.empty(4 * S)
    x0, x1 = planes(x, S)
    it, err = ctypes.c_int(), ctypes.c_double()
    conv = oracle.oracle_cg(Nx, Nt, ptr(U0), ptr(U1), ptr(p0), ptr(p1), ptr(x0), ptr(x1),
                            m0, 1e-10, 10000, ctypes.byref(it), ctypes.byref(err))
    assert conv == meta["cg_converged"] == 1
    assert it.value == meta["cg_iters"]
    assert bits_equal(x, a["ref_cgx"])


@pytest.mark.parametrize("name", NAMES)
def test_dot_adjointness(oracle, name):
    """<chi, D psi> = <D^dag chi, psi>: the reference's own dot values."""
    meta, a = load_fixture(name)
    S = meta["Nx"] * meta["Nt"]
    z1, z2 = np.empty(2), np.empty(2)
    c0, c1 = planes(a["chi"], S)
    d0, d1 = planes(a["ref_Dpsi"], S)
    oracle.oracle_dot(S, ptr(c0), ptr(c1), ptr(d0), ptr(d1), ptr(z1))
    assert bits_equal(z1, np.array(meta["dot_chi_Dpsi"]))
    e0, e1 = planes(a["ref_Ddagchi"], S)
    p0, p1 = planes(a["psi"], S)
    oracle.oracle_dot(S, ptr(e0), ptr(e1), ptr(p0), ptr(p1), ptr(z2))
    assert bits_equal(z2, np.array(meta["dot_Ddagchi_psi"]))
    assert abs(complex(*z1) - complex(*z2)) <= 1e-13 * abs(complex(*z1))


def test_cdiv_matches_python_smith(oracle):
    re, im = ctypes.c_double(), ctypes.c_double()
    oracle.oracle_cdiv(3.0, 0.0, 1.5, 0.0, ctypes.byref(re), ctypes.byref(im))
    assert (re.value, im.value) == (2.0, 0.0)
    oracle.oracle_cdiv(1.0, 2.0, 3.0, 4.0, ctypes.byref(re), ctypes.byref(im))
    assert abs(complex(re.value, im.value) - (1 + 2j) / (3 + 4j)) < 1e-16


@pytest.mark.parametrize("name", ["l16x16_b2_m-0p19", "l32x48_b3_m-0p10"])
def test_reference_decomposition_invariance_recorded(name):
    """make_golden.py --mpi recorded that the reference is bitwise
    decomposition-invariant for D, D^dag, DD^dag and the force (2x2 ranks)."""
    meta, _ = load_fixture(name)
    dec = meta.get("decomposition_2x2")
    if dec is None:
        pytest.skip("fixtures generated without --mpi")
    for k in ("ref_Dpsi", "ref_Ddagchi", "ref_DDdagpsi", "ref_force"):
        assert dec[k] == "bitwise"
    assert dec["cg_iters_2x2"] == meta["cg_iters"]
