"""Pin the oracle's gauge / molecular-dynamics restatement to the reference.

Fixtures (tests/golden/md*.npz, make_golden.py MD_FIXTURES) hold the outputs
of the unmodified reference's src/gauge_conf.cpp and src/hmc.cpp on seeded
U, chi and momenta P: plaquette field and sums, staples, Force_G, Force (CG +
fermion bilinear + gauge force), phi = D chi, Leapfrog -> (U', P') and the
Hamiltonian before and after. The oracle reproduces every one BIT FOR BIT
(the leapfrog's std::exp is glibc cexp in both).
"""
import ctypes

import numpy as np
import pytest

from conftest import bits_equal, load_md_fixture, md_fixture_names, planes, ptr

NAMES = md_fixture_names()
TOL, MAXIT = 1e-10, 10000


def setup(name):
    meta, a = load_md_fixture(name)
    return meta, a, meta["Nx"], meta["Nt"], meta["Nx"] * meta["Nt"]


@pytest.mark.parametrize("name", NAMES)
def test_plaquette_bitwise(oracle, name):
    meta, a, Nx, Nt, S = setup(name)
    U0, U1 = planes(a["U"], S)
    P = np.empty(2 * S)
    oracle.oracle_plaquette(Nx, Nt, ptr(U0), ptr(U1), ptr(P))
    assert bits_equal(P, a["ref_plaq"])
    sp, act = ctypes.c_double(), ctypes.c_double()
    oracle.oracle_plaquette_sums(Nx, Nt, ptr(U0), ptr(U1), meta["beta"], ctypes.byref(sp), ctypes.byref(act))
    assert sp.value == meta["sp"] and act.value == meta["gauge_action"]


@pytest.mark.parametrize("name", NAMES)
def test_staples_and_gauge_force_bitwise(oracle, name):
    meta, a, Nx, Nt, S = setup(name)
    U0, U1 = planes(a["U"], S)
    St = np.empty(4 * S)
    oracle.oracle_staples(Nx, Nt, ptr(U0), ptr(U1), ptr(St[:2 * S]), ptr(St[2 * S:]))
    assert bits_equal(St, a["ref_staple"])
    F = np.zeros(2 * S)
    oracle.oracle_gauge_force(Nx, Nt, ptr(U0), ptr(U1), meta["beta"], ptr(F[:S]), ptr(F[S:]))
    assert bits_equal(F, a["ref_gforce"])


@pytest.mark.parametrize("name", NAMES)
def test_md_force_bitwise(oracle, name):
    meta, a, Nx, Nt, S = setup(name)
    U0, U1 = planes(a["U"], S)
    c0, c1 = planes(a["chi"], S)
    phi = np.empty(4 * S)
    oracle.oracle_dirac(Nx, Nt, ptr(U0), ptr(U1), ptr(c0), ptr(c1), ptr(phi[:2 * S]), ptr(phi[2 * S:]),
                        meta["m0"], 0)
    assert bits_equal(phi, a["ref_phi"])
    F = np.empty(2 * S)
    it = ctypes.c_int()
    assert oracle.oracle_md_force(Nx, Nt, ptr(U0), ptr(U1), ptr(phi[:2 * S]), ptr(phi[2 * S:]), meta["m0"],
                                  meta["beta"], TOL, MAXIT, ptr(F[:S]), ptr(F[S:]), ctypes.byref(it)) == 1
    assert it.value == meta["force_cg_iters"]
    assert bits_equal(F, a["ref_mdforce"])


@pytest.mark.parametrize("name", NAMES)
def test_leapfrog_and_hamiltonian_bitwise(oracle, name):
    meta, a, Nx, Nt, S = setup(name)
    phi = a["ref_phi"]
    p0, p1 = planes(phi, S)
    U, P = a["U"].copy(), a["P"].copy()
    it = ctypes.c_int()
    H0 = oracle.oracle_hamiltonian(Nx, Nt, ptr(U[:2 * S]), ptr(U[2 * S:]), ptr(P[:S]), ptr(P[S:]), ptr(p0),
                                   ptr(p1), meta["m0"], meta["beta"], TOL, MAXIT, ctypes.byref(it))
    assert H0 == meta["H0"]
    cg = ctypes.c_long()
    assert oracle.oracle_leapfrog(Nx, Nt, ptr(U[:2 * S]), ptr(U[2 * S:]), ptr(P[:S]), ptr(P[S:]), ptr(p0), ptr(p1),
                                  meta["m0"], meta["beta"], meta["tau"], meta["md_steps"], TOL, MAXIT,
                                  ctypes.byref(cg)) == 1
    assert bits_equal(U, a["ref_U1"]) and bits_equal(P, a["ref_P1"])
    # every CG solve = its loop passes + 1 initial D D^dag call
    assert cg.value + (meta["md_steps"] - 1) == meta["leapfrog_ddag_calls"]
    H1 = oracle.oracle_hamiltonian(Nx, Nt, ptr(U[:2 * S]), ptr(U[2 * S:]), ptr(P[:S]), ptr(P[S:]), ptr(p0),
                                   ptr(p1), meta["m0"], meta["beta"], TOL, MAXIT, ctypes.byref(it))
    assert H1 == meta["H1"]
