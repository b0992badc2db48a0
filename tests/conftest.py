import ctypes
import json
import os
import subprocess

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs under gpurun)")
    config.addinivalue_line("markers", "multiproc: runs several worker processes on the one GPU")


@pytest.fixture(scope="session")
def oracle():
    """ctypes handle on oracle/liboracle.so (built on demand; test checker only)."""
    path = os.path.join(REPO, "oracle", "liboracle.so")
    src = os.path.join(REPO, "oracle", "sm_oracle.c")
    if not os.path.exists(path) or os.path.getmtime(path) < os.path.getmtime(src):
        subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle"), "oracle"], check=True)
    lib = ctypes.CDLL(path)
    vp, ci, cd = ctypes.c_void_p, ctypes.c_int, ctypes.c_double
    lib.oracle_dirac.argtypes = [ci, ci, vp, vp, vp, vp, vp, vp, cd, ci]
    lib.oracle_dirac_local.argtypes = [ci, ci, ci, ci, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, cd, ci]
    lib.oracle_ddag.argtypes = [ci, ci, vp, vp, vp, vp, vp, vp, vp, vp, cd]
    lib.oracle_force.argtypes = [ci, ci, vp, vp, vp, vp, vp, vp, vp, vp]
    lib.oracle_dot.argtypes = [ctypes.c_long, vp, vp, vp, vp, vp]
    lib.oracle_cdiv.argtypes = [cd, cd, cd, cd, vp, vp]
    lib.oracle_cg.argtypes = [ci, ci, vp, vp, vp, vp, vp, vp, cd, cd, ci,
                              ctypes.POINTER(ci), ctypes.POINTER(cd)]
    lib.oracle_cg.restype = ci
    lib.oracle_dirac_mt.argtypes = [ci, ci, vp, vp, vp, vp, vp, vp, cd, ci, ci]
    lib.oracle_plaquette.argtypes = [ci, ci, vp, vp, vp]
    lib.oracle_plaquette_sums.argtypes = [ci, ci, vp, vp, cd, vp, vp]
    lib.oracle_staples.argtypes = [ci, ci, vp, vp, vp, vp]
    lib.oracle_gauge_force.argtypes = [ci, ci, vp, vp, cd, vp, vp]
    lib.oracle_md_force.argtypes = [ci, ci, vp, vp, vp, vp, cd, cd, cd, ci, vp, vp, ctypes.POINTER(ci)]
    lib.oracle_md_force.restype = ci
    lib.oracle_leapfrog.argtypes = [ci, ci, vp, vp, vp, vp, vp, vp, cd, cd, cd, ci, cd, ci,
                                    ctypes.POINTER(ctypes.c_long)]
    lib.oracle_leapfrog.restype = ci
    lib.oracle_hamiltonian.argtypes = [ci, ci, vp, vp, vp, vp, vp, vp, cd, cd, cd, ci, ctypes.POINTER(ci)]
    lib.oracle_hamiltonian.restype = cd
    return lib


def load_manifest():
    with open(os.path.join(GOLDEN, "manifest.json")) as f:
        return json.load(f)


def load_fixture(name):
    meta = load_manifest()["fixtures"][name]
    with np.load(os.path.join(GOLDEN, meta["file"]), allow_pickle=False) as z:
        arrs = {k: z[k].copy() for k in z.files}
    return meta, arrs


def fixture_names():
    return sorted(load_manifest()["fixtures"].keys())


def load_md_fixture(name):
    meta = load_manifest()["md"][name]
    with np.load(os.path.join(GOLDEN, meta["file"]), allow_pickle=False) as z:
        arrs = {k: z[k].copy() for k in z.files}
    return meta, arrs


def md_fixture_names():
    return sorted(load_manifest().get("md", {}).keys())


def sm_opts(**kw):
    """Environment of the library's test-only switches: ONE variable,
    SM_TEST_OPTS="key=value,...", read when a context is created
    (schwingermodel_amd/csrc/sm_capi.cpp apply_test_opts lists the keys)."""
    return {"SM_TEST_OPTS": ",".join(f"{k}={v}" for k, v in kw.items())} if kw else {}


class opts_env:
    """Context manager: SM_TEST_OPTS set to **kw while a context is created."""

    def __init__(self, **kw):
        self.env = sm_opts(**kw)

    def __enter__(self):
        self.old = os.environ.get("SM_TEST_OPTS")
        os.environ.pop("SM_TEST_OPTS", None)
        os.environ.update(self.env)
        return self

    def __exit__(self, *exc):
        os.environ.pop("SM_TEST_OPTS", None)
        if self.old is not None:
            os.environ["SM_TEST_OPTS"] = self.old
        return False


def ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def planes(a, S):
    """Split a two-plane interleaved-complex field into its (mu0, mu1) views."""
    return a[: 2 * S], a[2 * S: 4 * S]


def bits_equal(a, b):
    return a.shape == b.shape and np.array_equal(a.view(np.uint64), b.view(np.uint64))
