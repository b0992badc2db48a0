"""Drop-in check: the reference's OWN code calling the GPU path.

oracle/_ref/sm_dropin_<Nx>x<Nt> is oracle/ref_harness.cpp + the reference's
src/variables.cpp linked against our shim schwingermodel_amd/csrc/
dirac_operator_hip.cpp (which replaces src/dirac_operator.cpp and
src/conjugate_gradient.cpp) and libsm_hip.so. Its outputs must equal the
golden vectors the unmodified reference produced: bitwise for D, D^dag,
D D^dag and the force, 1e-12 relative for the CG solution.

oracle/_ref/SM_<Nx>x<Nt>_hip is the reference HMC program (src/main.cpp,
hmc.cpp, gauge_conf.cpp, ...) on the shim: it must run a short simulation to
completion with physical output (statistical check only: the reference seeds
its RNGs from the clock, src/main.cpp:17, src/hmc.cpp:7-8).

Binaries are built by `make -C oracle dropin` in the dev container (they need
the reference sources) and travel to the GPU box in oracle/_ref/.
"""
import os
import subprocess

import numpy as np
import pytest

from conftest import REPO, bits_equal, load_fixture

pytestmark = pytest.mark.gpu
REF = os.path.join(REPO, "oracle", "_ref")
CASES = [("l16x16_b2_m-0p19", "16x16"), ("l32x48_b3_m-0p10", "32x48"), ("l64x64_b2_m0", "64x64")]


def env():
    return dict(os.environ, HOSTNAME=os.environ.get("HOSTNAME", "gpu-box"))


@pytest.mark.parametrize("name,size", CASES)
def test_dropin_harness_matches_reference(tmp_path, name, size):
    exe = os.path.join(REF, f"sm_dropin_{size}")
    if not os.path.exists(exe):
        pytest.skip("drop-in binary not built (needs /root/reference at build time)")
    meta, a = load_fixture(name)
    for k in ("U", "psi", "chi"):
        a[k].tofile(tmp_path / f"{k}.bin")
    r = subprocess.run([exe, "fixture", str(tmp_path), "1", "1", repr(meta["m0"]), "1e-10", "10000"],
                       capture_output=True, text=True, env=env(), timeout=300)
    assert r.returncode == 0, r.stderr
    out = {k: np.fromfile(tmp_path / f"{k}.bin", dtype=np.float64)
           for k in ("ref_Dpsi", "ref_Ddagchi", "ref_DDdagpsi", "ref_force", "ref_cgx")}
    for k in ("ref_Dpsi", "ref_Ddagchi", "ref_DDdagpsi", "ref_force"):
        assert bits_equal(out[k], a[k]), k
    x, xr = out["ref_cgx"], a["ref_cgx"]
    assert np.linalg.norm(x - xr) / np.linalg.norm(xr) <= 1e-12
    assert '"cg_converged": 1' in r.stdout


MPIEXEC = "/opt/conda/bin/mpiexec"


@pytest.mark.multiproc
@pytest.mark.parametrize("rx,rt", [(1, 2), (2, 1), (2, 2), (2, 4)])
def test_dropin_multirank_matches_reference(tmp_path, rx, rt):
    """The reference's own fixture driver on rx x rt MPI ranks (MPICH) over the
    shim: each t-column's ranks gather to their leader, the rt leaders run the
    t-shards of the GPU path (several leaders share this one GPU, so the shim
    picks its MPI host-staged transport), results scattered back. Bitwise
    against the 1-rank reference for D, D^dag, D D^dag and the force (the
    reference itself is decomposition-invariant there), 1e-12 for CG."""
    exe = os.path.join(REF, "sm_dropin_32x48")
    if not os.path.exists(exe) or not os.path.exists(MPIEXEC):
        pytest.skip("drop-in binary or MPICH not available")
    meta, a = load_fixture("l32x48_b3_m-0p10")
    for k in ("U", "psi", "chi"):
        a[k].tofile(tmp_path / f"{k}.bin")
    r = subprocess.run([MPIEXEC, "-n", str(rx * rt), exe, "fixture", str(tmp_path), str(rx), str(rt),
                        repr(meta["m0"]), "1e-10", "10000"], capture_output=True, text=True, env=env(), timeout=150)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    out = {k: np.fromfile(tmp_path / f"{k}.bin", dtype=np.float64)
           for k in ("ref_Dpsi", "ref_Ddagchi", "ref_DDdagpsi", "ref_force", "ref_cgx")}
    for k in ("ref_Dpsi", "ref_Ddagchi", "ref_DDdagpsi", "ref_force"):
        assert bits_equal(out[k], a[k]), k
    x, xr = out["ref_cgx"], a["ref_cgx"]
    assert np.linalg.norm(x - xr) / np.linalg.norm(xr) <= 1e-12
    assert '"cg_converged": 1' in r.stdout


@pytest.mark.multiproc
@pytest.mark.parametrize("rx,rt", [(1, 2), (2, 4)])
def test_dropin_multirank_peer_transport(tmp_path, rx, rt):
    """The same fixture driver with the shim's t-column leaders on the peer
    transport (SM_DROPIN_TRANSPORT=peer: sm_create_peer, the region handles
    all-gathered with MPI_Allgather, sm_peer_connect) -- the binding
    INTEGRATION.md shows -- here with the leaders sharing this one GPU (one
    hardware queue each, as in tests/test_peer_gpu.py)."""
    exe = os.path.join(REF, "sm_dropin_32x48")
    if not os.path.exists(exe) or not os.path.exists(MPIEXEC):
        pytest.skip("drop-in binary or MPICH not available")
    meta, a = load_fixture("l32x48_b3_m-0p10")
    for k in ("U", "psi", "chi"):
        a[k].tofile(tmp_path / f"{k}.bin")
    e = dict(env(), SM_DROPIN_TRANSPORT="peer", GPU_MAX_HW_QUEUES="1")
    r = subprocess.run([MPIEXEC, "-n", str(rx * rt), exe, "fixture", str(tmp_path), str(rx), str(rt),
                        repr(meta["m0"]), "1e-10", "10000"], capture_output=True, text=True, env=e, timeout=150)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    out = {k: np.fromfile(tmp_path / f"{k}.bin", dtype=np.float64)
           for k in ("ref_Dpsi", "ref_Ddagchi", "ref_DDdagpsi", "ref_force", "ref_cgx")}
    for k in ("ref_Dpsi", "ref_Ddagchi", "ref_DDdagpsi", "ref_force"):
        assert bits_equal(out[k], a[k]), k
    x, xr = out["ref_cgx"], a["ref_cgx"]
    assert np.linalg.norm(x - xr) / np.linalg.norm(xr) <= 1e-12
    assert '"cg_converged": 1' in r.stdout


@pytest.mark.multiproc
def test_reference_hmc_program_multirank(tmp_path):
    """The reference HMC program (src/main.cpp) on 2 x 2 MPI ranks over the
    shim: two t-column leaders drive two t-shards on this GPU (MPI host-staged
    transport), the reference's gauge/MD code runs its own 2 x 2 halo
    exchanges. Statistical check against the CPU reference's 1-rank numbers
    (its RNG is clock-seeded, src/main.cpp:17)."""
    exe = os.path.join(REF, "SM_64x64_hip")
    if not os.path.exists(exe) or not os.path.exists(MPIEXEC):
        pytest.skip("drop-in HMC binary or MPICH not available")
    params = "2\n2\n0\n10\n0.3\n2\n30\n20\n1\n0\n"
    r = subprocess.run([MPIEXEC, "-n", "4", exe], input=params, capture_output=True, text=True, env=env(),
                       cwd=tmp_path, timeout=150)
    assert r.returncode == 0, r.stderr[-2000:]
    sim = [f for f in os.listdir(tmp_path) if f.endswith("_SimData.txt")]
    assert sim, r.stdout[-2000:]
    lines = open(tmp_path / sim[0]).read().split("\n")
    ep = float(lines[lines.index("#Ep                           #dEp") + 1].split()[0])
    acc = float(lines[lines.index("#Acceptance rate") + 1].split()[0])
    assert 0.69 < ep < 0.75, (ep, acc)
    assert 0.5 < acc <= 1.0, acc
    assert "did not converge" not in r.stdout


def test_reference_hmc_program_on_gpu(tmp_path):
    exe = os.path.join(REF, "SM_64x64_hip")
    if not os.path.exists(exe):
        pytest.skip("drop-in HMC binary not built")
    # ranks_x ranks_t m0 MD_steps tau beta Ntherm Nmeas Nsteps save (src/main.cpp:33-57).
    # The unmodified CPU reference with these inputs (dev container, 64x64):
    #   Ep = 0.717813 +- 0.00133, acceptance 0.875 (57.6 s). Hot start, so
    #   short thermalisation; the band below is statistical, not bitwise.
    params = "1\n1\n0\n10\n0.3\n2\n30\n20\n1\n0\n"
    r = subprocess.run([exe], input=params, capture_output=True, text=True, env=env(),
                       cwd=tmp_path, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    sim = [f for f in os.listdir(tmp_path) if f.endswith("_SimData.txt")]
    assert sim, r.stdout[-2000:]
    lines = open(tmp_path / sim[0]).read().split("\n")
    ep = float(lines[lines.index("#Ep                           #dEp") + 1].split()[0])
    acc = float(lines[lines.index("#Acceptance rate") + 1].split()[0])
    assert 0.69 < ep < 0.75, (ep, acc)
    assert 0.5 < acc <= 1.0, acc
    assert "did not converge" not in r.stdout
