"""The device-initiated shard transport ("peer", sm_peer.h) on ONE GPU.

Each shard owns an uncached region; kernels store faces and scalar sums
straight into the neighbours' / every shard's region and wait on sequence
flags in their own. Two ways to run it on one MI355X:

* the peer loopback (sm_create_peer_loopback): one shard, its own neighbour on
  both sides -- every face goes out and back through the region, every sum
  through the in-kernel all-reduce, the CG pass is the one-launch peer pass.
  The self-sent faces are the shard's periodic wrap, so D, D^dag, D D^dag, the
  force and the gauge force equal the one-shard context bitwise, and CG takes
  the same iterations with x within 1e-13;
* 2 / 4 / 8 PROCESSES on the one GPU, each a t-shard, each mapping the others'
  regions through hipIpcOpenMemHandle (RCCL refuses two ranks on one GPU; the
  peer transport does not need it): the same checks as the host-staged worlds
  of test_dist_gpu.py, against the reference's golden vectors.
"""
import ctypes

import numpy as np
import pytest

from conftest import bits_equal, sm_opts
from distutil import run_world
from test_rccl_loopback_gpu import fields, run_all

pytestmark = pytest.mark.gpu

# One hardware queue per worker process: 2-8 processes share the one GPU here, and
# each spins one wave in a publishing kernel until the others' kernels have run.
# With several queues per process the GPU's hardware queue slots run out at 8
# processes and the scheduler time-slices whole queues, which can stretch a
# wait by orders of magnitude (a round-6 8-process run hit the time limits).
# Production runs one process per GPU.
PEER = {"SM_WORKER_TRANSPORT": "peer", "GPU_MAX_HW_QUEUES": "1"}


@pytest.fixture(scope="module")
def sm():
    import schwingermodel_amd
    return schwingermodel_amd


def test_peer_loopback_comm_info(sm):
    L = sm.Lattice(32, 48, loopback="peer")
    try:
        assert L.comm_info() == ("peer", 1, 0)
        t = ctypes.c_ulonglong(7)
        sm.check(sm.lib.sm_peer_status(L.ctx, ctypes.byref(t)))
        assert t.value == 0
    finally:
        L.close()


CASES = [
    ((32, 48), 0.0, -0.10, "l32x48_b3_m-0p10"),
    ((96, 1024), 0.3246, -0.08, None),
    ((64, 4096), 0.2374, -0.06, None),
    # the narrowest shards of the recompute-Ad pass: Wt 4 (lo and hi face
    # columns overlap: faces by exchange every pass) and 8 (stored by the pass)
    ((64, 4), 0.4, -0.05, None),
    ((64, 8), 0.4, -0.05, None),
]


@pytest.mark.parametrize("shape,sigma,m0,fixture", CASES, ids=["32x48_fixture", "96x1024", "64x4096", "64x4", "64x8"])
def test_peer_loopback_equals_one_shard(sm, shape, sigma, m0, fixture):
    Nx, Nt = shape
    S = Nx * Nt
    U, psi, chi, gold = fields(sm, Nx, Nt, sigma, fixture)
    one = sm.Lattice(Nx, Nt)
    ref = run_all(sm, one, U, psi, chi, m0, S)
    one.close()
    loop = sm.Lattice(Nx, Nt, loopback="peer")
    got = run_all(sm, loop, U, psi, chi, m0, S)
    sm.check(sm.lib.sm_peer_status(loop.ctx, None))
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


def test_peer_loopback_hmc_trajectory_and_even_odd(sm):
    """HMC trajectories (ghost links re-exchanged after every link update, the
    Metropolis restore) and the even-odd CG through the peer loopback equal the
    one-shard context."""
    Nx, Nt = 64, 64
    S = Nx * Nt
    U, psi, chi, _ = fields(sm, Nx, Nt, 0.4242)
    res = {}
    for name, kw in (("one", {}), ("peer", {"loopback": "peer"})):
        L = sm.Lattice(Nx, Nt, **kw)
        sm.check(sm.lib.sm_upload_gauge(L.ctx, ctypes.c_void_p(U[:2 * S].ctypes.data),
                                        ctypes.c_void_p(U[2 * S:].ctypes.data)))
        x = np.empty(4 * S)
        cg = sm.CGResult()
        P = lambda a: ctypes.c_void_p(a.ctypes.data)  # noqa: E731
        sm.check(sm.lib.sm_eo_cg(L.ctx, P(psi[:2 * S]), P(psi[2 * S:]), P(x[:2 * S]), P(x[2 * S:]),
                                 -0.05, 1e-10, 10000, ctypes.byref(cg)))
        prm = sm.HMCParams(0.0, 2.0, 0.5, 5, 1e-10, 10000, 7)
        trajs = []
        for t in range(3):
            r = sm.HMCResult()
            sm.check(sm.lib.sm_hmc_trajectory(L.ctx, ctypes.byref(prm), t, ctypes.byref(r)))
            trajs.append((r.dH, r.accepted, r.cg_iterations, r.cg_failures))
        Uo = np.empty(4 * S)
        sm.check(sm.lib.sm_download_gauge(L.ctx, P(Uo[:2 * S]), P(Uo[2 * S:])))
        sm.check(sm.lib.sm_peer_status(L.ctx, None))
        res[name] = (x, cg.iterations, cg.converged, trajs, Uo)
        L.close()
    x1, it1, c1, tr1, U1 = res["one"]
    x2, it2, c2, tr2, U2 = res["peer"]
    assert c1 == c2 == 1 and it1 == it2
    assert np.linalg.norm(x2 - x1) / np.linalg.norm(x1) <= 1e-13
    for a, b in zip(tr1, tr2):
        assert a[1:] == b[1:], (a, b)
        assert abs(a[0] - b[0]) <= 1e-9 * max(1.0, abs(a[0])), (a, b)
    assert np.linalg.norm(U2 - U1) / np.linalg.norm(U1) <= 1e-12


def test_peer_loopback_cg_after_nan_solve(sm):
    """A NaN solve must not poison the next one: the peer pass 0 reads d_0's
    faces from a fresh exchange into ring slot 2, never an older slot."""
    Nx, Nt = 64, 4096
    S = Nx * Nt
    U, psi, _, _ = fields(sm, Nx, Nt, 0.2374)
    P = lambda a: ctypes.c_void_p(a.ctypes.data)  # noqa: E731
    h = lambda a: (P(a[:2 * S]), P(a[2 * S:]))  # noqa: E731
    its = {}
    for name, kw in (("one", {}), ("peer", {"loopback": "peer"})):
        L = sm.Lattice(Nx, Nt, **kw)
        sm.check(sm.lib.sm_upload_gauge(L.ctx, *h(U)))
        sm.check(sm.lib.sm_tune_cg(L.ctx, 5, 0))
        bad = np.full(4 * S, np.nan)
        x = np.empty(4 * S)
        res = sm.CGResult()
        sm.lib.sm_cg(L.ctx, *h(bad), *h(x), -0.06, 1e-10, 6, ctypes.byref(res))
        assert res.converged == 0
        sm.check(sm.lib.sm_cg(L.ctx, *h(psi), *h(x), -0.06, 1e-10, 10000, ctypes.byref(res)))
        its[name] = (res.converged, res.iterations, x.copy())
        L.close()
    assert its["peer"][0] == its["one"][0] == 1 and its["peer"][1] == its["one"][1]
    assert np.linalg.norm(its["peer"][2] - its["one"][2]) / np.linalg.norm(its["one"][2]) <= 1e-13


# ---- several processes on the one GPU, each mapping the others' regions ----

@pytest.mark.multiproc
@pytest.mark.parametrize("fixture,world", [("l64x64_b2_m0", 2), ("l32x48_b3_m-0p10", 4),
                                           ("l64x64_b5_m-0p06", 4), ("gen:48x1024:0.3:-0.05", 2),
                                           ("gen:32x960:0.4242:0.0", 4), ("l64x64_b5_m-0p06", 8)])
def test_peer_world_matches_reference(tmp_path, fixture, world):
    """D, D^dag, D D^dag and the force bitwise against the reference; CG (the
    one-launch peer pass) in the reference's iterations to 1e-12; the same dot
    on every shard; sm_comm_info = (peer, world, rank)."""
    rep = run_world("gpu", fixture, world, tmp_path, timeout=220, extra_env=PEER)
    c = rep["checks"]
    for k in ("ref_Dpsi", "ref_Ddagchi", "ref_DDdagpsi", "ref_force"):
        assert c[k] is True, (k, c)
    assert c["ref_cgx"] <= 1e-12
    ref = rep["ref_cg_iters"]
    assert len(set(rep["cg_iters"])) == 1 and abs(rep["cg_iters"][0] - ref) <= max(1, ref // 100)
    assert all(rep["cg_converged"])
    assert len({tuple(d) for d in rep["dots"]}) == 1
    assert rep["comm_info"] == [[3, world, r] for r in range(world)], rep["comm_info"]
    assert rep["sums_in_pass"] == [1] * world, rep["sums_in_pass"]


@pytest.mark.multiproc
@pytest.mark.parametrize("cg,fixture,world", [(4, "l32x48_b3_m-0p10", 4), (0, "l64x64_b2_m0", 2),
                                              (5, "l16x16_b2_m-0p19", 4)])
def test_peer_world_other_cg_paths(tmp_path, cg, fixture, world):
    """The stored-Ad pass (2-deep faces of three fields in one exchange), the
    reference's six-launch sequence and the narrowest recompute-Ad shard (Wt 4)
    over the peer transport."""
    rep = run_world("gpu", fixture, world, tmp_path, timeout=160, extra_env=dict(PEER, **sm_opts(cg=cg)))
    assert rep["checks"]["ref_cgx"] <= 1e-12
    ref = rep["ref_cg_iters"]
    assert len(set(rep["cg_iters"])) == 1 and abs(rep["cg_iters"][0] - ref) <= max(1, ref // 100)
    assert all(rep["cg_converged"])


@pytest.mark.multiproc
@pytest.mark.parametrize("fixture,world", [("md32x48_b3_m0p1", 4), ("md64x64_b2_m0", 2)])
def test_peer_world_md(tmp_path, fixture, world):
    """The MD layer (plaquette, staples, gauge force, MD force, leapfrog,
    Hamiltonians, an HMC trajectory) on t-shards over the peer transport, with
    the bars of test_dist_gpu.py's host-staged worlds."""
    rep = run_world("md", fixture, world, tmp_path, timeout=160, extra_env=PEER)
    c = rep["checks"]
    for k in ("ref_plaq", "ref_staple", "ref_gforce"):
        assert c[k] is True, (k, c)
    for k in ("ref_mdforce", "ref_U1", "ref_P1"):
        assert c[k] <= 1e-8, (k, c)
    m = rep["meta"]
    assert len({tuple(s) for s in rep["sums"]}) == 1
    sp, act = rep["sums"][0]
    assert abs(sp - m["sp"]) <= 1e-12 * max(1.0, abs(m["sp"])) and abs(act - m["gauge_action"]) <= 1e-12 * m["gauge_action"]
    for key in ("H0", "H1"):
        assert len(set(rep[key])) == 1 and abs(rep[key][0] - m[key]) <= 1e-10 * abs(m[key])
    t = rep["traj"]
    assert len({tuple(x) for x in t["sharded"]}) == 1
    dH, acc, r = t["sharded"][0]
    assert abs(dH - t["single"][0]) <= 1e-6 * max(1.0, abs(t["single"][0]))
    assert acc == t["single"][1] and r == t["single"][2]
    assert t["U_rel"] <= 1e-8


@pytest.mark.multiproc
def test_peer_wait_time_limit(tmp_path):
    """A shard whose neighbour never takes part does not hang: its wait gives up
    at the time limit (here 2 s, SM_TEST_OPTS peer_wait_ms), sm_peer_status
    names the sequence number, and the solve that follows on the same context
    fails within seconds (every later wait gives up at once) with the peer
    error instead of waiting 10 s per pass."""
    env = dict(PEER, **sm_opts(peer_wait_ms=2000))
    rep = run_world("peerfail", "l32x48_b3_m-0p10", 2, tmp_path, timeout=120, extra_env=env)
    assert rep["status_rc"] != 0 and "timed out" in rep["status_msg"] and rep["timed_out_seq"] > 0, rep
    assert rep["apply_s"] < 30, rep
    assert rep["cg_rc"] != 0 and "peer transport" in rep["cg_msg"], rep
    assert rep["cg_s"] < 30, rep


@pytest.mark.multiproc
@pytest.mark.parametrize("fixture,world", [("gen:48x1024:0.3:-0.05", 2), ("gen:32x960:0.4242:0.0", 4),
                                           ("l64x64_b5_m-0p06", 4), ("l16x16_b2_m-0p19", 4)])
def test_in_pass_sums_on_split_launches(tmp_path, fixture, world):
    """The RCCL path's in-pass CG sums (rccl_peer_sums_setup: the pass's last
    block all-reduces through peer headers, no all-reduce call per pass) with
    several shards, on the host-staged transport that runs the same split
    interior / edge launches (test option hosted_psums=1; RCCL itself refuses
    two ranks on one GPU): the reference's iterations and solution, and
    bitwise operators (the sums path does not touch them)."""
    env = dict(sm_opts(hosted_psums=1, cg=5), GPU_MAX_HW_QUEUES="1")
    rep = run_world("gpu", fixture, world, tmp_path, timeout=200, extra_env=env)
    c = rep["checks"]
    for k in ("ref_Dpsi", "ref_Ddagchi", "ref_DDdagpsi", "ref_force"):
        assert c[k] is True, (k, c)
    assert c["ref_cgx"] <= 1e-12
    ref = rep["ref_cg_iters"]
    assert len(set(rep["cg_iters"])) == 1 and abs(rep["cg_iters"][0] - ref) <= max(1, ref // 100)
    assert all(rep["cg_converged"])
    assert rep["sums_in_pass"] == [1] * world, rep["sums_in_pass"]  # the in-pass sums really ran
