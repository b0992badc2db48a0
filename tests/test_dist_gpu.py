"""World-size > 1 on ONE GPU: the sharded HIP path through the host transport.

2-4 processes share cuda:0, each owning a t-shard (sm_create_hosted + gloo).
Same kernels, face packing, ghost links, antiperiodic-sign ownership and
scalar all-reduces as the RCCL path; only the wire differs. D, D^dag, D D^dag
and the force must equal the reference bitwise; CG must converge in the
reference's iteration count (+-1 %) to 1e-12 relative.
"""
import pytest

from conftest import sm_opts
from distutil import run_world

pytestmark = [pytest.mark.gpu, pytest.mark.multiproc]


@pytest.mark.parametrize("fixture,world", [("l64x64_b2_m0", 2), ("l32x48_b3_m-0p10", 4),
                                           ("l64x64_b5_m-0p06", 4),
                                           # Wt = 512 / 240: the fused CG runs interior and edge
                                           # t-blocks as separate launches (halo overlap path);
                                           # reference = one shard on the same GPU
                                           ("gen:48x1024:0.3:-0.05", 2), ("gen:32x960:0.4242:0.0", 4)])
def test_sharded_gpu_path_matches_reference(tmp_path, fixture, world):
    # bt = 64 so the Dirac apply of the larger shards also splits into interior
    # and edge t-blocks (the overlapped halo path)
    env = sm_opts(bt=64) if fixture.startswith("gen:") else None
    rep = run_world("gpu", fixture, world, tmp_path, timeout=140, extra_env=env)
    c = rep["checks"]
    for k in ("ref_Dpsi", "ref_Ddagchi", "ref_DDdagpsi", "ref_force"):
        assert c[k] is True, (k, c)
    assert c["ref_cgx"] <= 1e-12
    ref = rep["ref_cg_iters"]
    assert len(set(rep["cg_iters"])) == 1 and abs(rep["cg_iters"][0] - ref) <= max(1, ref // 100)
    assert all(rep["cg_converged"])
    assert len({tuple(d) for d in rep["dots"]}) == 1  # identical global dot on every shard
    # sm_comm_info: host-staged transport, no RCCL world (bench.py's rccl_ranks = 1)
    assert rep["comm_info"] == [[1, 1, 0]] * world, rep["comm_info"]
    assert rep["sums_in_pass"] == [0] * world  # host-staged default: the transport's all-reduce


@pytest.mark.parametrize("fixture,world", [("l32x48_b3_m-0p10", 4), ("gen:48x1024:0.3:-0.05", 2)])
def test_sharded_twodir_cg_matches_reference(tmp_path, fixture, world):
    """The two-direction CG (test option cg=4: d_{j-2} faces instead of r faces)
    on t-shards: the reference's iteration count and solution."""
    rep = run_world("gpu", fixture, world, tmp_path, timeout=140, extra_env=sm_opts(cg=4))
    assert rep["checks"]["ref_cgx"] <= 1e-12
    ref = rep["ref_cg_iters"]
    assert len(set(rep["cg_iters"])) == 1 and abs(rep["cg_iters"][0] - ref) <= max(1, ref // 100)
    assert all(rep["cg_converged"])


@pytest.mark.parametrize("fixture,world", [("l32x48_b3_m-0p10", 4), ("l64x64_b5_m-0p06", 2),
                                           ("gen:48x1024:0.3:-0.05", 2), ("gen:32x960:0.4242:0.0", 4),
                                           ("l16x16_b2_m-0p19", 4), ("l16x16_b2_m-0p19", 8)])
def test_sharded_recompute_cg_matches_reference(tmp_path, fixture, world):
    """The recompute-Ad CG (test option cg=5: 4-deep faces of d_{j-1}, d_{j-2}'s
    kept from the previous pass, 4-deep ghost links) on t-shards, including the
    interior/edge split of Wt = 512 / 240, the narrowest shard it takes (Wt = 4)
    and the fall-back to the stored-Ad pass below it (Wt = 2): the reference's
    iteration count and solution."""
    rep = run_world("gpu", fixture, world, tmp_path, timeout=140, extra_env=sm_opts(cg=5))
    assert rep["checks"]["ref_cgx"] <= 1e-12
    ref = rep["ref_cg_iters"]
    assert len(set(rep["cg_iters"])) == 1 and abs(rep["cg_iters"][0] - ref) <= max(1, ref // 100)
    assert all(rep["cg_converged"])


@pytest.mark.parametrize("fixture,world", [("md16x16_hot_m0", 2), ("md32x48_b3_m0p1", 4), ("md64x64_b2_m0", 2)])
def test_sharded_md_matches_reference(tmp_path, fixture, world):
    """MD layer on t-shards: bitwise plaquette / staples / gauge force, the
    CG-dependent MD force, leapfrog and Hamiltonians within the test_md_gpu
    tolerances, and an HMC trajectory equal to the one-shard trajectory."""
    rep = run_world("md", fixture, world, tmp_path, timeout=140)
    c = rep["checks"]
    for k in ("ref_plaq", "ref_staple", "ref_gforce"):
        assert c[k] is True, (k, c)
    for k in ("ref_mdforce", "ref_U1", "ref_P1"):
        assert c[k] <= 1e-8, (k, c)
    m = rep["meta"]
    assert len({tuple(s) for s in rep["sums"]}) == 1  # every shard has the global sums
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


@pytest.mark.parametrize("fixture,world,fused,folded,td", [
    ("gen:32x48:0.4242:0.0", 2, "1", "0", "1"),   # the one-pass eo CG (4-deep faces of d, Ad)
    ("gen:32x48:0.3:-0.1", 4, "1", "0", "1"),
    ("gen:32x48:0.3:-0.1", 6, "1", "0", "1"),     # Wt = 8: the narrowest shard it takes (faces = a whole neighbour)
    ("gen:32x48:0.3:-0.1", 8, "1", "0", "1"),     # Wt = 6 < 8: falls back to the six-launch iteration
    ("gen:32x48:0.3:-0.1", 4, "1", "0", "0"),     # the six-launch iteration
    ("gen:32x48:0.3:-0.1", 4, "0", "0", "0"),     # the two-launch Dhat (eo_hop with faces)
    ("gen:32x48:0.3:-0.1", 4, "1", "1", "0"),     # the folded eo CG (faces of d, r, Ad, W)
    # Wh = 128: three waves per strip, interior waves without halo lanes
    ("gen:24x512:0.3246:-0.05", 2, "1", "0", "1"), ("gen:24x512:0.3246:-0.05", 2, "1", "1", "0")])
def test_sharded_even_odd_matches_one_shard(tmp_path, fixture, world, fused, folded, td):
    """Even-odd layer on t-shards (checkerboard faces over the host transport)
    vs one shard: Dhat / Dhat^dag bitwise (same per-element arithmetic), the
    half-lattice CG to 1e-10 in the same iteration count (+-1 %), the MD force
    to 1e-10, and an HMC trajectory with the same accept decision."""
    rep = run_world("eo", fixture, world, tmp_path, timeout=140,
                    extra_env=sm_opts(eo_fused=fused, eo_cg_folded=folded, eo_cg_td=td))
    c = rep["checks"]
    assert c["dhat"] is True and c["dhatdag"] is True, c
    # the sharded dots sum per-shard partials: a different rounding order
    # than one shard, amplified by the condition number along the solve
    # (3e-12 measured at 32x48, m0 = -0.1); both solves reach |r| < 1e-10 |b|
    assert c["cgx"] <= 1e-10, c
    its = {it for conv, it in rep["cg"]}
    assert len(its) == 1 and all(conv for conv, it in rep["cg"])
    one = rep["cg_one"][1]
    assert abs(its.pop() - one) <= max(1, one // 100)
    assert c["force"] <= 1e-10, c
    assert len({tuple(t) for t in rep["traj"]}) == 1
    dH, acc, r = rep["traj"][0]
    assert abs(dH - rep["traj_one"][0]) <= 1e-6 * max(1.0, abs(rep["traj_one"][0]))
    assert acc == rep["traj_one"][1] and r == rep["traj_one"][2]
    assert c["traj_U"] <= 1e-8, c


@pytest.mark.parametrize("red", [1, 0], ids=["red", "nored"])
@pytest.mark.parametrize("max_iter", [10000, 16, 17], ids=["converge", "stop_even", "stop_odd"])
def test_sharded_even_odd_cg_schedules(tmp_path, red, max_iter):
    """The one-pass even-odd CG on 4 real t-shard processes (host transport),
    with the redundant scalars (every block of pass j+1 evaluates pass j's
    scalars from the all-reduced sums, test option red_shards=1) and with the
    scalar kernel after the all-reduce (red_shards=0), converged and cut off
    by max_iter after an even or an odd pass (the host keeps issuing passes
    past the stop, so the stopped state must survive the overshoot, ADVICE
    r02): every shard reports the one-shard iteration count and convergence
    flag, and x agrees with the one-shard solve to 1e-10 (the sharded
    reduction order)."""
    rep = run_world("eocg", "gen:32x48:0.3:-0.1", 4, tmp_path, timeout=140,
                    extra_env=dict(sm_opts(red_shards=red), SM_WORKER_EO_MAXIT=str(max_iter)))
    assert rep["Wt"] >= 8  # the one-pass kernel on t-shards, not the six-launch fall-back
    conv1, it1 = rep["cg_one"]
    for conv, it in rep["cg"]:
        assert conv == conv1, rep
        assert it == it1 if max_iter < 10000 else abs(it - it1) <= max(1, it1 // 100), rep
    if max_iter < 10000:
        assert conv1 == 0 and it1 == max_iter, rep
    assert rep["x_rel"] <= 1e-10, rep


@pytest.mark.parametrize("wish", ["11", "10", "01", "00"])
def test_link_angle_choice_is_per_shard(tmp_path, wish):
    """sm_cg_link_angles is per context, and on t-shards each shard decides
    for itself (its own links and the ghost links it receives): the codes
    rebuild every link bitwise, so shards that disagree still compute the
    same iterates through the same collectives. Two solves per rank (U
    re-uploaded in between, which re-opens the decision) and a third with the
    codes off everywhere: every shard uses the codes iff it asked, all solves
    converge in one count, and each shard's x is bitwise the codes-off x."""
    rep = run_world("angles", f"gen:64x512:0.3246:-0.05:{wish}", 2, tmp_path, timeout=120)
    for rank, solves in enumerate(rep["solves"]):
        assert all(conv == 1 for conv, it, used, h in solves), rep
        assert [used for conv, it, used, h in solves[:2]] == [int(wish[rank])] * 2, rep
        assert len({h for conv, it, used, h in solves}) == 1, rep  # bitwise one x
    assert len({it for r in rep["solves"] for conv, it, used, h in r}) == 1, rep


@pytest.mark.parametrize("wish,wish2", [("11", "01"), ("01", "11"), ("11", "10"), ("00", "10")])
def test_link_angle_toggle_on_one_rank(tmp_path, wish, wish2):
    """One rank changes its sm_cg_link_angles wish between two solves WITHOUT
    a new gauge upload, so only that rank rebuilds at the second solve. No
    collective depends on the choice, so nothing hangs or mixes sums: every
    solve converges in one iteration count on every rank, each solve uses the
    codes on exactly the ranks that asked, and x is bitwise the same
    throughout (the codes are exact)."""
    rep = run_world("angles", f"gen:64x512:0.3246:-0.05:{wish}:{wish2}", 2, tmp_path, timeout=120)
    for rank, solves in enumerate(rep["solves"]):
        assert all(conv == 1 for conv, it, used, h in solves), rep
        assert solves[0][2] == int(wish[rank]) and solves[1][2] == int(wish2[rank]), rep
        assert len({h for conv, it, used, h in solves}) == 1, rep
    assert len({it for r in rep["solves"] for conv, it, used, h in r}) == 1, rep
