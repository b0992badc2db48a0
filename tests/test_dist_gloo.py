"""World-size > 1 on CPU (gloo): the t-sharding scheme of the multi-GPU path.

Each rank owns t in [t0, t0+Wt) from sm_shard_plan (the product's host
geometry), exchanges its t-faces with schwingermodel_amd.dist.exchange_faces
(the transport the GPU's host-staged halo uses; the GPU ships spin-projected
faces over it, these full-spinor faces feed the oracle) and applies the oracle's local
operator; the gathered result must equal the reference's single-domain golden
vectors BIT FOR BIT (the reference itself is bitwise decomposition-invariant,
tests/golden/manifest.json "decomposition_2x2").
"""
import pytest

from distutil import run_world


@pytest.mark.parametrize("name,world,expect", [
    ("rccl:2,2", 2, [2, 2]),            # every communicator holds the job's ranks
    ("rccl:2,1", 2, None),              # one rank's communicator is alone: refused
    ("rccl:4,4,4,4", 4, [4, 4]),
    ("hosted:1,1", 2, [1, 1]),          # host-staged shards: no RCCL world, not refused
    ("peer:2,2", 2, [2, 2]),            # the peer transport's connected view holds the job's ranks
    ("peer:2,1", 2, None),              # one rank's view is alone: refused
])
def test_bench_rccl_world_check(tmp_path, name, world, expect):
    """bench.py reports the world the transport itself holds (sm_comm_info ->
    ncclCommCount, or the peer transport's connected shards), min and max over
    the ranks, and refuses to report an RCCL or peer run whose worlds disagree
    with WORLD_SIZE."""
    rep = run_world("commworld", name, world, tmp_path, timeout=120)
    for r in rep["ranks"]:
        if expect is None:
            assert "refused" in r and "WORLD_SIZE is 2" in r["refused"], r
        else:
            key = "peer_ranks" if name.startswith("peer") else "rccl_ranks"
            assert r["ok"][key] == expect and r["ok"]["transport"] == name.split(":")[0], r


@pytest.mark.parametrize("case,world", [("ok", 2), ("setup:1", 2), ("setup:0", 3), ("check", 2)])
def test_bench_peer_fallback_agreement(tmp_path, case, world):
    """bench.py's N > 1 default: the peer transport after its check against the
    host-staged one, RCCL on EVERY rank if the setup failed on any rank or the
    check failed (a mixed world would deadlock its first collective)."""
    rep = run_world("fallback", case, world, tmp_path, timeout=120)
    kinds = {r["kind"] for r in rep["ranks"]}
    if case == "ok":
        assert kinds == {"peer"} and all(r["check"]["ok"] for r in rep["ranks"]), rep
    else:
        assert kinds == {"rccl"}, rep
        for r in rep["ranks"]:
            assert r["check"]["fallback"] == "rccl" and r["check"]["reason"], r


@pytest.mark.parametrize("fixture,world", [("l64x64_b2_m0", 2), ("l32x48_b3_m-0p10", 2),
                                           ("l32x48_hot_m0", 4), ("l16x16_b2_m-0p19", 8)])
def test_sharded_operator_matches_reference(tmp_path, fixture, world):
    rep = run_world("oracle", fixture, world, tmp_path)
    assert rep["world"] == world
    assert rep["checks"] == {"ref_Dpsi": True, "ref_Ddagchi": True}
