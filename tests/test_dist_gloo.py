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


@pytest.mark.parametrize("fixture,world", [("l64x64_b2_m0", 2), ("l32x48_b3_m-0p10", 2),
                                           ("l32x48_hot_m0", 4), ("l16x16_b2_m-0p19", 8)])
def test_sharded_operator_matches_reference(tmp_path, fixture, world):
    rep = run_world("oracle", fixture, world, tmp_path)
    assert rep["world"] == world
    assert rep["checks"] == {"ref_Dpsi": True, "ref_Ddagchi": True}
