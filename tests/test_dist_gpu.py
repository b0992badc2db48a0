"""World-size > 1 on ONE GPU: the sharded HIP path through the host transport.

2-4 processes share cuda:0, each owning a t-shard (sm_create_hosted + gloo).
Same kernels, face packing, ghost links, antiperiodic-sign ownership and
scalar all-reduces as the RCCL path; only the wire differs. D, D^dag, D D^dag
and the force must equal the reference bitwise; CG must converge in the
reference's iteration count (+-1 %) to 1e-12 relative.
"""
import pytest

from distutil import run_world

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("fixture,world", [("l64x64_b2_m0", 2), ("l32x48_b3_m-0p10", 4),
                                           ("l64x64_b5_m-0p06", 4),
                                           # Wt = 512 / 240: the fused CG runs interior and edge
                                           # t-blocks as separate launches (halo overlap path);
                                           # reference = one shard on the same GPU
                                           ("gen:48x1024:0.3:-0.05", 2), ("gen:32x960:0.4242:0.0", 4)])
def test_sharded_gpu_path_matches_reference(tmp_path, fixture, world):
    # bt = 64 so the Dirac apply of the larger shards also splits into interior
    # and edge t-blocks (the overlapped halo path)
    env = {"SM_BT": "64"} if fixture.startswith("gen:") else None
    rep = run_world("gpu", fixture, world, tmp_path, timeout=600, extra_env=env)
    c = rep["checks"]
    for k in ("ref_Dpsi", "ref_Ddagchi", "ref_DDdagpsi", "ref_force"):
        assert c[k] is True, (k, c)
    assert c["ref_cgx"] <= 1e-12
    ref = rep["ref_cg_iters"]
    assert len(set(rep["cg_iters"])) == 1 and abs(rep["cg_iters"][0] - ref) <= max(1, ref // 100)
    assert all(rep["cg_converged"])
    assert len({tuple(d) for d in rep["dots"]}) == 1  # identical global dot on every shard
