"""The recompute-Ad CG's scheduling variants agree with each other.

Round 2 moved work out of separate kernels: the ticketed tail (the pass's last
block sums the partials and forms the scalars), the pipelined t-shard faces
(the edge launch packs d_j's faces and the exchange for the next pass follows
it) and the redundant t-shard scalars (every block evaluates the previous
pass's scalars from the all-reduced sums). Each one changes only where a sum
or a scalar step runs, or the order of a fixed-order sum, so a solve with it
and one with the older form (the environment switches read at context
creation, SM_TEST_OPTS) must reach the same iteration count and x to 1e-12 -- the
reduction-order band of every other CG parity test
(src/conjugate_gradient.cpp:28-66 is the recurrence all of them follow).
"""
import ctypes

import numpy as np
import pytest

from conftest import opts_env, ptr

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def sm():
    import schwingermodel_amd
    return schwingermodel_amd


def solve(sm, Nx, Nt, sigma, m0, opts, loopback=False, eo=False):
    S = Nx * Nt
    U, psi = np.empty(4 * S), np.empty(4 * S)
    sm.lib.sm_fill_gauge(4321, sigma, Nt, 0, Nx, 0, Nt, ptr(U[:2 * S]), ptr(U[2 * S:]))
    sm.lib.sm_fill_spinor(5678, Nt, 0, Nx, 0, Nt, ptr(psi[:2 * S]), ptr(psi[2 * S:]))
    with opts_env(**opts):
        L = sm.Lattice(Nx, Nt, loopback=loopback)  # the switches are read here
    try:
        sm.check(sm.lib.sm_upload_gauge(L.ctx, ptr(U[:2 * S]), ptr(U[2 * S:])))
        x = np.empty(4 * S)
        res = sm.CGResult()
        if eo:
            sm.check(sm.lib.sm_eo_cg(L.ctx, ptr(psi[:2 * S]), ptr(psi[2 * S:]), ptr(x[:2 * S]), ptr(x[2 * S:]),
                                     m0, 1e-10, 10000, ctypes.byref(res)))
        else:
            sm.check(sm.lib.sm_tune_cg(L.ctx, 5, 0))
            sm.check(sm.lib.sm_cg(L.ctx, ptr(psi[:2 * S]), ptr(psi[2 * S:]), ptr(x[:2 * S]), ptr(x[2 * S:]), m0,
                                  1e-10, 10000, ctypes.byref(res)))
    finally:
        L.close()
    assert res.converged == 1
    return res.iterations, x


def agree(a, b):
    (ia, xa), (ib, xb) = a, b
    assert abs(ia - ib) <= max(1, ia // 100), (ia, ib)
    rel = np.linalg.norm(xa - xb) / np.linalg.norm(xb)
    assert rel <= 1e-12, rel


# 1024^2 runs above the redundant-scalar threshold (the tail); 96 x 4096 has
# 74 wave columns, so the tail's groups of 64 tiles straddle block columns
@pytest.mark.parametrize("shape", [(1024, 1024), (96, 4096)], ids=["1024x1024", "96x4096"])
def test_ticketed_tail_matches_scalar_kernel(sm, shape):
    Nx, Nt = shape
    opts = {"ra_red_max_blocks": 0}
    agree(solve(sm, Nx, Nt, 0.3246, -0.10, opts), solve(sm, Nx, Nt, 0.3246, -0.10, dict(opts, tail=0)))


def test_even_odd_tail_matches_scalar_kernel(sm):
    agree(solve(sm, 256, 256, 0.3246, -0.05, {}, eo=True),
          solve(sm, 256, 256, 0.3246, -0.05, {"tail": 0}, eo=True))


# the t-shard path through the one-rank RCCL loopback: every variant against
# the older schedule (faces packed and sent at the start of each pass, the
# scalar kernel after the all-reduce, a separate local-sum kernel)
@pytest.mark.parametrize("opts", [
    {},
    {"red_shards": 0},
    {"face_pipe": 0},
    {"face_pipe": 1},
    {"face_pipe": 2},
    {"face_pipe": 1, "rccl_order": 0},
    {"edge_xchunk": 0},
    {"tail": 0},
], ids=["default", "no_red", "no_pipe", "pipe_behind_edge", "pipe_deferred", "pipe_unordered", "long_edge", "no_tail"])
def test_tshard_schedules_agree(sm, opts):
    old = {"face_pipe": 0, "red_shards": 0, "tail": 0}
    agree(solve(sm, 64, 4096, 0.2374, -0.06, opts, loopback=True),
          solve(sm, 64, 4096, 0.2374, -0.06, old, loopback=True))


@pytest.mark.parametrize("max_iter", [16, 17], ids=["stop_even", "stop_odd"])
def test_tshard_stop_at_max_iter_matches_one_shard(sm, max_iter):
    """A solve cut off by max_iter after an even or an odd pass: the t-shard
    path (redundant scalars flushed from the all-reduced sums, x rows still
    pending added by the finish kernel) returns the one-shard x and count."""
    Nx, Nt = 64, 4096
    S = Nx * Nt
    U, psi = np.empty(4 * S), np.empty(4 * S)
    sm.lib.sm_fill_gauge(4321, 0.2374, Nt, 0, Nx, 0, Nt, ptr(U[:2 * S]), ptr(U[2 * S:]))
    sm.lib.sm_fill_spinor(5678, Nt, 0, Nx, 0, Nt, ptr(psi[:2 * S]), ptr(psi[2 * S:]))
    out = {}
    for name, kw in (("one", {}), ("loop", {"loopback": True})):
        L = sm.Lattice(Nx, Nt, **kw)
        try:
            sm.check(sm.lib.sm_upload_gauge(L.ctx, ptr(U[:2 * S]), ptr(U[2 * S:])))
            sm.check(sm.lib.sm_tune_cg(L.ctx, 5, 0))
            x = np.empty(4 * S)
            res = sm.CGResult()
            sm.lib.sm_cg(L.ctx, ptr(psi[:2 * S]), ptr(psi[2 * S:]), ptr(x[:2 * S]), ptr(x[2 * S:]), -0.06, 1e-10,
                         max_iter, ctypes.byref(res))
            out[name] = (res.converged, res.iterations, res.residual, x)
        finally:
            L.close()
    (c1, i1, e1, x1), (c2, i2, e2, x2) = out["one"], out["loop"]
    assert c1 == c2 == 0 and i1 == i2 == max_iter, (c1, c2, i1, i2)
    assert abs(e1 - e2) <= 1e-12 * abs(e1), (e1, e2)
    assert np.linalg.norm(x2 - x1) / np.linalg.norm(x1) <= 1e-13


def test_even_odd_tshard_redundant_scalars_agree(sm):
    """The even-odd CG on t-shards (RCCL loopback) with the redundant scalars
    (every block evaluates the previous pass's scalars from the all-reduced
    sums) against the scalar kernel after the all-reduce."""
    agree(solve(sm, 64, 512, 0.3246, -0.05, {}, loopback=True, eo=True),
          solve(sm, 64, 512, 0.3246, -0.05, {"red_shards": 0}, loopback=True, eo=True))


def test_placement_modes_bitwise():
    """The placement rules of the streamed CG buffers (sm_ctx.h pad_alloc:
    own size, or >= 2 GiB each with the contiguous flag) change where the
    fields live, never the arithmetic: the same solve is bitwise identical
    under each, at a shape whose fields are 256 MiB (4096 x 2048, the smallest
    that takes the rule). DESIGN §2 gives why the default is what it is."""
    import schwingermodel_amd as sm
    ref = None
    for mode in (0, 5):
        it, x = solve(sm, 4096, 2048, 0.2374, 0.3, {"pad_alloc": mode})
        if ref is None:
            ref = (it, x)
        else:
            assert it == ref[0], (mode, it, ref[0])
            assert np.array_equal(x.view(np.uint64), ref[1].view(np.uint64)), mode


def test_placement_probe_report():
    """Context creation searches the placement of the CG pass's streamed
    buffers one buffer at a time (sm_capi.cpp placement_probe): at a shape
    that takes the rule (4096 x 2048, 256 MiB fields) the report gives the
    pass time of the initial placement and after each buffer's search, in
    sweeps of four (never slower than before it: a candidate is kept only if
    faster), and a solve on the probed placement equals the no-probe solve
    bitwise. Below the rule's size, or with the probe off through the public
    switch, nothing is probed."""
    import schwingermodel_amd as sm

    def report(L):
        us = (ctypes.c_double * 16)()
        n, k = ctypes.c_int(-1), ctypes.c_int(-2)
        sm.check(sm.lib.sm_placement_report(L.ctx, us, ctypes.byref(n), ctypes.byref(k)))
        return n.value, k.value, list(us)[:max(0, n.value)]

    L = sm.Lattice(4096, 2048)
    try:
        n, k, us = report(L)
    finally:
        L.close()
    assert n in (5, 9, 13) and 0 <= k < 16, (n, k)  # the initial set + 4 per sweep
    assert all(u > 0 for u in us) and all(b <= a for a, b in zip(us, us[1:])), us
    L = sm.Lattice(512, 512)
    try:
        assert report(L)[0] == 0
    finally:
        L.close()
    before = sm.lib.sm_get_placement_probe()
    sm.check(sm.lib.sm_set_placement_probe(0))
    try:
        L = sm.Lattice(4096, 2048)
        try:
            assert report(L)[0] == 0
        finally:
            L.close()
    finally:
        sm.check(sm.lib.sm_set_placement_probe(before))
    a = solve(sm, 4096, 2048, 0.2374, 0.3, {})
    b = solve(sm, 4096, 2048, 0.2374, 0.3, {"place_probe": 0})
    assert a[0] == b[0] and np.array_equal(a[1].view(np.uint64), b[1].view(np.uint64))
