#!/usr/bin/env python3
"""One rank of a t-sharded multi-process check (launched by tests/test_dist_*.py).

    RANK=r WORLD_SIZE=P MASTER_ADDR=127.0.0.1 MASTER_PORT=... \
        python tests/dist_worker.py <mode> <fixture> <result.json>

mode "oracle" (CPU, gloo): every rank applies the ORACLE's local operator to its
    t-shard with faces exchanged by schwingermodel_amd.dist.exchange_faces (the
    protocol of the GPU path) and the geometry of sm_shard_plan; rank 0 checks
    the gathered result bit-for-bit against the reference's golden vectors.
mode "md" (one GPU, gloo host transport): the molecular-dynamics layer
    (plaquette, staples, gauge force, MD force, Hamiltonian, leapfrog, one HMC
    trajectory) on t-shards vs the reference's MD fixture / one shard.
mode "eo" (one GPU, gloo host transport): the even-odd preconditioned layer
    (Dhat, Dhat^dag, half-lattice CG, MD force, one HMC trajectory) on
    t-shards with checkerboard faces vs one shard.
mode "gpu" (one GPU shared by all ranks, gloo host transport): every rank runs
    the HIP kernels on its shard through sm_create_hosted (same kernels, face
    packing, ghost links, sign ownership and scalar reductions as the RCCL
    path); rank 0 checks D / D^dag / D D^dag / force bitwise and CG to 1e-12.
"""
import ctypes
import json
import math
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)


# the shard transport of the one-GPU worlds: "hosted" (sm_create_hosted + gloo) or "peer"
# (sm_create_peer: device-initiated stores between the processes' regions)
TRANSPORT = os.environ.get("SM_WORKER_TRANSPORT", "hosted")

def shard_field(flat, Nx, Nt, t0, Wt):
    """Global two-plane interleaved field -> this shard's block (same layout)."""
    S = Nx * Nt
    out = []
    for p in range(2):
        plane = flat[2 * S * p: 2 * S * (p + 1)].view(np.complex128).reshape(Nx, Nt)
        out.append(np.ascontiguousarray(plane[:, t0:t0 + Wt]).reshape(-1))
    return out  # [mu0, mu1] complex arrays of Nx*Wt


def unshard(blocks, Nx, Nt, Wt, dtype):
    planes = []
    for p in range(2):
        g = np.concatenate([b[p].reshape(Nx, Wt) for b in blocks], axis=1)
        planes.append(g.reshape(-1).view(np.float64) if dtype == complex else g.reshape(-1))
    return np.concatenate(planes)


def faces(mu0, mu1, Nx, Wt):
    """[plane][x] faces of columns t = 0 (lo) and t = Wt-1 (hi), 4*Nx doubles each."""
    a0, a1 = mu0.reshape(Nx, Wt), mu1.reshape(Nx, Wt)
    lo = np.concatenate([a0[:, 0], a1[:, 0]]).view(np.float64).copy()
    hi = np.concatenate([a0[:, Wt - 1], a1[:, Wt - 1]]).view(np.float64).copy()
    return lo, hi


def single_reference(sm, a, meta):
    """One shard (nshard = 1) on this GPU: the reference for a sharded run."""
    Nx, Nt, m0 = meta["Nx"], meta["Nt"], meta["m0"]
    S = Nx * Nt
    P = lambda x: ctypes.c_void_p(x.ctypes.data)  # noqa: E731
    L = sm.Lattice(Nx, Nt, device=int(os.environ.get("SM_DEVICE", "0")))
    sm.check(sm.lib.sm_upload_gauge(L.ctx, P(a["U"]), P(a["U"][2 * S:])))
    for key, src, fn in (("ref_Dpsi", "psi", 0), ("ref_Ddagchi", "chi", 1), ("ref_DDdagpsi", "psi", 2)):
        out = np.empty(4 * S)
        i0, i1 = a[src][:2 * S], a[src][2 * S:]
        if fn < 2:
            sm.check(sm.lib.sm_dirac(L.ctx, P(i0), P(i1), P(out), P(out[2 * S:]), m0, fn))
        else:
            sm.check(sm.lib.sm_ddag(L.ctx, P(i0), P(i1), P(out), P(out[2 * S:]), m0))
        a[key] = out
    F = np.empty(2 * S)
    sm.check(sm.lib.sm_force(L.ctx, P(a["psi"]), P(a["psi"][2 * S:]), P(a["chi"]), P(a["chi"][2 * S:]),
                             P(F), P(F[S:])))
    a["ref_force"] = F
    x = np.empty(4 * S)
    res = sm.CGResult()
    sm.check(sm.lib.sm_cg(L.ctx, P(a["psi"]), P(a["psi"][2 * S:]), P(x), P(x[2 * S:]), m0, 1e-10, 10000,
                          ctypes.byref(res)))
    a["ref_cgx"] = x
    meta["cg_iters"] = res.iterations
    L.close()


def shard_real(flat, Nx, Nt, t0, Wt):
    """Global two-plane real field (re_field) -> this shard's two planes."""
    S = Nx * Nt
    return [np.ascontiguousarray(flat[S * p: S * (p + 1)].reshape(Nx, Nt)[:, t0:t0 + Wt]).reshape(-1)
            for p in range(2)]


def run_md(name, result_path, dist, rank, world):
    """mode "md": the MD layer on t-shards (hosted transport) vs the reference's
    MD fixture, plus one HMC trajectory vs the same trajectory on one shard."""
    from conftest import bits_equal, load_md_fixture
    import schwingermodel_amd as sm
    from schwingermodel_amd import dist as smd
    meta, a = load_md_fixture(name)
    Nx, Nt = meta["Nx"], meta["Nt"]
    S = Nx * Nt
    t0, Wt = ctypes.c_int(), ctypes.c_int()
    sm.check(sm.lib.sm_shard_plan(Nt, world, rank, ctypes.byref(t0), ctypes.byref(Wt)))
    t0, Wt = t0.value, Wt.value
    V = Nx * Wt
    P_ = lambda x: ctypes.c_void_p(x.ctypes.data)  # noqa: E731
    U = shard_field(a["U"], Nx, Nt, t0, Wt)
    phi = shard_field(a["ref_phi"], Nx, Nt, t0, Wt)
    Pm = shard_real(a["P"], Nx, Nt, t0, Wt)
    prm = sm.HMCParams(meta["m0"], meta["beta"], meta["tau"], meta["md_steps"], 1e-10, 10000, 99)
    dev = int(os.environ.get("SM_DEVICE", "0"))
    ctx, tr = smd.create_shard_context(Nx, Nt, transport=TRANSPORT, device=dev)
    sm.check(sm.lib.sm_upload_gauge(ctx, P_(U[0]), P_(U[1])))
    local = {}
    sp, act = ctypes.c_double(), ctypes.c_double()
    plaq = np.empty(V, complex)
    sm.check(sm.lib.sm_plaquette(ctx, meta["beta"], ctypes.byref(sp), ctypes.byref(act), P_(plaq)))
    local["sums"] = (sp.value, act.value)
    local["ref_plaq"] = (plaq, plaq)
    S0, S1 = np.empty(V, complex), np.empty(V, complex)
    sm.check(sm.lib.sm_staples(ctx, P_(S0), P_(S1)))
    local["ref_staple"] = (S0, S1)
    F0, F1 = np.zeros(V), np.zeros(V)
    sm.check(sm.lib.sm_gauge_force(ctx, meta["beta"], P_(F0), P_(F1)))
    local["ref_gforce"] = (F0, F1)
    G0, G1 = np.empty(V), np.empty(V)
    res = sm.CGResult()
    sm.check(sm.lib.sm_md_force(ctx, ctypes.byref(prm), P_(phi[0]), P_(phi[1]), P_(G0), P_(G1), ctypes.byref(res)))
    local["ref_mdforce"] = (G0, G1)
    h = sm.HamiltonianTerms()
    sm.check(sm.lib.sm_hamiltonian(ctx, ctypes.byref(prm), P_(phi[0]), P_(phi[1]), P_(Pm[0]), P_(Pm[1]),
                                   ctypes.byref(h)))
    local["H0"] = h.H
    it, fails = ctypes.c_long(), ctypes.c_int()
    sm.check(sm.lib.sm_leapfrog(ctx, ctypes.byref(prm), P_(phi[0]), P_(phi[1]), P_(Pm[0]), P_(Pm[1]),
                                ctypes.byref(it), ctypes.byref(fails)))
    U1a, U1b = np.empty(V, complex), np.empty(V, complex)
    sm.check(sm.lib.sm_download_gauge(ctx, P_(U1a), P_(U1b)))
    local["ref_U1"] = (U1a, U1b)
    local["ref_P1"] = (Pm[0].copy(), Pm[1].copy())
    sm.check(sm.lib.sm_hamiltonian(ctx, ctypes.byref(prm), P_(phi[0]), P_(phi[1]), P_(Pm[0]), P_(Pm[1]),
                                   ctypes.byref(h)))
    local["H1"] = h.H
    # one full HMC trajectory from the fixture's U (device draws keyed on the
    # global site: every sharding draws the same momenta and sources)
    sm.check(sm.lib.sm_upload_gauge(ctx, P_(U[0]), P_(U[1])))
    r = sm.HMCResult()
    sm.check(sm.lib.sm_hmc_trajectory(ctx, ctypes.byref(prm), 3, ctypes.byref(r)))
    Ua, Ub = np.empty(V, complex), np.empty(V, complex)
    sm.check(sm.lib.sm_download_gauge(ctx, P_(Ua), P_(Ub)))
    local["traj"] = (r.dH, r.accepted, r.r)
    local["traj_U"] = (Ua, Ub)
    sm.lib.sm_destroy(ctx)
    gathered = [None] * world
    dist.all_gather_object(gathered, local)
    if rank == 0:
        rep = {"world": world, "fixture": name, "checks": {}}
        for key in ("ref_plaq", "ref_staple", "ref_gforce"):
            dtype = float if key == "ref_gforce" else complex
            g = unshard([d[key] for d in gathered], Nx, Nt, Wt, dtype)
            if key == "ref_plaq":
                g = g[:2 * S]
            rep["checks"][key] = bool(bits_equal(g, a[key]))
        for key in ("ref_mdforce", "ref_P1"):
            g = unshard([d[key] for d in gathered], Nx, Nt, Wt, float)
            rep["checks"][key] = float(np.linalg.norm(g - a[key]) / np.linalg.norm(a[key]))
        g = unshard([d["ref_U1"] for d in gathered], Nx, Nt, Wt, complex)
        rep["checks"]["ref_U1"] = float(np.linalg.norm(g - a["ref_U1"]) / np.linalg.norm(a["ref_U1"]))
        rep["sums"] = [d["sums"] for d in gathered]
        rep["H0"] = [d["H0"] for d in gathered]
        rep["H1"] = [d["H1"] for d in gathered]
        rep["meta"] = {k: meta[k] for k in ("sp", "gauge_action", "H0", "H1")}
        # the same trajectory on one shard of the same GPU
        L = sm.Lattice(Nx, Nt, device=dev)
        sm.check(sm.lib.sm_upload_gauge(L.ctx, P_(a["U"]), P_(a["U"][2 * S:])))
        r1 = sm.HMCResult()
        sm.check(sm.lib.sm_hmc_trajectory(L.ctx, ctypes.byref(prm), 3, ctypes.byref(r1)))
        U1 = np.empty(4 * S)
        sm.check(sm.lib.sm_download_gauge(L.ctx, P_(U1), P_(U1[2 * S:])))
        L.close()
        g = unshard([d["traj_U"] for d in gathered], Nx, Nt, Wt, complex)
        rep["traj"] = {"sharded": [d["traj"] for d in gathered], "single": (r1.dH, r1.accepted, r1.r),
                       "U_rel": float(np.linalg.norm(g - U1) / np.linalg.norm(U1))}
        with open(result_path, "w") as f:
            json.dump(rep, f)
    dist.barrier()
    dist.destroy_process_group()


def eo_ops(sm, ctx, V, fields, m0, prm):
    """The even-odd layer on one context (one shard or a t-shard): Dhat and
    Dhat^dag of psi, the half-lattice CG, the even-odd MD force and one
    even-odd HMC trajectory (which leaves U changed). `fields` = (U, psi, phi)
    as plane pairs of this context's block."""
    P_ = lambda x: ctypes.c_void_p(x.ctypes.data)  # noqa: E731
    (U0, U1), (p0, p1), (f0, f1) = fields
    out = {}
    step = lambda m: print(f"[eo_ops V={V}] {m}", file=sys.stderr, flush=True)  # noqa: E731
    step("dhat")
    for key, dag in (("dhat", 0), ("dhatdag", 1)):
        o0, o1 = np.empty(V, complex), np.empty(V, complex)
        sm.check(sm.lib.sm_eo_dhat(ctx, dag, P_(p0), P_(p1), P_(o0), P_(o1), m0))
        out[key] = (o0, o1)
    x0, x1 = np.empty(V, complex), np.empty(V, complex)
    res = sm.CGResult()
    step("eo_cg")
    sm.check(sm.lib.sm_eo_cg(ctx, P_(p0), P_(p1), P_(x0), P_(x1), m0, 1e-10, 10000, ctypes.byref(res)))
    step(f"eo_cg done {res.converged} {res.iterations}")
    out["cgx"] = (x0, x1)
    out["cg"] = (res.converged, res.iterations)
    G0, G1 = np.empty(V), np.empty(V)
    sm.check(sm.lib.sm_md_force(ctx, ctypes.byref(prm), P_(f0), P_(f1), P_(G0), P_(G1), ctypes.byref(res)))
    out["force"] = (G0, G1)
    step("trajectory")
    r = sm.HMCResult()
    sm.check(sm.lib.sm_hmc_trajectory(ctx, ctypes.byref(prm), 5, ctypes.byref(r)))
    Ua, Ub = np.empty(V, complex), np.empty(V, complex)
    sm.check(sm.lib.sm_download_gauge(ctx, P_(Ua), P_(Ub)))
    out["traj"] = (r.dH, r.accepted, r.r)
    out["traj_U"] = (Ua, Ub)
    return out


def run_eo(name, result_path, dist, rank, world):
    """mode "eo": the even-odd preconditioned layer on t-shards (hosted
    transport, checkerboard faces) vs the same calls on one shard.
    name = gen:<Nx>x<Nt>:<sigma>:<m0> (synthetic fields)."""
    import schwingermodel_amd as sm
    from schwingermodel_amd import dist as smd
    _, dims, sigma, m0s = name.split(":")
    Nx, Nt = (int(v) for v in dims.split("x"))
    sigma, m0 = float(sigma), float(m0s)
    S = Nx * Nt
    g = {k: np.empty(4 * S) for k in ("U", "psi", "phi")}
    sm.lib.sm_fill_gauge(4321, sigma, Nt, 0, Nx, 0, Nt, g["U"].ctypes.data, g["U"][2 * S:].ctypes.data)
    sm.lib.sm_fill_spinor(5678, Nt, 0, Nx, 0, Nt, g["psi"].ctypes.data, g["psi"][2 * S:].ctypes.data)
    sm.lib.sm_fill_spinor(1357, Nt, 0, Nx, 0, Nt, g["phi"].ctypes.data, g["phi"][2 * S:].ctypes.data)
    prm = sm.HMCParams(m0, 2.0, 0.5, 6, 1e-10, 10000, 77, 1)
    t0, Wt = ctypes.c_int(), ctypes.c_int()
    sm.check(sm.lib.sm_shard_plan(Nt, world, rank, ctypes.byref(t0), ctypes.byref(Wt)))
    t0, Wt = t0.value, Wt.value
    V = Nx * Wt
    mine = [shard_field(g[k], Nx, Nt, t0, Wt) for k in ("U", "psi", "phi")]
    dev = int(os.environ.get("SM_DEVICE", "0"))
    ctx, tr = smd.create_shard_context(Nx, Nt, transport=TRANSPORT, device=dev)
    sm.check(sm.lib.sm_upload_gauge(ctx, ctypes.c_void_p(mine[0][0].ctypes.data),
                                    ctypes.c_void_p(mine[0][1].ctypes.data)))
    local = eo_ops(sm, ctx, V, mine, m0, prm)
    sm.lib.sm_destroy(ctx)
    gathered = [None] * world
    dist.all_gather_object(gathered, local)
    if rank == 0:
        L = sm.Lattice(Nx, Nt, device=dev)
        full = [shard_field(g[k], Nx, Nt, 0, Nt) for k in ("U", "psi", "phi")]
        sm.check(sm.lib.sm_upload_gauge(L.ctx, ctypes.c_void_p(full[0][0].ctypes.data),
                                        ctypes.c_void_p(full[0][1].ctypes.data)))
        one = eo_ops(sm, L.ctx, S, full, m0, prm)
        L.close()
        from conftest import bits_equal
        rep = {"world": world, "Wt": Wt, "checks": {}}
        for key in ("dhat", "dhatdag", "cgx", "force", "traj_U"):
            dtype = float if key == "force" else complex
            gsh = unshard([d[key] for d in gathered], Nx, Nt, Wt, dtype)
            ref = unshard([one[key]], Nx, Nt, Nt, dtype)
            rep["checks"][key] = (bool(bits_equal(gsh, ref)) if key.startswith("dhat")
                                  else float(np.linalg.norm(gsh - ref) / np.linalg.norm(ref)))
        rep["cg"] = [list(d["cg"]) for d in gathered]
        rep["cg_one"] = list(one["cg"])
        rep["traj"] = [list(d["traj"]) for d in gathered]
        rep["traj_one"] = list(one["traj"])
        with open(result_path, "w") as f:
            json.dump(rep, f)
    dist.barrier()
    dist.destroy_process_group()


def run_eocg(name, result_path, dist, rank, world):
    """mode "eocg": only the even-odd half-lattice CG on t-shards (hosted
    transport) vs one shard, with max_iter from SM_WORKER_EO_MAXIT (a cut-off
    solve stops mid-chunk and further passes are issued past the stop: the
    redundant t-shard scalars must keep the stopped state). Reports each
    shard's (converged, iterations) and the relative difference of x."""
    import schwingermodel_amd as sm
    from schwingermodel_amd import dist as smd
    _, dims, sigma, m0s = name.split(":")
    Nx, Nt = (int(v) for v in dims.split("x"))
    sigma, m0 = float(sigma), float(m0s)
    maxit = int(os.environ.get("SM_WORKER_EO_MAXIT", "10000"))
    S = Nx * Nt
    g = {k: np.empty(4 * S) for k in ("U", "psi")}
    sm.lib.sm_fill_gauge(4321, sigma, Nt, 0, Nx, 0, Nt, g["U"].ctypes.data, g["U"][2 * S:].ctypes.data)
    sm.lib.sm_fill_spinor(5678, Nt, 0, Nx, 0, Nt, g["psi"].ctypes.data, g["psi"][2 * S:].ctypes.data)
    t0, Wt = ctypes.c_int(), ctypes.c_int()
    sm.check(sm.lib.sm_shard_plan(Nt, world, rank, ctypes.byref(t0), ctypes.byref(Wt)))
    t0, Wt = t0.value, Wt.value
    P_ = lambda x: ctypes.c_void_p(x.ctypes.data)  # noqa: E731

    def solve(ctx, V, U, p):
        sm.check(sm.lib.sm_upload_gauge(ctx, P_(U[0]), P_(U[1])))
        x0, x1 = np.empty(V, complex), np.empty(V, complex)
        res = sm.CGResult()
        sm.check(sm.lib.sm_eo_cg(ctx, P_(p[0]), P_(p[1]), P_(x0), P_(x1), m0, 1e-10, maxit, ctypes.byref(res)))
        return (x0, x1), (int(res.converged), int(res.iterations))

    mine = [shard_field(g[k], Nx, Nt, t0, Wt) for k in ("U", "psi")]
    dev = int(os.environ.get("SM_DEVICE", "0"))
    ctx, tr = smd.create_shard_context(Nx, Nt, transport=TRANSPORT, device=dev)
    x, cg = solve(ctx, Nx * Wt, mine[0], mine[1])
    sm.lib.sm_destroy(ctx)
    gathered = [None] * world
    dist.all_gather_object(gathered, (x, cg))
    if rank == 0:
        L = sm.Lattice(Nx, Nt, device=dev)
        full = [shard_field(g[k], Nx, Nt, 0, Nt) for k in ("U", "psi")]
        x1, cg1 = solve(L.ctx, S, full[0], full[1])
        L.close()
        gsh = unshard([d[0] for d in gathered], Nx, Nt, Wt, complex)
        ref = unshard([x1], Nx, Nt, Nt, complex)
        rep = {"world": world, "Wt": Wt, "max_iter": maxit, "cg": [list(d[1]) for d in gathered],
               "cg_one": list(cg1), "x_rel": float(np.linalg.norm(gsh - ref) / np.linalg.norm(ref))}
        with open(result_path, "w") as f:
            json.dump(rep, f)
    dist.barrier()
    dist.destroy_process_group()


def bits_sha(*arrays):
    import hashlib
    h = hashlib.sha256()
    for a in arrays:
        h.update(np.ascontiguousarray(a).view(np.uint8))
    return h.hexdigest()


def run_angles(name, result_path, dist, rank, world):
    """mode "angles": each shard's own link-code choice in the recompute-Ad
    CG. name = gen:<Nx>x<Nt>:<sigma>:<m0>:<wish> where wish is one 0/1 digit
    per rank for sm_cg_link_angles. Each rank solves twice (the second solve
    re-decides after U is re-uploaded), then once more with the codes off, and
    reports (converged, iterations, in_use, SHA-256 of x) per solve; nothing
    may hang. With a sixth field (gen:...:<wish>:<wish2>) the ranks set wish2
    between the solves and do NOT re-upload U, so only the ranks whose wish
    changed rebuild at the second solve."""
    import schwingermodel_amd as sm
    from schwingermodel_amd import dist as smd
    parts = name.split(":")
    _, dims, sigma, m0s, wish = parts[:5]
    wish2 = parts[5] if len(parts) > 5 else None
    Nx, Nt = (int(v) for v in dims.split("x"))
    sigma, m0 = float(sigma), float(m0s)
    S = Nx * Nt
    g = {k: np.empty(4 * S) for k in ("U", "psi")}
    sm.lib.sm_fill_gauge(4321, sigma, Nt, 0, Nx, 0, Nt, g["U"].ctypes.data, g["U"][2 * S:].ctypes.data)
    sm.lib.sm_fill_spinor(5678, Nt, 0, Nx, 0, Nt, g["psi"].ctypes.data, g["psi"][2 * S:].ctypes.data)
    t0, Wt = ctypes.c_int(), ctypes.c_int()
    sm.check(sm.lib.sm_shard_plan(Nt, world, rank, ctypes.byref(t0), ctypes.byref(Wt)))
    U, p = (shard_field(g[k], Nx, Nt, t0.value, Wt.value) for k in ("U", "psi"))
    P_ = lambda x: ctypes.c_void_p(x.ctypes.data)  # noqa: E731
    ctx, tr = smd.create_shard_context(Nx, Nt, transport=TRANSPORT, device=int(os.environ.get("SM_DEVICE", "0")))
    sm.check(sm.lib.sm_tune_cg(ctx, 5, 0))
    sm.check(sm.lib.sm_cg_link_angles(ctx, int(wish[rank]), None))
    out = []
    for k in range(2):
        if k == 0 or wish2 is None:
            sm.check(sm.lib.sm_upload_gauge(ctx, P_(U[0]), P_(U[1])))
        else:
            sm.check(sm.lib.sm_cg_link_angles(ctx, int(wish2[rank]), None))
        x0, x1 = np.empty(Nx * Wt.value, complex), np.empty(Nx * Wt.value, complex)
        res = sm.CGResult()
        sm.check(sm.lib.sm_cg(ctx, P_(p[0]), P_(p[1]), P_(x0), P_(x1), m0, 1e-10, 10000, ctypes.byref(res)))
        used = ctypes.c_int(-1)
        sm.check(sm.lib.sm_cg_link_angles(ctx, -1, ctypes.byref(used)))
        out.append([int(res.converged), int(res.iterations), int(used.value), bits_sha(x0, x1)])
    # the same solve with every shard on the complex links: the reference
    # point of the bitwise comparison (the codes are exact)
    sm.check(sm.lib.sm_cg_link_angles(ctx, 0, None))
    x0, x1 = np.empty(Nx * Wt.value, complex), np.empty(Nx * Wt.value, complex)
    res = sm.CGResult()
    sm.check(sm.lib.sm_cg(ctx, P_(p[0]), P_(p[1]), P_(x0), P_(x1), m0, 1e-10, 10000, ctypes.byref(res)))
    out.append([int(res.converged), int(res.iterations), 0, bits_sha(x0, x1)])
    sm.lib.sm_destroy(ctx)
    gathered = [None] * world
    dist.all_gather_object(gathered, out)
    if rank == 0:
        with open(result_path, "w") as f:
            json.dump({"world": world, "solves": gathered}, f)
    dist.barrier()
    dist.destroy_process_group()


def fill_block(sm, Nx, Nt, t0, Wt, sigma, seeds=(4321, 5678, 91011), nthreads=8):
    """U, psi, chi of the t-block [t0, t0+Wt) of the global synthetic fields
    (counter-based, row-separable: row blocks are filled in threads)."""
    from concurrent.futures import ThreadPoolExecutor
    V = Nx * Wt
    f = {k: np.empty(4 * V) for k in ("U", "psi", "chi")}
    rows = max(1, -(-Nx // nthreads))

    def job(x0):
        nx = min(rows, Nx - x0)
        o = 2 * x0 * Wt
        sm.lib.sm_fill_gauge(seeds[0], sigma, Nt, x0, nx, t0, Wt, f["U"][o:].ctypes.data, f["U"][2 * V + o:].ctypes.data)
        for k, s in (("psi", seeds[1]), ("chi", seeds[2])):
            sm.lib.sm_fill_spinor(s, Nt, x0, nx, t0, Wt, f[k][o:].ctypes.data, f[k][2 * V + o:].ctypes.data)
    with ThreadPoolExecutor(nthreads) as ex:
        list(ex.map(job, range(0, Nx, rows)))
    return f


def big_ops(sm, ctx, V, f, m0, ops):
    """The operators on one context (host pointers, reference layout): D psi,
    D^dag chi, force(psi, chi) (ops 'full'), the CG solve of D D^dag x = psi and
    its true residual terms |psi - D D^dag x|^2, |psi|^2 (local sums)."""
    P = lambda x: ctypes.c_void_p(x.ctypes.data)  # noqa: E731
    out = {}
    if ops == "full":
        for key, src, dag in (("Dpsi", "psi", 0), ("Ddagchi", "chi", 1)):
            o = np.empty(4 * V)
            sm.check(sm.lib.sm_dirac(ctx, P(f[src]), P(f[src][2 * V:]), P(o), P(o[2 * V:]), m0, dag))
            out[key] = o
        F = np.empty(2 * V)
        sm.check(sm.lib.sm_force(ctx, P(f["psi"]), P(f["psi"][2 * V:]), P(f["chi"]), P(f["chi"][2 * V:]),
                                 P(F), P(F[V:])))
        out["force"] = F
    x = np.empty(4 * V)
    res = sm.CGResult()
    sm.check(sm.lib.sm_cg(ctx, P(f["psi"]), P(f["psi"][2 * V:]), P(x), P(x[2 * V:]), m0, 1e-10, 20000,
                          ctypes.byref(res)))
    out["x"] = x
    out["cg"] = (int(res.converged), int(res.iterations))
    Ax = np.empty(4 * V)
    sm.check(sm.lib.sm_ddag(ctx, P(x), P(x[2 * V:]), P(Ax), P(Ax[2 * V:]), m0))
    r = f["psi"] - Ax
    out["res_sq"] = (float(r @ r), float(f["psi"] @ f["psi"]))
    return out


def block_of(a, Nx, Nt, t0, Wt, planes_complex=True):
    """Columns [t0, t0+Wt) of a global two-plane field (complex planes of Nx*Nt,
    or real planes for the force), as this shard's flat layout."""
    S = Nx * Nt
    if planes_complex:
        return np.concatenate([np.ascontiguousarray(a[2 * S * p:2 * S * (p + 1)].view(np.complex128)
                                                    .reshape(Nx, Nt)[:, t0:t0 + Wt]).reshape(-1).view(np.float64)
                               for p in range(2)])
    return np.concatenate([np.ascontiguousarray(a[S * p:S * (p + 1)].reshape(Nx, Nt)[:, t0:t0 + Wt]).reshape(-1)
                           for p in range(2)])


def large_fixture(Nx, Nt, sigma, m0):
    """The reference's full-size summary fixture for these inputs (manifest
    'large', tests/golden/make_golden.py --large), or None: (meta, arrays)."""
    with open(os.path.join(REPO, "tests", "golden", "manifest.json")) as fh:
        large = json.load(fh).get("large", {})
    for meta in large.values():
        if (meta["Nx"], meta["Nt"]) == (Nx, Nt) and abs(meta["sigma"] - sigma) < 1e-12 and abs(meta["m0"] - m0) < 1e-12:
            with np.load(os.path.join(REPO, "tests", "golden", meta["file"]), allow_pickle=False) as z:
                return meta, {k: z[k].copy() for k in z.files}
    return None


def run_big(name, result_path, dist, rank, world):
    """mode "big": BASELINE configs at their real shard shapes on ONE GPU.
    name = big:<Nx>x<Nt>:<sigma>:<m0>:<ops>, ops 'full' (D, D^dag, force, CG)
    or 'cg'. Rank 0 first runs the one-shard reference on the GPU and stores
    its outputs as .npy next to the result file; then every rank runs its
    t-shard (hosted transport) and compares its own block: D / D^dag / force
    bitwise, CG iterations, |x - x_one| and the true residual summed over ranks.
    No rank ever holds the whole sharded result."""
    import time
    import schwingermodel_amd as sm
    from schwingermodel_amd import dist as smd
    import torch
    _, dims, sigma, m0s, ops = name.split(":")
    Nx, Nt = (int(v) for v in dims.split("x"))
    sigma, m0 = float(sigma), float(m0s)
    S = Nx * Nt
    d = os.path.dirname(result_path)
    dev = int(os.environ.get("SM_DEVICE", "0"))
    if rank == 0:
        t = time.time()
        g = fill_block(sm, Nx, Nt, 0, Nt, sigma)
        L = sm.Lattice(Nx, Nt, device=dev)
        sm.check(sm.lib.sm_upload_gauge(L.ctx, ctypes.c_void_p(g["U"].ctypes.data),
                                        ctypes.c_void_p(g["U"][2 * S:].ctypes.data)))
        one = big_ops(sm, L.ctx, S, g, m0, ops)
        L.close()
        del g
        for k in ("Dpsi", "Ddagchi", "force", "x"):
            if k in one:
                np.save(os.path.join(d, f"one_{k}.npy"), one.pop(k))
        with open(os.path.join(d, "one.json"), "w") as fh:
            json.dump({"cg": one["cg"], "res_sq": one["res_sq"], "seconds": time.time() - t}, fh)
        del one
    dist.barrier()
    t0, Wt = ctypes.c_int(), ctypes.c_int()
    sm.check(sm.lib.sm_shard_plan(Nt, world, rank, ctypes.byref(t0), ctypes.byref(Wt)))
    t0, Wt = t0.value, Wt.value
    V = Nx * Wt
    f = fill_block(sm, Nx, Nt, t0, Wt, sigma, nthreads=2)
    ctx, tr = smd.create_shard_context(Nx, Nt, transport=TRANSPORT, device=dev)
    sm.check(sm.lib.sm_upload_gauge(ctx, ctypes.c_void_p(f["U"].ctypes.data),
                                    ctypes.c_void_p(f["U"][2 * V:].ctypes.data)))
    ts = time.time()
    mine = big_ops(sm, ctx, V, f, m0, ops)
    ts = time.time() - ts
    sm.lib.sm_destroy(ctx)
    local = {"cg": mine["cg"], "bitwise": {}}
    fix = large_fixture(Nx, Nt, sigma, m0)
    if fix is not None:
        # this shard's share of the reference fixture's sampled x, and the
        # exactly rounded sum of squares of its block of x
        _, ref = fix
        sites = ref["sites"]
        gx, gt = sites // Nt, sites % Nt
        sel = np.nonzero((gt >= t0) & (gt < t0 + Wt))[0]
        loc = gx[sel] * Wt + (gt[sel] - t0)
        xc = mine["x"].view(np.complex128)
        local["fix"] = {"sel": sel.tolist(), "p0": xc[loc].view(np.float64).tolist(),
                        "p1": xc[V + loc].view(np.float64).tolist(), "sumsq": math.fsum(mine["x"] ** 2)}
    for k in ("Dpsi", "Ddagchi", "force"):
        if k in mine:
            ref = np.load(os.path.join(d, f"one_{k}.npy"), mmap_mode="r")
            local["bitwise"][k] = bool(np.array_equal(block_of(ref, Nx, Nt, t0, Wt, k != "force").view(np.uint64),
                                                      mine[k].view(np.uint64)))
    xr = block_of(np.load(os.path.join(d, "one_x.npy"), mmap_mode="r"), Nx, Nt, t0, Wt)
    dx = mine["x"] - xr
    sums = torch.tensor([float(dx @ dx), float(xr @ xr), mine["res_sq"][0], mine["res_sq"][1]], dtype=torch.float64)
    dist.all_reduce(sums)
    gathered = [None] * world
    dist.all_gather_object(gathered, local)
    if rank == 0:
        with open(os.path.join(d, "one.json")) as fh:
            one = json.load(fh)
        rep = {"world": world, "Wt": Wt, "one_cg": one["cg"], "one_relres": (one["res_sq"][0] / one["res_sq"][1]) ** 0.5,
               "cg": [g["cg"] for g in gathered],
               "bitwise": {k: all(g["bitwise"][k] for g in gathered) for k in gathered[0]["bitwise"]},
               "x_rel": float((sums[0] / sums[1]) ** 0.5), "relres": float((sums[2] / sums[3]) ** 0.5),
               "seconds_one": one["seconds"], "seconds_sharded": ts}
        if fix is not None:
            meta, ref = fix
            n = len(ref["sites"])
            samp = np.empty((2, n), np.complex128)
            for g in gathered:
                sel = np.asarray(g["fix"]["sel"], np.int64)
                samp[0, sel] = np.asarray(g["fix"]["p0"]).view(np.complex128)
                samp[1, sel] = np.asarray(g["fix"]["p1"]).view(np.complex128)
            xs, xr = samp.reshape(-1).view(np.float64), ref["ref_cgx"]
            ref_sq = meta["fsum_sq"]["ref_cgx"]
            sq = math.fsum(g["fix"]["sumsq"] for g in gathered)
            rep["fixture"] = {"name": meta["file"], "cg_iters": meta["cg_iters"],
                              "x_rel": float(np.linalg.norm(xs - xr) / np.linalg.norm(xr)),
                              "sumsq_rel": abs(sq - ref_sq) / ref_sq,
                              "spread": meta.get("reference_decomposition_spread", [])}
        with open(result_path, "w") as fh:
            json.dump(rep, fh)
    dist.barrier()
    dist.destroy_process_group()


def run_commworld(name, result_path, dist, rank, world):
    """mode "commworld" (CPU, gloo): bench.py's comm_world over real ranks with
    a stand-in context whose sm_comm_info reports the RCCL rank count given
    per rank in `name` ("<transport>:<n0>,<n1>,..."): the min / max over ranks
    and the refusal when RCCL's own count differs from WORLD_SIZE."""
    sys.path.insert(0, REPO)
    import argparse
    import bench
    transport, counts = name.split(":")
    n = int(counts.split(",")[rank])

    class FakeLattice:
        def comm_info(self):
            return transport, n, rank

    sh = argparse.Namespace(L=FakeLattice())
    args = argparse.Namespace(transport=transport)
    rt = {"world": world, "rank": rank}
    try:
        out = {"ok": bench.comm_world(args, rt, sh)}
    except SystemExit as e:
        out = {"refused": str(e)}
    gathered = [None] * world
    dist.all_gather_object(gathered, out)
    if rank == 0:
        with open(result_path, "w") as f:
            json.dump({"world": world, "ranks": gathered}, f)
    dist.barrier()
    dist.destroy_process_group()


def run_fallback(name, result_path, dist, rank, world):
    """mode "fallback" (CPU, gloo): bench.make_shard's agreement over real
    ranks with stand-in shards. `name`: "ok", "setup:<rank>" (creating the
    peer shard raises on that rank only) or "check" (the peer check fails).
    Every rank must end on the same transport: peer, or RCCL with a reason."""
    sys.path.insert(0, REPO)
    import argparse
    import bench

    class FakeShard:
        def __init__(self, rt, Nx, Nt, sigma, transport=None):
            if transport == "peer" and name.startswith("setup:") and rank == int(name.split(":")[1]):
                raise RuntimeError("stand-in peer setup failure")
            self.kind = transport or "rccl"

        def close(self):
            pass

    bench.Shard = FakeShard
    bench.peer_check = lambda rt, sh, m0: {"ok": name != "check"}
    rt = {"world": world, "rank": rank, "transport": "peer"}
    sh, chk = bench.make_shard(argparse.Namespace(transport="peer"), rt, 64, 64, 0.1, -0.1)
    gathered = [None] * world
    dist.all_gather_object(gathered, {"kind": sh.kind, "check": chk})
    if rank == 0:
        with open(result_path, "w") as f:
            json.dump({"world": world, "ranks": gathered}, f)
    dist.barrier()
    dist.destroy_process_group()


def run_peerfail(name, result_path, dist, rank, world):
    """mode "peerfail" (one GPU, peer transport): every rank connects, then only
    rank 0 applies D and solves; the others stay alive (their regions mapped)
    but never take part. Rank 0's waits must hit the time limit
    (SM_TEST_OPTS peer_wait_ms), sm_peer_status must report it, and the solve
    that follows must fail fast (every later wait gives up at once) instead of
    hanging. The other ranks leave only after rank 0 is done."""
    import time
    import schwingermodel_amd as sm
    from schwingermodel_amd import dist as smd
    from conftest import load_fixture
    meta, a = load_fixture(name)
    Nx, Nt = meta["Nx"], meta["Nt"]
    S = Nx * Nt
    t0, Wt = ctypes.c_int(), ctypes.c_int()
    sm.check(sm.lib.sm_shard_plan(Nt, world, rank, ctypes.byref(t0), ctypes.byref(Wt)))
    V = Nx * Wt.value
    ctx, _ = smd.create_shard_context(Nx, Nt, transport="peer", device=int(os.environ.get("SM_DEVICE", "0")))
    U = shard_field(a["U"], Nx, Nt, t0.value, Wt.value)
    psi = shard_field(a["psi"], Nx, Nt, t0.value, Wt.value)
    P = lambda x: ctypes.c_void_p(x.ctypes.data)  # noqa: E731
    out = {}
    if rank == 0:
        sm.check(sm.lib.sm_upload_gauge(ctx, P(U[0]), P(U[1])))  # (the ghost-link exchange times out here)
        o0, o1 = np.empty(V, complex), np.empty(V, complex)
        t = time.time()
        sm.lib.sm_dirac(ctx, P(psi[0]), P(psi[1]), P(o0), P(o1), meta["m0"], 0)
        seq = ctypes.c_ulonglong(0)
        out["status_rc"] = sm.lib.sm_peer_status(ctx, ctypes.byref(seq))
        out["status_msg"] = sm.lib.sm_last_error().decode()
        out["timed_out_seq"] = seq.value
        out["apply_s"] = time.time() - t
        x0, x1 = np.empty(V, complex), np.empty(V, complex)
        res = sm.CGResult()
        t = time.time()
        out["cg_rc"] = sm.lib.sm_cg(ctx, P(psi[0]), P(psi[1]), P(x0), P(x1), meta["m0"], 1e-10, 200, ctypes.byref(res))
        out["cg_msg"] = sm.lib.sm_last_error().decode()
        out["cg_s"] = time.time() - t
        with open(result_path, "w") as f:
            json.dump(out, f)
    dist.barrier()
    sm.lib.sm_destroy(ctx)
    dist.barrier()
    dist.destroy_process_group()


def main():
    mode, name, result_path = sys.argv[1], sys.argv[2], sys.argv[3]
    import datetime
    import torch.distributed as dist
    print(f"[worker {os.environ.get('RANK')}] init_process_group", file=sys.stderr, flush=True)
    dist.init_process_group("gloo", timeout=datetime.timedelta(minutes=20))
    rank, world = dist.get_rank(), dist.get_world_size()
    print(f"[worker {rank}/{world}] {mode} {name}", file=sys.stderr, flush=True)
    if mode == "md":
        return run_md(name, result_path, dist, rank, world)
    if mode == "eo":
        return run_eo(name, result_path, dist, rank, world)
    if mode == "eocg":
        return run_eocg(name, result_path, dist, rank, world)
    if mode == "angles":
        return run_angles(name, result_path, dist, rank, world)
    if mode == "big":
        return run_big(name, result_path, dist, rank, world)
    if mode == "commworld":
        return run_commworld(name, result_path, dist, rank, world)
    if mode == "fallback":
        return run_fallback(name, result_path, dist, rank, world)
    if mode == "peerfail":
        return run_peerfail(name, result_path, dist, rank, world)
    from conftest import bits_equal, load_fixture
    import schwingermodel_amd as sm
    from schwingermodel_amd import dist as smd

    if name.startswith("gen:"):
        # gen:<Nx>x<Nt>:<sigma>:<m0> -- synthetic fields; reference = one shard on this GPU
        _, dims, sigma, m0s = name.split(":")
        Nx, Nt = (int(v) for v in dims.split("x"))
        sigma, m0 = float(sigma), float(m0s)
        S = Nx * Nt
        a = {k: np.empty(4 * S) for k in ("U", "psi", "chi")}
        sm.lib.sm_fill_gauge(4321, sigma, Nt, 0, Nx, 0, Nt, a["U"].ctypes.data, a["U"][2 * S:].ctypes.data)
        sm.lib.sm_fill_spinor(5678, Nt, 0, Nx, 0, Nt, a["psi"].ctypes.data, a["psi"][2 * S:].ctypes.data)
        sm.lib.sm_fill_spinor(91011, Nt, 0, Nx, 0, Nt, a["chi"].ctypes.data, a["chi"][2 * S:].ctypes.data)
        meta = {"Nx": Nx, "Nt": Nt, "m0": m0}
        if rank == 0:
            single_reference(sm, a, meta)
    else:
        meta, a = load_fixture(name)
        Nx, Nt, m0 = meta["Nx"], meta["Nt"], meta["m0"]
    t0, Wt = ctypes.c_int(), ctypes.c_int()
    sm.check(sm.lib.sm_shard_plan(Nt, world, rank, ctypes.byref(t0), ctypes.byref(Wt)))
    t0, Wt = t0.value, Wt.value
    V = Nx * Wt
    U = shard_field(a["U"], Nx, Nt, t0, Wt)
    psi = shard_field(a["psi"], Nx, Nt, t0, Wt)
    chi = shard_field(a["chi"], Nx, Nt, t0, Wt)
    P = lambda x: ctypes.c_void_p(x.ctypes.data)  # noqa: E731
    local = {}

    if mode == "oracle":
        o = ctypes.CDLL(os.path.join(REPO, "oracle", "liboracle.so"))
        vp, ci, cd = ctypes.c_void_p, ctypes.c_int, ctypes.c_double
        o.oracle_dirac_local.argtypes = [ci, ci, ci, ci] + [vp] * 11 + [cd, ci]
        # ghost link U_t(x, -1): the down-neighbour's U_t(x, Wt-1)
        ulo, uhi = faces(U[0], U[1], Nx, Wt)
        g_lo, g_hi = np.empty(4 * Nx), np.empty(4 * Nx)
        smd.exchange_faces(ulo, uhi, g_lo, g_hi)
        for key, src, dag in (("ref_Dpsi", psi, 0), ("ref_Ddagchi", chi, 1)):
            lo, hi = faces(src[0], src[1], Nx, Wt)
            r_lo, r_hi = np.empty(4 * Nx), np.empty(4 * Nx)
            smd.exchange_faces(lo, hi, r_lo, r_hi)
            out0, out1 = np.empty(V, complex), np.empty(V, complex)
            o.oracle_dirac_local(Nx, Wt, t0, Nt, P(U[0]), P(U[1]), P(src[0]), P(src[1]),
                                 P(r_lo[:2 * Nx]), P(r_lo[2 * Nx:]), P(g_lo[:2 * Nx]),
                                 P(r_hi[:2 * Nx]), P(r_hi[2 * Nx:]), P(out0), P(out1), m0, dag)
            local[key] = (out0, out1)
    else:
        ctx, tr = smd.create_shard_context(Nx, Nt, transport=TRANSPORT, device=int(os.environ.get("SM_DEVICE", "0")))
        ci = [ctypes.c_int(-1) for _ in range(3)]
        sm.check(sm.lib.sm_comm_info(ctx, *(ctypes.byref(v) for v in ci)))
        local["comm_info"] = tuple(v.value for v in ci)  # host-staged: transport 1, no RCCL world
        ip = ctypes.c_int(-1)
        sm.check(sm.lib.sm_cg_sums_in_pass(ctx, ctypes.byref(ip)))
        local["sums_in_pass"] = ip.value
        sm.check(sm.lib.sm_upload_gauge(ctx, P(U[0]), P(U[1])))
        for key, src, fn in (("ref_Dpsi", psi, 0), ("ref_Ddagchi", chi, 1), ("ref_DDdagpsi", psi, 2)):
            out0, out1 = np.empty(V, complex), np.empty(V, complex)
            if fn < 2:
                sm.check(sm.lib.sm_dirac(ctx, P(src[0]), P(src[1]), P(out0), P(out1), m0, fn))
            else:
                sm.check(sm.lib.sm_ddag(ctx, P(src[0]), P(src[1]), P(out0), P(out1), m0))
            local[key] = (out0, out1)
        F0, F1 = np.empty(V), np.empty(V)
        sm.check(sm.lib.sm_force(ctx, P(psi[0]), P(psi[1]), P(chi[0]), P(chi[1]), P(F0), P(F1)))
        local["ref_force"] = (F0, F1)
        x0, x1 = np.empty(V, complex), np.empty(V, complex)
        res = sm.CGResult()
        sm.check(sm.lib.sm_cg(ctx, P(psi[0]), P(psi[1]), P(x0), P(x1), m0, 1e-10, 10000, ctypes.byref(res)))
        local["ref_cgx"] = (x0, x1)
        local["cg"] = (res.converged, res.iterations)
        z = np.empty(2)
        sm.check(sm.lib.sm_dot(ctx, P(chi[0]), P(chi[1]), P(psi[0]), P(psi[1]), P(z)))
        local["dot"] = tuple(z)
        sm.lib.sm_destroy(ctx)

    gathered = [None] * world
    dist.all_gather_object(gathered, local)
    if rank == 0:
        report = {"world": world, "mode": mode, "fixture": name, "checks": {}, "Wt": Wt}
        for key in ("ref_Dpsi", "ref_Ddagchi", "ref_DDdagpsi", "ref_force", "ref_cgx"):
            if key not in local:
                continue
            dtype = float if key == "ref_force" else complex
            g = unshard([d[key] for d in gathered], Nx, Nt, Wt, dtype)
            if key == "ref_cgx":
                report["checks"][key] = float(np.linalg.norm(g - a[key]) / np.linalg.norm(a[key]))
            else:
                report["checks"][key] = bool(bits_equal(g, a[key]))
        if "cg" in local:
            report["cg_iters"] = [d["cg"][1] for d in gathered]
            report["cg_converged"] = [d["cg"][0] for d in gathered]
            report["ref_cg_iters"] = meta["cg_iters"]
            report["dots"] = [list(d["dot"]) for d in gathered]
        if "comm_info" in local:
            report["comm_info"] = [list(d["comm_info"]) for d in gathered]
            report["sums_in_pass"] = [d.get("sums_in_pass") for d in gathered]
        with open(result_path, "w") as f:
            json.dump(report, f)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    import faulthandler
    import signal
    faulthandler.register(signal.SIGUSR1, all_threads=True)  # distutil.run_world: stack dump on a timeout
    if os.environ.get("SM_WORKER_WATCHDOG"):  # thread-based dump, works whatever the main thread is doing
        faulthandler.dump_traceback_later(float(os.environ["SM_WORKER_WATCHDOG"]), exit=False)
    main()
