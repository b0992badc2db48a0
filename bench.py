#!/usr/bin/env python3
"""Benchmark of the hot path: CG on D D^dagger + the Wilson-Dirac apply, fp64.

Metric (BASELINE.json): CG iterations/s and Dirac-apply achieved HBM GB/s on a
4096 x 4096 lattice (beta = 5 synthetic U(1) field, sigma = 0.2374, m0 = -0.06).

One "step" = one CG iteration (src/conjugate_gradient.cpp:31-63): Ad = D D^dag d,
<d,Ad>, x += alpha d, r -= alpha Ad, <r,r>, stop test, d = beta d + r -- all on
device, inputs resident in HBM. The CG runs with tol = 0 so every timed
iteration does the full work.

Multi-GPU (python -m torch.distributed.run --nproc-per-node N bench.py --gpus N):
one process per GPU, the lattice sharded along t with RCCL halos; weak scaling,
each GPU owns 4096 x 4096 sites (global lattice 4096 x 4096N). `value` is the
whole-job rate in 4096^2-lattice CG iterations per second (= it/s x N).
`--strong` instead splits one fixed 4096 x 4096 lattice over the N GPUs
 and reports that lattice's it/s.
torch.distributed (gloo) is used only for the RCCL unique id, barriers and the
max-over-ranks timing.
"""
import argparse
import ctypes
import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

NX = 4096
NT_PER_GPU = 4096
SIGMA_B5 = 0.2374      # beta = 5
M0 = -0.06
SEED_U, SEED_CHI = 4321, 91011
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
BYTES_PER_SITE_APPLY = 96  # read psi 32 + U 32, write 32
# algorithmic HBM bytes per site of one CG iteration, by path
BYTES_PER_SITE_CG = {"recompute": 160, "twodir": 224, "onepass": 288, "fused": 320, "fused_inkernel": 320,
                     "sixkernel": 576}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--applies", type=int, default=100, help="timed Dirac applies")
    ap.add_argument("--nx", type=int, default=NX)
    ap.add_argument("--nt-per-gpu", type=int, default=NT_PER_GPU)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=int(os.environ.get("SM_CPU_THREADS", "16")))
    ap.add_argument("--transport", choices=["rccl", "hosted"], default="rccl",
                    help="multi-GPU wire: RCCL (production) or the host-staged test transport")
    ap.add_argument("--device", type=int, default=None, help="override LOCAL_RANK -> GPU mapping")
    ap.add_argument("--cg-path", choices=["recompute", "twodir", "onepass", "fused", "fused_inkernel", "sixkernel"],
                    default="recompute")
    ap.add_argument("--strong", action="store_true",
                    help="strong scaling (SURVEY.md §8d config 4): a fixed nx x nt-per-gpu lattice split over the N GPUs")
    return ap.parse_args()


def cpu_baseline(args, threads):
    """CPU reference timed on this host on a bounded sample of the same workload.

    Preferred: the unmodified reference (oracle/_ref/sm_ref_4096x4096, built in
    the dev container) under MPI with a 2D decomposition (ranks_x >= 2; the
    reference deadlocks for ranks_x = 1). Fallback: the oracle
    restatement (single thread CG, threaded D)."""
    exe = os.path.join(REPO, "oracle", "_ref", f"sm_ref_{args.nx}x{args.nt_per_gpu}")
    mpirun = "/opt/conda/bin/mpirun"
    ncg = 12
    if os.path.exists(exe) and os.path.exists(mpirun):
        rx = 4 if threads >= 16 else 2
        rt = max(1, threads // rx)
        cmd = [mpirun, "-n", str(rx * rt), exe, "bench", str(rx), str(rt), str(SEED_U),
               repr(SIGMA_B5), str(SEED_CHI), repr(M0), "3", str(ncg)]
        try:
            env = dict(os.environ, HOSTNAME=os.environ.get("HOSTNAME", "localhost"))
            out = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env)
            if out.returncode == 0:
                r = json.loads(out.stdout.strip().splitlines()[-1])
                return {"value": r["cg_it_per_s"], "unit": "CG iterations/s (4096^2)",
                        "cores": rx * rt, "kind": "reference",
                        "sample": f"{r['cg_iters']} CG iterations + 3 D applies at {args.nx}x{args.nt_per_gpu}, "
                                  f"MPI {rx}x{rt} ranks (unmodified reference via oracle/_ref)",
                        "dirac_apply_GBps": r["apply_GBps"]}
        except Exception as e:  # noqa: BLE001 -- fall through to the port
            print(f"[bench] reference CPU baseline failed: {e}", file=sys.stderr)
    # oracle port: single-threaded CG, a few iterations
    import numpy as np
    o = ctypes.CDLL(os.path.join(REPO, "oracle", "liboracle.so"))
    vp, ci, cd = ctypes.c_void_p, ctypes.c_int, ctypes.c_double
    o.oracle_cg.argtypes = [ci, ci, vp, vp, vp, vp, vp, vp, cd, cd, ci, ctypes.POINTER(ci), ctypes.POINTER(cd)]
    import schwingermodel_amd as sm
    Nx, Nt = args.nx, args.nt_per_gpu
    S = Nx * Nt
    U0, U1, p0, p1 = (np.empty(2 * S) for _ in range(4))
    sm.lib.sm_fill_gauge(SEED_U, SIGMA_B5, Nt, 0, Nx, 0, Nt, U0.ctypes.data, U1.ctypes.data)
    sm.lib.sm_fill_spinor(SEED_CHI, Nt, 0, Nx, 0, Nt, p0.ctypes.data, p1.ctypes.data)
    x0, x1 = np.empty(2 * S), np.empty(2 * S)
    it, err = ctypes.c_int(), ctypes.c_double()
    n = 4
    t = time.perf_counter()
    o.oracle_cg(Nx, Nt, U0.ctypes.data, U1.ctypes.data, p0.ctypes.data, p1.ctypes.data,
                x0.ctypes.data, x1.ctypes.data, M0, 0.0, n, ctypes.byref(it), ctypes.byref(err))
    dt = time.perf_counter() - t
    return {"value": it.value / dt, "unit": "CG iterations/s (4096^2)", "cores": 1, "kind": "port",
            "sample": f"{it.value} CG iterations (incl. initial DD^dag) at {Nx}x{Nt}, oracle/sm_oracle.c"}


def load_traffic(nx, nt):
    """HBM bytes per dslash launch from the committed rocprofv3 PMC summary
    (profiles/*_dslash_pmc.json, FETCH_SIZE x2 + WRITE_SIZE per the gfx950 rule)."""
    best = None
    pdir = os.path.join(REPO, "profiles")
    if os.path.isdir(pdir):
        for f in sorted(os.listdir(pdir)):
            if f.endswith("_dslash_pmc.json"):
                try:
                    with open(os.path.join(pdir, f)) as fh:
                        d = json.load(fh)
                    if d.get("Nx") == nx and d.get("Nt") == nt:
                        best = d.get("hbm_bytes_per_launch")
                except Exception:  # noqa: BLE001
                    pass
    return best


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    import numpy as np
    import torch
    import torch.distributed as dist
    import schwingermodel_amd as sm
    from schwingermodel_amd import dist as smd

    if world > 1:
        dist.init_process_group("gloo")
    device = local_rank if args.device is None else args.device
    torch.cuda.set_device(device)

    def barrier():
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()

    Nx, Wt = args.nx, args.nt_per_gpu
    if args.strong:
        if Wt % world:
            raise SystemExit(f"--strong: Nt={Wt} is not divisible by {world} GPUs")
        Wt //= world
    Nt = Wt * world
    transport = None
    if world > 1 and args.transport == "hosted":
        ctx, transport = smd.create_hosted_context(Nx, Nt, device=device)
        L = sm.Lattice.__new__(sm.Lattice)
        L.ctx, L.Nx, L.Nt, L.Wt, L.t0, L.V = ctx, Nx, Nt, Wt, rank * Wt, Nx * Wt
    else:
        uid = smd.broadcast_unique_id() if world > 1 else None
        L = sm.Lattice(Nx, Nt, nshard=world, shard=rank, device=device, unique_id=uid)
    V = L.V
    t0 = L.t0
    # a real (non-null) torch stream: the library launches on it, so the torch
    # events below bracket exactly the kernels being timed
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    sm.check(sm.lib.sm_set_stream(L.ctx, ctypes.c_void_p(stream.cuda_stream)))

    # synthetic inputs of the benchmark shape (counter-based: each shard makes its slice)
    U = torch.empty(4 * V, dtype=torch.float64)
    chi = torch.empty(4 * V, dtype=torch.float64)
    Un, cn = U.numpy(), chi.numpy()
    sm.lib.sm_fill_gauge(SEED_U, SIGMA_B5, Nt, 0, Nx, t0, Wt, Un.ctypes.data, Un[2 * V:].ctypes.data)
    sm.lib.sm_fill_spinor(SEED_CHI, Nt, 0, Nx, t0, Wt, cn.ctypes.data, cn[2 * V:].ctypes.data)
    dU = U.cuda()
    phi = chi.cuda()
    x = torch.empty_like(phi)
    out = torch.empty_like(phi)
    sm.check(sm.lib.sm_upload_gauge_dev(L.ctx, ctypes.c_void_p(dU.data_ptr())))
    del U, chi

    # ---- Dirac apply: HIP events on the stream the kernel is launched on ----
    for _ in range(10):
        sm.check(sm.lib.sm_dirac_dev(L.ctx, ctypes.c_void_p(phi.data_ptr()), ctypes.c_void_p(out.data_ptr()), M0, 0))
    barrier()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(args.applies):
        sm.check(sm.lib.sm_dirac_dev(L.ctx, ctypes.c_void_p(phi.data_ptr()), ctypes.c_void_p(out.data_ptr()), M0, 0))
    e1.record(stream)
    barrier()
    apply_s = e0.elapsed_time(e1) / 1e3 / args.applies
    apply_GBps = BYTES_PER_SITE_APPLY * V / apply_s / 1e9

    sm.check(sm.lib.sm_tune_cg(L.ctx, {"recompute": 5, "twodir": 4, "onepass": 3, "fused": 1, "fused_inkernel": 2, "sixkernel": 0}[args.cg_path], 0))
    # ---- CG iterations (tol = 0: never converges, full work every step) ----
    sm.check(sm.lib.sm_cg_begin(L.ctx, ctypes.c_void_p(phi.data_ptr()), ctypes.c_void_p(x.data_ptr()), M0, 0.0))
    sm.check(sm.lib.sm_cg_iterate(L.ctx, args.warmup))
    barrier()
    c0, c1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    w0 = time.perf_counter()
    c0.record(stream)
    sm.check(sm.lib.sm_cg_iterate(L.ctx, args.steps))
    c1.record(stream)
    barrier()
    wall = time.perf_counter() - w0
    res = sm.CGResult()
    sm.check(sm.lib.sm_cg_status(L.ctx, ctypes.byref(res)))
    # the one-pass iteration's pass 0 (in the warmup) only forms Ad_0: every
    # later pass is one full reference iteration
    setup_passes = 1 if args.cg_path in ("onepass", "twodir", "recompute") else 0
    assert res.iterations == args.warmup + args.steps - setup_passes and res.converged == 0
    t_ev = c0.elapsed_time(c1) / 1e3
    t_local = max(wall, t_ev)
    if world > 1:
        t_local, apply_s = smd.max_over_ranks([t_local, apply_s])
        apply_GBps = BYTES_PER_SITE_APPLY * V / apply_s / 1e9

    if rank == 0:
        it_per_s = args.steps / t_local
        # weak: 4096^2-lattice iterations per second, whole job; strong: the
        # one fixed lattice's iterations per second
        value = it_per_s if args.strong else it_per_s * world
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline(args, args.cpu_threads)
        traffic = load_traffic(Nx, Wt)
        line = {
            "metric": "CG iterations/sec + Dirac-apply achieved HBM GB/s, 4096^2 fp64",
            "value": round(value, 3),
            "unit": (f"CG iterations/s (one {Nx}x{Nt} lattice over all GPUs)" if args.strong
                     else f"CG iterations/s ({Nx}x{Wt} sites per GPU, whole job)"),
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1e3 * t_local / args.steps, 4),
            "higher_is_better": True,
            "scaling": "strong" if args.strong else "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (counter-based U(1) field theta~N(0,0.2374^2), complex-Gaussian RHS)",
            "config": {"workload": f"CG on D D^dag, {Nx}x{Nt} lattice (beta=5 field, m0={M0}), "
                                   f"t-sharded over {world} GPU(s)",
                       "transport": args.transport if world > 1 else None,
                       "Nx": Nx, "Nt": Nt, "sites_per_gpu": V, "m0": M0, "sigma": SIGMA_B5,
                       "parallelism": f"t-shard x{world}" + (" (RCCL halos)" if world > 1 else "")},
            "dirac_apply_GBps": round(apply_GBps, 1),
            "dirac_apply_us": round(apply_s * 1e6, 2),
            "roofline": {"bound": "hbm", "achieved": round(apply_GBps, 1), "peak": HBM_PEAK_GBPS,
                         "unit": "GB/s", "frac": round(apply_GBps / HBM_PEAK_GBPS, 4),
                         "traffic": traffic,
                         "kernel": "dslash_kernel<D> (96 B/site algorithmic)"},
            "cpu_baseline": cpu,
            # the CG iteration's own streaming rate (informational; the graded
            # roofline is the Dirac apply's): algorithmic bytes / time per step
            "cg_iteration": {"path": args.cg_path, "bytes_per_site": BYTES_PER_SITE_CG[args.cg_path],
                             "achieved_GBps": round(BYTES_PER_SITE_CG[args.cg_path] * V * it_per_s / 1e9, 1),
                             "reference_sequence_bytes_per_site": 576},
        }
        print(json.dumps(line), flush=True)
    L.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
