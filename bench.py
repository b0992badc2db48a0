#!/usr/bin/env python3
"""Benchmark of the hot path: CG on D D^dagger + the Wilson-Dirac apply, fp64.

Metric (BASELINE.json): CG iterations/s and Dirac-apply achieved HBM GB/s on a
4096 x 4096 lattice (beta = 5 synthetic U(1) field, sigma = 0.2374, m0 = -0.06),
at 1/2/4/8 GPUs.

One "step" = one CG iteration (src/conjugate_gradient.cpp:31-63): Ad = D D^dag d,
<d,Ad>, x += alpha d, r -= alpha Ad, <r,r>, stop test, d = beta d + r -- all on
device, inputs resident in HBM. The CG runs with tol = 0 so every timed
iteration does the full work.

Workloads (BASELINE.json configs):
  --config 3  (default for N = 1)  4096^2, beta=5 field, m0=-0.06, one GPU.
  --config 4  (default for N > 1)  the SAME 4096^2 lattice sharded along t over
              the N GPUs (strong scaling: N = 1 and N = 8 run one workload).
              The weak-scaling variant of config 4 (4096 x 512N, so N = 8 is
              4096^2) is measured too and reported under "weak".
  --config 5  8192^2, beta=2 field (sigma 0.4242), m0=-0.19 (near m_crit),
              sharded over N GPUs: CG to 1e-10 from x0 = phi (the reference's
              start), time to solution, iterations and the true residual.

Multi-GPU: one process per GPU. Launched by the driver as
`python -m torch.distributed.run --nproc-per-node N bench.py --gpus N`
(WORLD_SIZE must equal --gpus). `python bench.py --gpus N` with no
WORLD_SIZE spawns the N ranks itself, before anything touches the GPU.
torch.distributed (gloo) is control plane only: the RCCL unique id / the peer
regions' IPC handles, barriers and the max-over-ranks timing.

Transports (N > 1): `--transport rccl` (the default, north_star's "RCCL halo
exchange over xGMI") carries the headline `value`; the same run then times
the device-initiated peer transport on the same workload as the extra key
`peer_transport` (include/sm_hip.h sm_create_peer: kernels store faces and
sums straight into the other GPUs' regions over xGMI; `--no-peer` skips it).
Before timing the peer transport every rank checks it against the
host-staged transport on the same shard (D and D^dag bitwise, 30 CG
iterations to 1e-12); after timing, both transports' timed solves are
checked against themselves (recursive against true residual).
`--transport peer` makes the peer transport the headline (falling back to
RCCL if its check or setup fails anywhere); `--transport hosted` runs the
shards over the host-staged transport (several ranks may share one GPU;
tests / rehearsal; `--device 0` puts peer ranks on one GPU too).
"""
import argparse
import ctypes
import json
import os
import re
import socket
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

SEED_U, SEED_CHI = 4321, 91011
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
BYTES_PER_SITE_APPLY = 96  # read psi 32 + U 32, write 32
# algorithmic HBM bytes per site of one CG iteration, by path
BYTES_PER_SITE_CG = {"recompute": 160, "twodir": 224, "sixkernel": 576}
# the recompute-Ad pass streams 128 B/site besides the links; it reads the
# links as exact codes (sm_cg_link_codes, csrc/sm_linkcode.h): 17 B/site with
# both links' flag nibbles packed in one byte (fresh fields), 20 with 16-bit
# flag words, 32 as complex links (sm_cg_link_bytes reports which)
BYTES_PER_SITE_CG_NOLINKS = 128
CG_PATH_ID = {"recompute": 5, "twodir": 4, "sixkernel": 0}

# BASELINE.json configs on the GPU (1 and 2 are the CPU-plumbing / 1024^2 parity cases)
CONFIGS = {
    3: dict(Nx=4096, Nt=4096, sigma=0.2374, m0=-0.06,
            name="config 3: 4096x4096 lattice, beta=5 field, m0=-0.06"),
    4: dict(Nx=4096, Nt=4096, sigma=0.2374, m0=-0.06,
            name="config 4: 4096x4096 lattice (beta=5 field, m0=-0.06) t-sharded over the GPUs (strong)"),
    5: dict(Nx=8192, Nt=8192, sigma=0.4242, m0=-0.19,
            name="config 5: 8192x8192 lattice near m_crit (beta=2 field, m0=-0.19), CG to 1e-10"),
}


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None, help="ranks (default: WORLD_SIZE, else 1)")
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--applies", type=int, default=100, help="timed Dirac applies")
    ap.add_argument("--config", type=int, choices=[3, 4, 5], default=None,
                    help="BASELINE.json config (default: 3 on one GPU, 4 on several)")
    ap.add_argument("--nx", type=int, default=None, help="override the config's lattice (tests)")
    ap.add_argument("--nt", type=int, default=None)
    ap.add_argument("--no-weak", action="store_true", help="skip the weak-scaling extra of config 3/4")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=None,
                    help="host cores for the CPU baseline (default: this process's CPU share)")
    ap.add_argument("--cpu-iters", type=int, default=50, help="CG iterations of the CPU baseline sample")
    ap.add_argument("--transport", choices=["rccl", "peer", "hosted"], default="rccl",
                    help="multi-GPU wire of the headline: RCCL, the device-initiated peer transport (checked "
                         "against the host-staged one first, RCCL if that fails), or the host-staged test transport")
    ap.add_argument("--no-peer", action="store_true",
                    help="N > 1 with --transport rccl (or hosted): skip the extra timing of the peer transport")
    ap.add_argument("--device", type=int, default=None, help="override the rank -> GPU mapping")
    ap.add_argument("--cg-path", choices=list(CG_PATH_ID), default="recompute")
    ap.add_argument("--rank-timeout", type=float, default=900.0,
                    help="seconds before a rank that has not finished (e.g. stuck in ncclCommInitRank or a "
                         "mismatched collective) dumps its stacks and exits 124; the spawner then ends the others")
    ap.add_argument("--no-link-angles", action="store_true",
                    help="recompute-Ad CG reads the complex links (160 B/site) instead of their exact "
                         "codes (145 or 148; the default from 4M sites per shard)")
    ap.add_argument("--evolved-trajectories", type=int, default=50,
                    help="N = 1: also time the CG on the field after this many pure-gauge leapfrog "
                         "trajectories (the HMC's link update; 0 skips)")
    return ap.parse_args(argv)


# --------------------------------------------------------------------------- launch

def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn_ranks(n, argv=None, timeout=900.0, script=None, poll=0.2):
    """`bench.py --gpus N` without a launcher: start N fresh rank processes
    (nothing in this parent touches the GPU) and wait for them with a
    deadline. The first rank to fail, or the deadline, ends the others
    (SIGTERM, then SIGKILL): a hung rank fails the job loudly instead of
    holding the node. Returns the worst exit code (124 on the deadline)."""
    port = str(_free_port())
    argv = sys.argv[1:] if argv is None else argv
    script = script or os.path.abspath(__file__)
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, script] + list(argv), env=env))
    rc = 0
    deadline = time.monotonic() + timeout
    try:
        while True:
            codes = [p.poll() for p in procs]
            bad = [c for c in codes if c not in (None, 0)]
            if bad:
                rc = max(abs(c) for c in bad) or 1
                print(f"[bench] a rank exited with {bad[0]}: ending the others", file=sys.stderr)
                break
            if all(c == 0 for c in codes):
                break
            if time.monotonic() > deadline:
                rc = 124
                print(f"[bench] ranks still running after {timeout:.0f} s: ending them", file=sys.stderr)
                break
            time.sleep(poll)
    finally:
        for p in procs:
            if p.poll() is None:
                p.terminate()
        for p in procs:
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
    return rc


def start_rank_watchdog(seconds):
    """In-process deadline for a rank (also under torch.distributed.run): dump
    every thread's stack to stderr and exit 124, so a rank stuck in a
    collective fails the job instead of hanging it (the launcher then ends
    the other ranks)."""
    import faulthandler
    import threading

    def fire():
        print(f"[bench] rank {os.environ.get('RANK', '0')}: no result after {seconds:.0f} s, exiting 124",
              file=sys.stderr, flush=True)
        faulthandler.dump_traceback(file=sys.stderr, all_threads=True)
        sys.stderr.flush()
        os._exit(124)

    t = threading.Timer(seconds, fire)
    t.daemon = True
    t.start()
    return t


# --------------------------------------------------------------------------- CPU baseline

def cpu_share():
    """Host cores this process may use: the affinity mask, capped by
    OMP_NUM_THREADS (the GPU box sets it to the box's CPU share; nproc there
    shows the whole machine)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return max(1, n)


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def decompose(threads):
    """ranks_x x ranks_t <= threads, both powers of two (they must divide the
    power-of-two lattice, include/mpi_setup.h:6-23), both >= 2 (the reference
    deadlocks when either is 1), as square as possible."""
    p = 1 << (max(4, threads).bit_length() - 1)
    k = p.bit_length() - 1
    rx = 1 << ((k + 1) // 2)
    return rx, p // rx


def cpu_baseline(cfg, threads, ncg):
    """CPU reference timed on this host on a bounded sample of the same workload.

    Preferred: the unmodified reference (oracle/_ref/sm_ref_<Nx>x<Nt>, built in
    the dev container from /root/reference) under MPI with a 2D decomposition.
    Fallback: the bit-exact oracle restatement (one thread)."""
    Nx, Nt, m0, sigma = cfg["Nx"], cfg["Nt"], cfg["m0"], cfg["sigma"]
    exe = os.path.join(REPO, "oracle", "_ref", f"sm_ref_{Nx}x{Nt}")
    mpirun = "/opt/conda/bin/mpirun"
    model = cpu_model()
    # >= 4 threads: both ranks_x and ranks_t >= 2 (the reference's halos to
    # itself deadlock under MPICH when either is 1)
    if os.path.exists(exe) and os.path.exists(mpirun) and threads >= 4:
        rx, rt = decompose(threads)
        cmd = [mpirun, "-n", str(rx * rt), exe, "bench", str(rx), str(rt), str(SEED_U),
               repr(sigma), str(SEED_CHI), repr(m0), "3", str(ncg)]
        try:
            # the reference's blocking sends rely on eager delivery (tests/golden/make_golden.py
            # MPI_EAGER_ENV): transport settings only
            env = dict(os.environ, HOSTNAME=os.environ.get("HOSTNAME", "localhost"), OMP_NUM_THREADS="1",
                       MPIR_CVAR_NEMESIS_SHM_EAGER_MAX_SZ="1048576", MPIR_CVAR_CH3_EAGER_MAX_MSG_SIZE="1048576")
            out = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env)
            if out.returncode == 0:
                r = json.loads(out.stdout.strip().splitlines()[-1])
                return {"value": r["cg_it_per_s"], "unit": f"CG iterations/s ({Nx}x{Nt})",
                        "cores": rx * rt, "kind": "reference", "cpu_model": model,
                        "decomposition": f"MPI ranks_x={rx} x ranks_t={rt}",
                        "sample": f"{r['cg_iters']} CG iterations (tol 0) + 3 D applies at {Nx}x{Nt}, "
                                  f"unmodified reference (oracle/_ref) under MPICH, {rx}x{rt} ranks, 1 thread each",
                        "dirac_apply_GBps": r["apply_GBps"]}
            print(f"[bench] reference CPU baseline rc={out.returncode}: {out.stderr[-400:]}", file=sys.stderr)
        except Exception as e:  # noqa: BLE001 -- fall through to the port
            print(f"[bench] reference CPU baseline failed: {e}", file=sys.stderr)
    # oracle port: single-threaded CG, a few iterations (test checker used as the timed baseline)
    import numpy as np
    import schwingermodel_amd as sm
    o = ctypes.CDLL(os.path.join(REPO, "oracle", "liboracle.so"))
    vp, ci, cd = ctypes.c_void_p, ctypes.c_int, ctypes.c_double
    o.oracle_cg.argtypes = [ci, ci, vp, vp, vp, vp, vp, vp, cd, cd, ci, ctypes.POINTER(ci), ctypes.POINTER(cd)]
    S = Nx * Nt
    U0, U1, p0, p1 = (np.empty(2 * S) for _ in range(4))
    sm.lib.sm_fill_gauge(SEED_U, sigma, Nt, 0, Nx, 0, Nt, U0.ctypes.data, U1.ctypes.data)
    sm.lib.sm_fill_spinor(SEED_CHI, Nt, 0, Nx, 0, Nt, p0.ctypes.data, p1.ctypes.data)
    x0, x1 = np.empty(2 * S), np.empty(2 * S)
    it, err = ctypes.c_int(), ctypes.c_double()
    n = max(2, min(ncg, 8))
    t = time.perf_counter()
    o.oracle_cg(Nx, Nt, U0.ctypes.data, U1.ctypes.data, p0.ctypes.data, p1.ctypes.data,
                x0.ctypes.data, x1.ctypes.data, m0, 0.0, n, ctypes.byref(it), ctypes.byref(err))
    dt = time.perf_counter() - t
    return {"value": it.value / dt, "unit": f"CG iterations/s ({Nx}x{Nt})", "cores": 1, "kind": "port",
            "cpu_model": model, "decomposition": "1 thread",
            "sample": f"{it.value} CG iterations (incl. initial DD^dag) at {Nx}x{Nt}, oracle/sm_oracle.c"}


def lib_build_id():
    """sm_build_id() of the library this process runs (schwingermodel_amd/build.py
    source_id: a hash of its sources and flags); None for a build without it."""
    import schwingermodel_amd as sm
    fn = getattr(sm.lib, "sm_build_id", None)
    if fn is None:
        return None
    fn.restype = ctypes.c_char_p
    return fn().decode()


def load_traffic(nx, nt, build_id):
    """HBM bytes per launch of the Dirac apply and of the CG pass from a
    committed rocprofv3 PMC summary (profiles/*_dslash_pmc.json, FETCH_SIZE +
    WRITE_SIZE with the gfx950 rule, tools/summarize_prof.py) of THIS build:
    the newest summary (natural order) whose build_id is the running
    library's and which holds this local shape. A summary of another build is
    never cited. Returns (file, apply bytes, CG pass bytes) or None."""
    best = None
    pdir = os.path.join(REPO, "profiles")
    if build_id and os.path.isdir(pdir):
        def natural(f):
            return [int(t) if t.isdigit() else t for t in re.split(r"(\d+)", f)]
        for f in sorted(os.listdir(pdir), key=natural):
            if f.endswith("_dslash_pmc.json"):
                try:
                    with open(os.path.join(pdir, f)) as fh:
                        d = json.load(fh)
                    if d.get("build_id") == build_id and d.get("Nx") == nx and d.get("Nt") == nt:
                        best = (f, d.get("hbm_bytes_per_launch"), d.get("cg_pass_hbm_bytes_per_launch"))
                except Exception:  # noqa: BLE001
                    pass
    return best


# --------------------------------------------------------------------------- GPU side

class Shard:
    """This rank's t-shard of an Nx x Nt lattice with its fields resident in HBM."""

    def __init__(self, rt, Nx, Nt, sigma, transport=None):
        import torch
        import schwingermodel_amd as sm
        from schwingermodel_amd import dist as smd
        self.sm, self.rt = sm, rt
        world, rank, device = rt["world"], rt["rank"], rt["device"]
        if Nt % world:
            raise SystemExit(f"Nt={Nt} is not divisible by {world} GPUs")
        self.kind = (transport or rt["transport"]) if world > 1 else None
        self.transport = None
        if world > 1 and self.kind in ("hosted", "peer"):
            ctx, self.transport = smd.create_shard_context(Nx, Nt, device=device, transport=self.kind)
            L = sm.Lattice.__new__(sm.Lattice)
            L.ctx, L.Nx, L.Nt, L.Wt, L.t0 = ctx, Nx, Nt, Nt // world, rank * (Nt // world)
            L.V, L.shard, L.nshard = Nx * L.Wt, rank, world
        else:
            uid = smd.broadcast_unique_id() if world > 1 else None
            L = sm.Lattice(Nx, Nt, nshard=world, shard=rank, device=device, unique_id=uid)
        self.L, self.Nx, self.Nt, self.Wt, self.V = L, Nx, Nt, L.Wt, L.V
        sm.check(sm.lib.sm_set_stream(L.ctx, ctypes.c_void_p(rt["stream"].cuda_stream)))
        # synthetic inputs (counter-based: each shard makes its own slice, no transfer)
        U = torch.empty(4 * self.V, dtype=torch.float64)
        chi = torch.empty(4 * self.V, dtype=torch.float64)
        _fill(sm, Nx, Nt, L.t0, L.Wt, sigma, U.numpy(), chi.numpy())
        self.U = U.cuda()
        self.phi = chi.cuda()
        del U, chi
        self.x = torch.empty_like(self.phi)
        self.out = torch.empty_like(self.phi)
        sm.check(sm.lib.sm_upload_gauge_dev(L.ctx, self.p(self.U)))

    @staticmethod
    def p(t):
        return ctypes.c_void_p(t.data_ptr())

    def close(self):
        self.L.close()


def peer_check(rt, sh, m0, iters=30):
    """The peer transport against the host-staged one on this rank's shard,
    before anything is timed: D and D^dag of the bench RHS must be bitwise
    equal, and `iters` CG iterations (tol 0, same x0) within 1e-12 of each
    other (the passes' partial sums are added in another tile order, so the
    iterates agree to rounding). Every rank runs it; the verdict is the worst
    over ranks. A stale or missing face anywhere shows as a bitwise mismatch
    of D on the shard that read it."""
    import torch
    sm = sh.sm
    from schwingermodel_amd import dist as smd
    ctx_h, tr_h = smd.create_hosted_context(sh.Nx, sh.Nt, device=rt["device"])
    outs = {}
    try:
        sm.check(sm.lib.sm_set_stream(ctx_h, ctypes.c_void_p(rt["stream"].cuda_stream)))
        sm.check(sm.lib.sm_upload_gauge_dev(ctx_h, sh.p(sh.U)))
        for name, ctx in (("peer", sh.L.ctx), ("hosted", ctx_h)):
            o = [torch.empty_like(sh.phi) for _ in range(2)]
            for dag in (0, 1):
                sm.check(sm.lib.sm_dirac_dev(ctx, sh.p(sh.phi), sh.p(o[dag]), m0, dag))
            x = torch.empty_like(sh.phi)
            sm.check(sm.lib.sm_cg_begin(ctx, sh.p(sh.phi), sh.p(x), m0, 0.0))
            sm.check(sm.lib.sm_cg_iterate(ctx, iters))
            res = sm.CGResult()
            sm.check(sm.lib.sm_cg_finish(ctx, ctypes.byref(res)))
            torch.cuda.synchronize()
            outs[name] = (o, x, res.iterations)
    finally:
        sm.lib.sm_destroy(ctx_h)
        del tr_h
    (op, xp, ip), (oh, xh, ih) = outs["peer"], outs["hosted"]
    d_bad = float(not (torch.equal(op[0], oh[0]) and torch.equal(op[1], oh[1])))
    num, den = float(torch.sum((xp - xh) ** 2)), float(torch.sum(xh ** 2))
    bad, it_bad, num, den = max_over_ranks(rt, [d_bad, float(ip != ih), num, den])
    # (the max of the per-rank sums bounds the global ones' ratio within a factor N)
    rel = (num / den) ** 0.5 if den > 0 else float("inf")
    ok = bad == 0.0 and it_bad == 0.0 and rel <= 1e-12
    return {"against": "host-staged transport, same shard", "D_Ddag_bitwise": bad == 0.0,
            "cg_iterations": iters, "cg_x_rel": rel, "ok": ok}


def make_shard(args, rt, Nx, Nt, sigma, m0, fallback=True):
    """This rank's shard over args.transport; for the peer transport (N > 1)
    after peer_check, falling back to RCCL on every rank if the setup or the
    check failed on any (fallback=False: no shard, (None, report)). Returns
    (shard, check report or None)."""
    if rt["world"] == 1 or args.transport != "peer":
        return Shard(rt, Nx, Nt, sigma), None
    err, sh, chk = "", None, None
    try:
        sh = Shard(rt, Nx, Nt, sigma, "peer")
    except Exception as e:  # noqa: BLE001 -- every rank must reach the vote below
        err = f"peer setup: {e}"
    (bad,) = max_over_ranks(rt, [float(bool(err))])
    if not bad:
        chk = peer_check(rt, sh, m0)
        if not chk["ok"]:
            err = "peer transport differs from the host-staged one"
    elif not err:
        err = "peer setup failed on another rank"
    if not err:
        return sh, chk
    print(f"[bench] rank {rt['rank']}: {err}" + ("; falling back to RCCL" if fallback else ""), file=sys.stderr,
          flush=True)
    if sh is not None:
        sh.close()
    if not fallback:
        return None, dict(chk or {}, ok=False, reason=err)
    return Shard(rt, Nx, Nt, sigma, "rccl"), dict(chk or {}, fallback="rccl", reason=err)


def time_peer(args, rt, Nx, Nt, sigma, m0):
    """N > 1 beside the RCCL headline: the same workload over the peer
    transport (checked first; nothing is timed if the check fails), the CG
    steps and the Dirac apply timed exactly as the headline's, and the timed
    solve checked against itself."""
    import argparse
    a = argparse.Namespace(**vars(args))
    a.transport = "peer"
    sh, chk = make_shard(a, rt, Nx, Nt, sigma, m0, fallback=False)
    if sh is None:
        return {"transport_check": chk}
    try:
        begin_cg(sh, m0, args.cg_path, args.no_link_angles)
        apply_time = time_applies(rt, sh, m0, args.applies)
        t_cg, _ = time_cg_steps(rt, sh, m0, args.cg_path, args.warmup, args.steps, args.no_link_angles, begun=True)
        apply_s = apply_time()
        solve = timed_solve_check(sh, m0)
        t_cg, apply_s = max_over_ranks(rt, [t_cg, apply_s])
        (bad,) = max_over_ranks(rt, [float(not solve["ok"])])
    finally:
        sh.close()
    return {"value": round(args.steps / t_cg, 3), "ms_per_step": round(1e3 * t_cg / args.steps, 4),
            "unit": f"CG iterations/s (one {Nx}x{Nt} lattice over all GPUs)",
            "dirac_apply_us": round(apply_s * 1e6, 2),
            "dirac_apply_GBps": round(BYTES_PER_SITE_APPLY * sh.V / apply_s / 1e9, 1),
            "transport_check": chk, "timed_solve_check": dict(solve, ok_all_ranks=bad == 0.0)}


def _fill(sm, Nx, Nt, t0, Wt, sigma, U, chi, nthreads=8):
    """Row blocks of the counter-based generator in threads (it is row-separable)."""
    from concurrent.futures import ThreadPoolExecutor
    V = Nx * Wt
    rows = max(1, -(-Nx // nthreads))

    def job(x0):
        nx = min(rows, Nx - x0)
        off = 2 * x0 * Wt
        sm.lib.sm_fill_gauge(SEED_U, sigma, Nt, x0, nx, t0, Wt, U[off:].ctypes.data, U[2 * V + off:].ctypes.data)
        sm.lib.sm_fill_spinor(SEED_CHI, Nt, x0, nx, t0, Wt, chi[off:].ctypes.data, chi[2 * V + off:].ctypes.data)
    with ThreadPoolExecutor(nthreads) as ex:
        list(ex.map(job, range(0, Nx, rows)))


def barrier(rt):
    import torch
    import torch.distributed as dist
    torch.cuda.synchronize()
    if rt["world"] > 1:
        dist.barrier()


def max_over_ranks(rt, vals):
    from schwingermodel_amd import dist as smd
    return smd.max_over_ranks(vals) if rt["world"] > 1 else list(vals)


def time_applies(rt, sh, m0, n):
    """Dirac apply D, HIP events on the stream the kernel is launched on.
    Returns a function that reads the time per apply: the events are read
    after the CG timing, so the CG warmup passes queue right behind the
    applies and the GPU never idles between the two timed phases (an idle
    gap of a few ms before a solve sends the chip into a ~40-pass clock
    transient, 10-25 % slower passes: tools/cg_transient.py,
    profiles/r03_q_cg_transient.jsonl)."""
    import torch
    sm = sh.sm
    for _ in range(10):
        sm.check(sm.lib.sm_dirac_dev(sh.L.ctx, sh.p(sh.phi), sh.p(sh.out), m0, 0))
    barrier(rt)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(rt["stream"])
    for _ in range(n):
        sm.check(sm.lib.sm_dirac_dev(sh.L.ctx, sh.p(sh.phi), sh.p(sh.out), m0, 0))
    e1.record(rt["stream"])
    return lambda: e0.elapsed_time(e1) / 1e3 / n


def placement_report(sh):
    """The context's placement probe (sm_placement_report): the CG pass time of
    the initial placement of its streamed buffers and after the search of each
    buffer (the library names them, sm_placement_buffer_name), and which
    buffers were re-placed."""
    sm = sh.sm
    us = (ctypes.c_double * 16)()
    n, chosen = ctypes.c_int(0), ctypes.c_int(0)
    sm.check(sm.lib.sm_placement_report(sh.L.ctx, us, ctypes.byref(n), ctypes.byref(chosen)))
    names = []
    while (nm := sm.lib.sm_placement_buffer_name(len(names))) is not None:
        names.append(nm.decode())
    rep = {"us_per_pass": [round(us[k], 1) for k in range(n.value)],
           "moved": [names[i] for i in range(len(names)) if chosen.value >> i & 1]}
    if n.value:
        rep["probe_kept_us"] = rep["us_per_pass"][-1]
    return rep


def check_rccl_world(transport, world, nmin, nmax):
    """The world the transport itself reports (sm_comm_info: ncclCommCount of
    the RCCL communicator, or the shards the peer transport connected), min and
    max over ranks, against the job: with N > 1 every rank's RCCL / peer world
    must hold exactly WORLD_SIZE ranks, or the line would describe a job that
    did not run. Returns None when it holds, else the reason."""
    if transport in ("rccl", "peer") and world > 1 and not nmin == nmax == world:
        return f"{transport} worlds hold {nmin}..{nmax} ranks, WORLD_SIZE is {world}"
    return None


def comm_world(args, rt, sh):
    """{"transport", "rccl_ranks" | "peer_ranks": [min, max] over ranks} from
    sm_comm_info (the transport that actually runs, after any fallback);
    exits non-zero when its own count differs from WORLD_SIZE."""
    transport, n, _ = sh.L.comm_info()
    mx, neg_mn = max_over_ranks(rt, [float(n), float(-n)])
    nmin, nmax = int(-neg_mn), int(mx)
    why = check_rccl_world(transport, rt["world"], nmin, nmax)
    if why:
        raise SystemExit(f"[bench] {why}: refusing to report this run")
    ip = ctypes.c_int(0)
    if hasattr(sh.L, "ctx"):
        sh.sm.check(sh.sm.lib.sm_cg_sums_in_pass(sh.L.ctx, ctypes.byref(ip)))
    return {"transport": transport, ("peer_ranks" if transport == "peer" else "rccl_ranks"): [nmin, nmax],
            "cg_sums": "in-pass" if ip.value else ("collective" if rt["world"] > 1 else "one shard")}


def cg_bytes_per_site(sh, cg_path):
    """Algorithmic bytes per site of the CG iteration the last solve ran."""
    sm = sh.sm
    if cg_path != "recompute":
        return BYTES_PER_SITE_CG[cg_path]
    b = ctypes.c_int(0)
    sm.check(sm.lib.sm_cg_link_bytes(sh.L.ctx, ctypes.byref(b)))
    return BYTES_PER_SITE_CG_NOLINKS + b.value


def begin_cg(sh, m0, cg_path, link_angles_off=False):
    """sm_cg_begin of the timed solve (x0 = phi, r0, d0; the link codes are
    built here, with a host read of their device check): CG setup, not timed."""
    sm = sh.sm
    sm.check(sm.lib.sm_tune_cg(sh.L.ctx, CG_PATH_ID[cg_path], 0))
    sm.check(sm.lib.sm_cg_link_angles(sh.L.ctx, 0 if link_angles_off else -1, None))  # -1: the size default
    sm.check(sm.lib.sm_cg_begin(sh.L.ctx, sh.p(sh.phi), sh.p(sh.x), m0, 0.0))


def time_cg_steps(rt, sh, m0, cg_path, warmup, steps, link_angles_off=False, begun=False):
    """K CG iterations (tol = 0: never converges, the full work every step)
    bracketed by a barrier + device synchronisation on both sides, after W
    untimed warmup iterations."""
    import torch
    sm = sh.sm
    if not begun:
        begin_cg(sh, m0, cg_path, link_angles_off)
    sm.check(sm.lib.sm_cg_iterate(sh.L.ctx, warmup))
    barrier(rt)
    c0, c1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    w0 = time.perf_counter()
    c0.record(rt["stream"])
    sm.check(sm.lib.sm_cg_iterate(sh.L.ctx, steps))
    c1.record(rt["stream"])
    barrier(rt)
    wall = time.perf_counter() - w0
    res = sm.CGResult()
    sm.check(sm.lib.sm_cg_status(sh.L.ctx, ctypes.byref(res)))
    # the one-pass iterations' pass 0 (in the warmup) only forms Ad_0: every
    # later pass is one full reference iteration
    setup_passes = 1 if cg_path in ("twodir", "recompute") else 0
    if res.iterations != warmup + steps - setup_passes or res.converged != 0:
        raise SystemExit(f"CG ran {res.iterations} iterations (converged={res.converged}), "
                         f"expected {warmup + steps - setup_passes}")
    return max(wall, c0.elapsed_time(c1) / 1e3), cg_bytes_per_site(sh, cg_path)


def time_evolved(args, rt, sh, cfg, m0):
    """The CG rate on the bench field after `--evolved-trajectories`
    leapfrog trajectories (sm_quenched_trajectory: HMC::Leapfrog with the gauge
    force, 10 MD steps each, so |U| drifts off 1 by the rounding of
    U <- U exp(i eps P), src/hmc.cpp:70-100). Reports whether the CG pass
    still reads the exact link codes (sm_linkcode.h) and the rate it runs at.
    Not part of the headline timing."""
    sm = sh.sm
    ntraj = args.evolved_trajectories
    prm = sm.HMCParams(m0=m0, beta=5.0, tau=1.0, md_steps=10, cg_tol=1e-10, cg_max_iter=10000, seed=2024,
                       even_odd=0)
    t = time.perf_counter()
    for k in range(ntraj):
        sm.check(sm.lib.sm_quenched_trajectory(sh.L.ctx, ctypes.byref(prm), k))
    t_md = time.perf_counter() - t
    err, bad = ctypes.c_double(-1.0), ctypes.c_long(-1)
    sm.check(sm.lib.sm_link_code_check(sh.L.ctx, None, ctypes.byref(err), ctypes.byref(bad)))
    t_cg, bps = time_cg_steps(rt, sh, m0, args.cg_path, args.warmup, args.steps, args.no_link_angles)
    return {"field": f"config-3 field after {ntraj} pure-gauge leapfrog trajectories (beta 5, 10 MD steps, "
                     "sm_quenched_trajectory)",
            "md_seconds": round(t_md, 3), "links_not_encodable": bad.value, "largest_decode_error": err.value,
            "link_codes_in_use": bps < BYTES_PER_SITE_CG["recompute"], "bytes_per_site": bps,
            "value": round(args.steps / t_cg, 3), "ms_per_step": round(1e3 * t_cg / args.steps, 4),
            "unit": "CG iterations/s"}


def true_relres(sh, m0):
    """||phi - D D^dag x|| / ||phi|| over all shards (sm_dot_dev is global)."""
    import numpy as np
    import torch
    sm = sh.sm
    Ax = torch.empty_like(sh.phi)
    sm.check(sm.lib.sm_ddag_dev(sh.L.ctx, sh.p(sh.x), sh.p(Ax), m0))
    r = sh.phi - Ax
    rr, pp = np.zeros(2), np.zeros(2)
    sm.check(sm.lib.sm_dot_dev(sh.L.ctx, sh.p(r), sh.p(r), ctypes.c_void_p(rr.ctypes.data)))
    sm.check(sm.lib.sm_dot_dev(sh.L.ctx, sh.p(sh.phi), sh.p(sh.phi), ctypes.c_void_p(pp.ctypes.data)))
    return float(np.sqrt(rr[0] / pp[0]))


WIRES = {"rccl": " (RCCL halos over xGMI)", "peer": " (device-initiated stores over xGMI)",
         "hosted": " (host-staged halos)"}


def timed_solve_check(sh, m0):
    """N > 1: the timed solve checked against itself after the timing. The CG's
    recursive residual (sqrt <r,r> from the device scalars, the same on every
    shard) must agree with the true residual ||phi - D D^dag x|| / ||phi|| of
    the x the passes built: a face or a sum lost or stale in any timed pass
    on any shard breaks that agreement, whatever the transport. After ~200
    iterations at tol 0 the two differ by rounding (~1e-13 of ||phi||) against
    a residual of ~1e-3, so the bar (1e-6 relative) is loose and still catches
    any wrong pass."""
    sm = sh.sm
    res = sm.CGResult()
    sm.check(sm.lib.sm_cg_finish(sh.L.ctx, ctypes.byref(res)))
    rec = res.residual / res.phi_norm if res.phi_norm else float("nan")
    true = true_relres(sh, m0)
    ok = abs(true - rec) <= 1e-6 * rec
    return {"recursive_relres": rec, "true_relres": true, "ok": bool(ok)}


def base_line(args, rt, cfg, Nx, Nt, sh):
    world = rt["world"]
    return {
        "metric": "CG iterations/sec + Dirac-apply achieved HBM GB/s, 4096^2 fp64, 1/2/4/8 GPU",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "higher_is_better": True,
        "vs_baseline": None,
        "dtype": "f64",
        "data": f"synthetic (counter-based U(1) field theta~N(0,{cfg['sigma']}^2) seed {SEED_U}, "
                f"complex-Gaussian RHS seed {SEED_CHI})",
        "config": {"workload": cfg["name"] + (f" [overridden: {Nx}x{Nt}]" if (Nx, Nt) != (cfg["Nx"], cfg["Nt"])
                                                 else ""),
                   "Nx": Nx, "Nt": Nt, "m0": cfg["m0"], "sigma": cfg["sigma"],
                   "sites_per_gpu": sh.V, "shard": f"{Nx}x{sh.Wt}",
                   "transport": sh.kind if world > 1 else None,
                   "parallelism": f"t-shard x{world}" + (WIRES[sh.kind] if world > 1 else "")},
    }


def run_config34(args, rt, cfg_id):
    import torch  # noqa: F401
    cfg = CONFIGS[cfg_id]
    Nx, Nt = args.nx or cfg["Nx"], args.nt or cfg["Nt"]
    m0, world, rank = cfg["m0"], rt["world"], rt["rank"]
    sh, tcheck = make_shard(args, rt, Nx, Nt, cfg["sigma"], m0)
    placement = placement_report(sh)
    world_seen = comm_world(args, rt, sh)
    begin_cg(sh, m0, args.cg_path, args.no_link_angles)
    apply_time = time_applies(rt, sh, m0, args.applies)
    t_cg, cg_bps = time_cg_steps(rt, sh, m0, args.cg_path, args.warmup, args.steps, args.no_link_angles, begun=True)
    apply_s = apply_time()
    solve_check = timed_solve_check(sh, m0) if world > 1 else None
    t_cg, apply_s = max_over_ranks(rt, [t_cg, apply_s])
    if "probe_kept_us" in placement:
        # the probe times short bursts; the timed run sustains its own pass time
        # (both are reported)
        placement["sustained_us_per_pass"] = round(1e6 * t_cg / args.steps, 1)
    V = sh.V
    evolved = time_evolved(args, rt, sh, cfg, m0) if world == 1 and args.evolved_trajectories > 0 else None
    sh.close()
    weak = None
    if not args.no_weak:
        # config 4's weak-scaling curve: 4096 x 512N sites, 4096 x 512 per GPU
        wNt = (Nt // 8) * world
        shw = Shard(rt, Nx, wNt, cfg["sigma"], sh.kind)
        tw, _ = time_cg_steps(rt, shw, m0, args.cg_path, args.warmup, args.steps, args.no_link_angles)
        (tw,) = max_over_ranks(rt, [tw])
        weak = {"lattice": f"{Nx}x{wNt}", "sites_per_gpu": shw.V, "ms_per_step": round(1e3 * tw / args.steps, 4),
                "value": round(args.steps / tw * world, 3),
                "unit": f"CG iterations/s of a {Nx}x{Nt // 8}-site slab per GPU, whole job (it/s x N)",
                "scaling": "weak"}
        shw.close()
    peer = None
    # (also beside the host-staged headline: the one-GPU rehearsal of this path)
    if world > 1 and args.transport in ("rccl", "hosted") and not args.no_peer:
        peer = time_peer(args, rt, Nx, Nt, cfg["sigma"], m0)
    if rank != 0:
        return
    it_per_s = args.steps / t_cg
    apply_GBps = BYTES_PER_SITE_APPLY * V / apply_s / 1e9
    line = base_line(args, rt, cfg, Nx, Nt, sh)
    line.update({
        "value": round(it_per_s, 3),
        "unit": f"CG iterations/s (one {Nx}x{Nt} lattice over all GPUs)",
        "ms_per_step": round(1e3 * t_cg / args.steps, 4),
        "scaling": "strong",
    })
    # the CPU reference beside every N (north_star: "next to the reference MPI
    # path timed on the same box's host cores"), on rank 0 after the GPU
    # timing: the same whole lattice, a bounded sample
    cpu = None
    if not args.no_cpu_baseline:
        cpu = cpu_baseline(dict(cfg, Nx=Nx, Nt=Nt), args.cpu_threads or cpu_share(), args.cpu_iters)
    bid = lib_build_id()
    tr = load_traffic(Nx, sh.Wt, bid)
    line.update({
        "dirac_apply_GBps": round(apply_GBps, 1),
        "dirac_apply_us": round(apply_s * 1e6, 2),
        "roofline": {"bound": "hbm", "achieved": round(apply_GBps, 1), "peak": HBM_PEAK_GBPS,
                     "unit": "GB/s", "frac": round(apply_GBps / HBM_PEAK_GBPS, 4),
                     "traffic": tr[1] if tr else None,
                     "traffic_source": tr[0] if tr else f"no PMC summary of build {bid} under profiles/",
                     "build_id": bid,
                     "kernel": f"dslash_kernel<D>, {BYTES_PER_SITE_APPLY} B/site algorithmic x {V} sites per launch"},
        "cpu_baseline": cpu,
        # the CG iteration's own streaming rate (informational; the graded
        # roofline is the Dirac apply's): algorithmic bytes / time per step
        "cg_iteration": {"path": args.cg_path, "link_codes": cg_bps < BYTES_PER_SITE_CG["recompute"],
                         "bytes_per_site": cg_bps,
                         "achieved_GBps_per_gpu": round(cg_bps * V * it_per_s / 1e9, 1),
                         "frac_of_peak": round(cg_bps * V * it_per_s / 1e9 / HBM_PEAK_GBPS, 4),
                         # counter bytes of the pass kernel (one launch = one iteration), same PMC file
                         "traffic": tr[2] if tr and len(tr) > 2 else None,
                         "traffic_bytes_per_site": round(tr[2] / V, 2) if tr and len(tr) > 2 and tr[2] else None,
                         "reference_sequence_bytes_per_site": 576},
        "weak": weak,
        "hmc_evolved_field": evolved,
        "placement_probe": placement,
        "comm": world_seen,
    })
    if tcheck is not None:
        line["comm"]["transport_check"] = tcheck
    if solve_check is not None:
        line["comm"]["timed_solve_check"] = solve_check
    if peer is not None:
        line["peer_transport"] = peer
    print(json.dumps(line), flush=True)
    if solve_check is not None and not solve_check["ok"]:
        raise SystemExit("[bench] the timed sharded solve's recursive and true residuals disagree")


def run_config5(args, rt):
    cfg = CONFIGS[5]
    Nx, Nt = args.nx or cfg["Nx"], args.nt or cfg["Nt"]
    m0, world, rank = cfg["m0"], rt["world"], rt["rank"]
    sm = None
    sh, tcheck = make_shard(args, rt, Nx, Nt, cfg["sigma"], m0)
    placement = placement_report(sh)
    world_seen = comm_world(args, rt, sh)
    sm = sh.sm
    sm.check(sm.lib.sm_tune_cg(sh.L.ctx, CG_PATH_ID[args.cg_path], 0))
    sm.check(sm.lib.sm_cg_link_angles(sh.L.ctx, 0 if args.no_link_angles else -1, None))
    tol = 1e-10
    # warm the kernels once on a short solve, then the timed solve from x0 = phi
    res = sm.CGResult()
    sm.check(sm.lib.sm_cg_dev(sh.L.ctx, sh.p(sh.phi), sh.p(sh.x), m0, tol, 5, ctypes.byref(res)))
    barrier(rt)
    t = time.perf_counter()
    sm.check(sm.lib.sm_cg_dev(sh.L.ctx, sh.p(sh.phi), sh.p(sh.x), m0, tol, 100000, ctypes.byref(res)))
    barrier(rt)
    dt = time.perf_counter() - t
    (dt,) = max_over_ranks(rt, [dt])
    rel = true_relres(sh, m0)
    cg_bps = cg_bytes_per_site(sh, args.cg_path)
    V = sh.V
    line = base_line(args, rt, cfg, Nx, Nt, sh)
    sh.close()
    if rank != 0:
        return
    line.update({
        "value": round(res.iterations / dt, 3),
        "unit": f"CG iterations/s (one {Nx}x{Nt} lattice over all GPUs, solve to tol 1e-10)",
        "ms_per_step": round(1e3 * dt / max(1, res.iterations), 4),
        "steps": res.iterations, "warmup": 0,
        "scaling": "strong",
        "time_to_solution_s": round(dt, 4),
        "iterations": res.iterations, "converged": res.converged,
        "cg_residual_rel": res.residual / res.phi_norm if res.phi_norm else None,
        "true_relres": rel,
        "cg_iteration": {"path": args.cg_path, "link_codes": cg_bps < BYTES_PER_SITE_CG["recompute"],
                         "bytes_per_site": cg_bps,
                         "achieved_GBps_per_gpu": round(cg_bps * V * res.iterations / dt / 1e9, 1)},
        "placement_probe": placement,
        "comm": world_seen,
    })
    if tcheck is not None:
        line["comm"]["transport_check"] = tcheck
    print(json.dumps(line), flush=True)
    if not res.converged or not rel < 1e-9:
        raise SystemExit(f"config 5: converged={res.converged} true relres {rel:.3e}")


def main():
    args = parse()
    env_world = os.environ.get("WORLD_SIZE")
    if args.gpus is None:
        args.gpus = int(env_world) if env_world else 1
    if args.gpus < 1:
        raise SystemExit("--gpus must be >= 1")
    if env_world is None and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus, timeout=args.rank_timeout + 60))
    world = int(env_world or "1")
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}: refusing to measure the wrong job")
    rank = int(os.environ.get("RANK", "0"))
    watchdog = start_rank_watchdog(args.rank_timeout)
    local_rank = int(os.environ.get("LOCAL_RANK", str(rank)))
    cfg_id = args.config or (3 if world == 1 else 4)
    if cfg_id == 3 and world > 1:
        cfg_id = 4

    import torch
    import torch.distributed as dist
    ndev = torch.cuda.device_count()  # does not initialise the GPU on this image
    if args.device is not None:
        device = args.device
        if args.transport == "rccl" and world > 1:
            raise SystemExit("--device with --transport rccl: RCCL needs one GPU per rank")
    elif args.transport == "hosted":
        device = local_rank % max(1, ndev)
    else:
        if world > 1 and ndev < int(os.environ.get("LOCAL_WORLD_SIZE", world)):
            raise SystemExit(f"{world} RCCL ranks need one GPU each, {ndev} visible (use --transport hosted)")
        device = local_rank
    if world > 1:
        dist.init_process_group("gloo")
    torch.cuda.set_device(device)
    # a real (non-null) torch stream: the library launches on it, so the torch
    # events bracket exactly the kernels being timed
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    rt = {"world": world, "rank": rank, "device": device, "stream": stream, "transport": args.transport}
    try:
        if cfg_id == 5:
            run_config5(args, rt)
        else:
            run_config34(args, rt, cfg_id)
    finally:
        if world > 1:
            dist.destroy_process_group()
        watchdog.cancel()


if __name__ == "__main__":
    main()
