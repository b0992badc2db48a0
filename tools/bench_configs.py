#!/usr/bin/env python3
"""Time-to-solution for the BASELINE.json configs on one GPU (JSON lines).

    python tools/bench_configs.py [--configs 2,3,5] [--hmc]

config 2: 1024^2, beta=3 field (sigma 0.3246), m0=-0.10, CG to 1e-10
config 3: 4096^2, beta=5 field (sigma 0.2374), m0=-0.06, CG to 1e-10
config 5: 8192^2, beta=2 field (sigma 0.4242), m0=-0.19 (near m_crit), CG to 1e-10,
          here on ONE GPU (8 GiB per field fits the 288 GB HBM)
--hmc:    config 1 (64^2, beta=2, m0=0, 10 MD steps) with the parameters of the
          recorded reference run (manifest "hmc_stat": 50 + 100 + 99 trajectories):
          `sm_hmc` (whole HMC on the device), the reference program with its
          D/CG on the GPU through the drop-in shim (oracle/_ref/SM_64x64_hip),
          and with --hmc-ref the unmodified CPU reference (SM_64x64_ref, ~4 min).
--hmc-large N: seconds per device HMC trajectory at N^2 (beta=3 field start,
          m0=0.10, tau=0.5, 10 MD steps), the MD step at production size.
Inputs are resident in HBM before timing; the solve includes sm_cg_begin
(x0 = phi, r0, norms) and the final x update, like conjugate_gradient().
"""
import argparse
import ctypes
import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

CONFIGS = {
    2: dict(N=1024, sigma=0.3246, m0=-0.10),
    3: dict(N=4096, sigma=0.2374, m0=-0.06),
    5: dict(N=8192, sigma=0.4242, m0=-0.19),
}


def fill_parallel(sm, N, sigma, U, p, nthreads=16):
    """Counter-based generator is row-separable: fill row blocks in threads."""
    from concurrent.futures import ThreadPoolExecutor
    V = N * N
    rows = max(1, N // nthreads)

    def job(x0):
        nx = min(rows, N - x0)
        off = 2 * x0 * N
        sm.lib.sm_fill_gauge(4321, sigma, N, x0, nx, 0, N, U[off:].ctypes.data, U[2 * V + off:].ctypes.data)
        sm.lib.sm_fill_spinor(91011, N, x0, nx, 0, N, p[off:].ctypes.data, p[2 * V + off:].ctypes.data)
    with ThreadPoolExecutor(nthreads) as ex:
        list(ex.map(job, range(0, N, rows)))


def run_config(cid, tol=1e-10):
    import torch
    import schwingermodel_amd as sm
    c = CONFIGS[cid]
    N = c["N"]
    V = N * N
    L = sm.Lattice(N, N)
    s = torch.cuda.Stream()
    torch.cuda.set_stream(s)
    vp = ctypes.c_void_p
    sm.check(sm.lib.sm_set_stream(L.ctx, vp(s.cuda_stream)))
    U = torch.empty(4 * V, dtype=torch.float64)
    p = torch.empty(4 * V, dtype=torch.float64)
    t = time.perf_counter()
    fill_parallel(sm, N, c["sigma"], U.numpy(), p.numpy())
    gen_s = time.perf_counter() - t
    dU, dp = U.cuda(), p.cuda()
    del U, p
    x = torch.empty_like(dp)
    sm.check(sm.lib.sm_upload_gauge_dev(L.ctx, vp(dU.data_ptr())))
    torch.cuda.synchronize()
    res = sm.CGResult()
    t = time.perf_counter()
    sm.check(sm.lib.sm_cg_dev(L.ctx, vp(dp.data_ptr()), vp(x.data_ptr()), c["m0"], tol, 100000, ctypes.byref(res)))
    torch.cuda.synchronize()
    dt = time.perf_counter() - t
    # independent true residual |phi - D D^dag x| / |phi|
    Ax = torch.empty_like(dp)
    sm.check(sm.lib.sm_ddag_dev(L.ctx, vp(x.data_ptr()), vp(Ax.data_ptr()), c["m0"]))
    torch.cuda.synchronize()
    relres = float(torch.linalg.vector_norm(dp - Ax) / torch.linalg.vector_norm(dp))
    out = {"config": cid, "lattice": f"{N}x{N}", "sigma": c["sigma"], "m0": c["m0"], "tol": tol,
           "converged": res.converged, "iterations": res.iterations, "seconds": round(dt, 4),
           "it_per_s": round(res.iterations / dt, 1), "ms_per_it": round(1e3 * dt / max(1, res.iterations), 4),
           "true_relres": relres, "host_gen_s": round(gen_s, 2)}
    L.close()
    return out


def run_hmc(with_ref=False):
    import re
    import tempfile
    with open(os.path.join(REPO, "tests", "golden", "manifest.json")) as f:
        c = json.load(f)["hmc_stat"]
    params = (f"1\n1\n{c['m0']}\n{c['md_steps']}\n{c['tau']}\n{c['beta']}\n{c['Ntherm']}\n{c['Nmeas']}\n"
              f"{c['Nsteps']}\n0\n")
    ntraj = c["Ntherm"] + c["Nmeas"] + c["Nsteps"] * (c["Nmeas"] - 1)
    out = {"config": 1, "lattice": "64x64", "trajectories": ntraj,
           "params": {k: c[k] for k in ("m0", "md_steps", "tau", "beta", "Ntherm", "Nmeas", "Nsteps")},
           "reference_recorded": {k: c[k] for k in ("Ep", "dEp", "acceptance", "seconds")}}
    progs = {"sm_hmc": [os.path.join(REPO, "schwingermodel_amd", "sm_hmc"), "64", "64", "1"],
             "sm_hmc_even_odd": [os.path.join(REPO, "schwingermodel_amd", "sm_hmc"), "64", "64", "1", "--even-odd"],
             "dropin_shim": [os.path.join(REPO, "oracle", "_ref", "SM_64x64_hip")]}
    if with_ref:
        progs["reference_cpu"] = [os.path.join(REPO, "oracle", "_ref", "SM_64x64_ref")]
    env = dict(os.environ, HOSTNAME=os.environ.get("HOSTNAME", "box"))
    for tag, cmd in progs.items():
        if not os.path.exists(cmd[0]):
            out[tag] = None
            continue
        with tempfile.TemporaryDirectory() as d:
            t = time.perf_counter()
            r = subprocess.run(cmd, input=params, capture_output=True, text=True, env=env, cwd=d, timeout=1200)
            dt = time.perf_counter() - t
        ep = re.search(r"Ep = (\S+) dEp = (\S+)", r.stdout)
        acc = re.search(r"Acceptance rate: (\S+)", r.stdout)
        rep = re.search(r"Execution time = (\S+) s", r.stdout)
        out[tag] = {"wall_s": round(dt, 2), "hmc_s": float(rep.group(1)) if rep else None,
                    "Ep": float(ep.group(1)) if ep else None, "dEp": float(ep.group(2)) if ep else None,
                    "acceptance_stdout": float(acc.group(1)) if acc else None,
                    "rc": r.returncode, "err": r.stderr[-300:] if r.returncode else ""}
    return out


def run_hmc_large(N, ntraj=3, even_odd=0):
    import ctypes
    import schwingermodel_amd as sm
    L = sm.Lattice(N, N)
    sm.check(sm.lib.sm_fill_gauge_dev(L.ctx, 4321, 0.3246))
    p = sm.HMCParams(0.10, 3.0, 0.5, 10, 1e-10, 10000, 7, even_odd)
    rows = []
    for traj in range(ntraj):
        r = sm.HMCResult()
        t = time.perf_counter()
        sm.check(sm.lib.sm_hmc_trajectory(L.ctx, ctypes.byref(p), traj, ctypes.byref(r)))
        dt = time.perf_counter() - t
        rows.append({"traj": traj, "seconds": round(dt, 3), "cg_iterations": r.cg_iterations, "dH": r.dH,
                     "accepted": r.accepted, "ms_per_cg_it": round(1e3 * dt / max(1, r.cg_iterations), 4)})
    L.close()
    return {"hmc_large": f"{N}x{N}", "even_odd": even_odd, "beta": 3.0, "m0": 0.10, "tau": 0.5, "md_steps": 10,
            "trajectories": rows}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="2,3,5")
    ap.add_argument("--hmc", action="store_true")
    ap.add_argument("--hmc-ref", action="store_true", help="with --hmc: also the CPU reference (~4 min)")
    ap.add_argument("--hmc-large", type=int, default=0)
    ap.add_argument("--tag", default="", help="cg_path tag added to every line")
    a = ap.parse_args()

    def emit(d):
        if a.tag:
            d["cg_path"] = a.tag
        print(json.dumps(d), flush=True)

    for cid in [int(v) for v in a.configs.split(",") if v]:
        emit(run_config(cid))
    if a.hmc:
        emit(run_hmc(a.hmc_ref))
    if a.hmc_large:
        emit(run_hmc_large(a.hmc_large))
        emit(run_hmc_large(a.hmc_large, even_odd=1))


if __name__ == "__main__":
    main()
