#!/usr/bin/env python3
"""Generate the golden fixtures in tests/golden/ from the REFERENCE itself.

Test infrastructure only. Runs in the dev container, where /root/reference
exists: `make -C oracle ref` compiles the unmodified reference sources
(src/variables.cpp, src/dirac_operator.cpp, src/conjugate_gradient.cpp) with
our driver oracle/ref_harness.cpp into oracle/_ref/sm_ref_<Nx>x<Nt>. For each
fixture this script

  1. writes the inputs U, psi, chi with the counter-based generator
     (`sm_ref_* gen`, schwingermodel_amd/csrc/sm_fields.h),
  2. runs the reference on them (`sm_ref_* fixture`, single rank) and keeps
     D psi, D^dag chi, D D^dag psi, phi_dag_partialD_phi(U, psi, chi) and the
     CG solution of D D^dag x = psi (tol 1e-10, max_iter 10000 as
     src/main.cpp:26-27) plus the CG iteration count,
  3. optionally re-runs on a 2x2 MPI decomposition (`--mpi`) and records that
     the reference is decomposition-invariant (bitwise for D/D^dag/force).

Output: tests/golden/<name>.npz (inputs + outputs, float64, the reference's
global layout: two planes of interleaved complex, n = x*Nt + t) and
tests/golden/manifest.json. The fixtures are data, not reference source.
"""
import argparse
import hashlib
import json
import math
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF_DIR = os.path.join(REPO, "oracle", "_ref")

SEED_U, SEED_PSI, SEED_CHI = 4321, 5678, 91011

# name, Nx, Nt, sigma (>0 Gaussian theta, <0 hot, 0 cold), m0
FIXTURES = [
    ("l4x2_hot_m0p2", 4, 2, -1.0, 0.2),
    ("l8x8_hot_m0p2", 8, 8, -1.0, 0.2),
    ("l8x8_cold_m0", 8, 8, 0.0, 0.0),
    ("l16x16_b2_m-0p19", 16, 16, 0.4242, -0.19),
    ("l32x48_b3_m-0p10", 32, 48, 0.3246, -0.10),
    ("l32x48_hot_m0", 32, 48, -1.0, 0.0),
    ("l40x24_hot_m0p2", 40, 24, -1.0, 0.2),
    ("l64x64_b2_m0", 64, 64, 0.4242, 0.0),
    ("l64x64_b5_m-0p06", 64, 64, 0.2374, -0.06),
]

OUTS = ["ref_Dpsi", "ref_Ddagchi", "ref_DDdagpsi", "ref_force", "ref_cgx"]

# Molecular-dynamics fixtures: the reference's gauge / HMC code
# (`sm_ref_* md`) on U (generator), chi (generator) and momenta P (numpy,
# seeded, stored in the fixture): plaquette field, staples, Force_G, Force,
# phi = D chi, Leapfrog -> (U', P'), Hamiltonians before / after.
# name, Nx, Nt, sigma, m0, beta, tau, md_steps
MD_FIXTURES = [
    ("md8x8_b2_m0p1", 8, 8, 0.4242, 0.1, 2.0, 1.0, 5),
    ("md16x16_hot_m0", 16, 16, -1.0, 0.0, 2.0, 1.0, 4),
    ("md32x48_b3_m0p1", 32, 48, 0.3246, 0.1, 3.0, 0.5, 6),
    ("md64x64_b2_m0", 64, 64, 0.4242, 0.0, 2.0, 1.0, 10),
]
MD_OUTS = ["ref_plaq", "ref_staple", "ref_gforce", "ref_phi", "ref_mdforce", "ref_U1", "ref_P1"]
SEED_P = 2468


# The reference's halo exchange posts all its blocking MPI_Send calls before
# its MPI_Recv calls (src/dirac_operator.cpp:66-88), so it relies on eager
# delivery. MPICH's shared-memory eager limit is below 64 KiB, and at 8192^2
# on 2x4 ranks a column halo is 4096 x 16 B = 64 KiB: every rank then waits in
# MPI_Send forever (observed round 4: a 6-hour run that never finished its
# first D_phi). Raising the eager limits changes only the transport, not one
# arithmetic operation of the reference.
MPI_EAGER_ENV = {"MPIR_CVAR_NEMESIS_SHM_EAGER_MAX_SZ": "1048576", "MPIR_CVAR_CH3_EAGER_MAX_MSG_SIZE": "1048576"}


def run(cmd, **kw):
    env = dict(os.environ, HOSTNAME=os.environ.get("HOSTNAME", "localhost"), **MPI_EAGER_ENV)
    r = subprocess.run(cmd, capture_output=True, text=True, env=env, **kw)
    if r.returncode != 0:
        raise RuntimeError(f"{cmd} failed: {r.stderr}")
    return r.stdout


# Large-lattice summary fixtures (BASELINE configs 2, 3 and 5): full outputs
# are too big to commit, so keep the reference's outputs at SAMPLE_SITES seeded
# random sites plus global norms; the GPU test regenerates the inputs with the
# same counter-based generator (bit-exact, tests/test_capi_host.py) and
# compares. name, Nx, Nt, sigma, m0, (ranks_x, ranks_t) of the reference run.
# 1 rank is the reference's own sequential dot order; 8192^2 runs on 2x4 MPI
# ranks (a 1-rank solve there takes ~8 h on one core), which changes only the
# dots' summation order (the operators are decomposition-invariant bitwise,
# manifest "decomposition_2x2").
LARGE = [("l1024x1024_b3_m-0p10", 1024, 1024, 0.3246, -0.10, (1, 1)),
         ("l4096x4096_b5_m-0p06", 4096, 4096, 0.2374, -0.06, (1, 1)),
         ("l8192x8192_b2_m-0p19", 8192, 8192, 0.4242, -0.19, (2, 4))]
SAMPLE_SITES = 4096


def _fsum_sq(a, chunk=1 << 22):
    """Exactly rounded sum of squares of a (math.fsum), streamed in chunks so
    that an 8192^2 field never becomes one Python list."""
    import itertools
    return math.fsum(itertools.chain.from_iterable((a[i:i + chunk] * a[i:i + chunk]).tolist()
                                                   for i in range(0, a.size, chunk)))


def run_large_reference(name, nx, nt, sigma, m0, ranks, workdir, mpirun):
    """Generate the inputs and run the reference's fixture mode in workdir
    (resumable: a finished run leaves meta.json there)."""
    exe = os.path.join(REF_DIR, f"sm_ref_{nx}x{nt}")
    mpath = os.path.join(workdir, "meta.json")
    if os.path.exists(mpath) and os.path.getsize(mpath) > 0:
        with open(mpath) as f:
            return json.load(f)
    os.makedirs(workdir, exist_ok=True)
    run([exe, "gen", workdir, str(SEED_U), repr(sigma), str(SEED_PSI), str(SEED_CHI)])
    rx, rt = ranks
    cmd = [exe, "fixture", workdir, str(rx), str(rt), repr(m0), "1e-10", "10000"]
    if rx * rt > 1:
        cmd = [mpirun, "-n", str(rx * rt)] + cmd
    meta = json.loads(run(cmd))
    with open(mpath, "w") as f:
        json.dump(meta, f)
    return meta


def make_large(name, nx, nt, sigma, m0, ranks, workdir, mpirun):
    meta = run_large_reference(name, nx, nt, sigma, m0, ranks, workdir, mpirun)
    S = nx * nt
    meta_sha, meta_sumsq = {}, {}
    rng = np.random.default_rng(20261015)
    sites = np.sort(rng.choice(S, SAMPLE_SITES, replace=False))
    out = {"sites": sites}
    for k in OUTS:
        a = np.fromfile(os.path.join(workdir, k + ".bin"), dtype=np.float64)
        if k == "ref_force":
            out[k] = np.concatenate([a[:S][sites], a[S:][sites]])
        else:
            c0 = a[:2 * S].view(np.complex128)
            c1 = a[2 * S:].view(np.complex128)
            out[k] = np.concatenate([c0[sites], c1[sites]]).view(np.float64)
        # machine-independent whole-field checks: SHA-256 of the bytes (the
        # bitwise outputs) and the exactly rounded sum of squares (CG x)
        meta_sha[k] = hashlib.sha256(a.tobytes()).hexdigest()
        meta_sumsq[k] = _fsum_sq(a)
        del a
    meta.update({"sigma": sigma, "file": name + ".npz", "summary": True, "sample_sites": SAMPLE_SITES,
                 "sha256": meta_sha, "fsum_sq": meta_sumsq})
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **out)
    return meta


def large_spread(name, ranks, workdir_root, mpirun):
    """The reference's own reduction-order spread for a large fixture: rerun
    its fixture mode on the same inputs with another MPI decomposition (the
    operators are decomposition-invariant bitwise; the dots sum in another
    order) and record the iteration counts and ||x_a - x_b|| / ||x_a||. This
    is the band inside which two correct fp64 CG solves of this system differ
    from each other by rounding order alone."""
    nx, nt = next((e[1], e[2]) for e in LARGE if e[0] == name)
    base = os.path.join(workdir_root, name)
    rx, rt = ranks
    alt = os.path.join(workdir_root, f"{name}_{rx}x{rt}")
    os.makedirs(alt, exist_ok=True)
    for k in ("U", "psi", "chi"):
        dst = os.path.join(alt, k + ".bin")
        if not os.path.exists(dst):
            os.symlink(os.path.join(base, k + ".bin"), dst)
    mpath = os.path.join(alt, "meta.json")
    if os.path.exists(mpath) and os.path.getsize(mpath) > 0:
        with open(mpath) as f:
            meta2 = json.load(f)
    else:
        exe = os.path.join(REF_DIR, f"sm_ref_{nx}x{nt}")
        with open(os.path.join(base, "meta.json")) as f:
            m0 = json.load(f)["m0"]
        cmd = [exe, "fixture", alt, str(rx), str(rt), repr(m0), "1e-10", "10000"]
        if rx * rt > 1:
            cmd = [mpirun, "-n", str(rx * rt)] + cmd
        meta2 = json.loads(run(cmd))
        with open(mpath, "w") as f:
            json.dump(meta2, f)
    xa = np.fromfile(os.path.join(base, "ref_cgx.bin"), dtype=np.float64)
    xb = np.fromfile(os.path.join(alt, "ref_cgx.bin"), dtype=np.float64)
    sa, sb = _fsum_sq(xa), _fsum_sq(xb)
    return {"ranks_x": rx, "ranks_t": rt, "cg_iters": meta2["cg_iters"],
            "cg_true_relres": meta2["cg_true_relres"],
            "x_rel_to_fixture": float(np.linalg.norm(xa - xb) / np.linalg.norm(xa)),
            "sum_x2_rel_to_fixture": abs(sb - sa) / sa}


def make_jackknife():
    """Reference Jackknife_error(dat, 20) and mean(dat) (src/statistics.cpp)
    on seeded series, including lengths that are not multiples of the 20 bins
    and shorter than one sample per bin (the reference's integer binning)."""
    exe = os.path.join(REF_DIR, "sm_ref_8x8")
    rng = np.random.default_rng(1357)
    cases = []
    for n in (3, 19, 20, 22, 45, 100, 257):
        dat = (0.7 + 0.05 * rng.standard_normal(n)).tolist()
        out = run([exe, "jk", "20"] + [repr(v) for v in dat]).split()
        cases.append({"bin": 20, "data": dat, "jackknife_error": float(out[0]), "mean": float(out[1])})
    return cases


# Statistical HMC reference: the unmodified reference
# program (oracle/_ref/SM_64x64_ref, built by `make -C oracle refapp`) on its
# own stdin parameters. Its RNG is seeded from the clock, so parity with it is
# statistical: Ep, gS within their jackknife errors, acceptance close.
HMC_STAT = {"name": "hmc64x64_b2_m0", "Nx": 64, "Nt": 64, "m0": 0.0, "md_steps": 10, "tau": 0.3, "beta": 2.0,
            "Ntherm": 50, "Nmeas": 100, "Nsteps": 1}


def parse_hmc_output(stdout, simdata):
    import re
    ep = re.search(r"Ep = (\S+) dEp = (\S+)", stdout)
    gs = re.search(r"gS = (\S+) dgS = (\S+)", stdout)
    lines = [ln for ln in simdata.splitlines() if ln and not ln.startswith("#")]
    acc_file = float(lines[-2])  # "#Acceptance rate" value, then "#Execution time"
    t = re.search(r"Execution time = (\S+) s", stdout)
    return {"Ep": float(ep.group(1)), "dEp": float(ep.group(2)), "gS": float(gs.group(1)),
            "dgS": float(gs.group(2)), "acceptance": acc_file, "seconds": float(t.group(1))}


def make_hmc_stat(log_dir=None):
    c = HMC_STAT
    params = f"1\n1\n{c['m0']}\n{c['md_steps']}\n{c['tau']}\n{c['beta']}\n{c['Ntherm']}\n{c['Nmeas']}\n{c['Nsteps']}\n0\n"
    exe = os.path.join(REF_DIR, f"SM_{c['Nx']}x{c['Nt']}_ref")
    with tempfile.TemporaryDirectory() as d:
        d = log_dir or d
        if not os.path.exists(os.path.join(d, "run1.log")):
            out = run([exe], input=params, cwd=d, timeout=1800)
        else:
            with open(os.path.join(d, "run1.log")) as f:
                out = f.read()
        sim = [f for f in os.listdir(d) if f.endswith("_SimData.txt")][0]
        with open(os.path.join(d, sim)) as f:
            res = parse_hmc_output(out, f.read())
    return dict(c, **res, program="reference src/main.cpp (CPU, 1 rank)")


def make_hmc_stat_chains(k, prior):
    """k more independent runs of the reference HMC program (it seeds rand()
    from the clock in seconds, src/main.cpp:17, so the starts are 2 s apart),
    run in parallel; returns each chain's statistics and the pooled mean of
    these and the prior recorded chain (independent: error = sqrt(sum dEp^2) / n)."""
    import time
    c = HMC_STAT
    params = f"1\n1\n{c['m0']}\n{c['md_steps']}\n{c['tau']}\n{c['beta']}\n{c['Ntherm']}\n{c['Nmeas']}\n{c['Nsteps']}\n0\n"
    exe = os.path.join(REF_DIR, f"SM_{c['Nx']}x{c['Nt']}_ref")
    chains = []
    with tempfile.TemporaryDirectory() as root:
        procs = []
        for i in range(k):
            d = os.path.join(root, f"chain{i}")
            os.makedirs(d)
            env = dict(os.environ, HOSTNAME=os.environ.get("HOSTNAME", "localhost"))
            p = subprocess.Popen([exe], stdin=subprocess.PIPE, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                                 cwd=d, text=True, env=env)
            p.stdin.write(params)
            p.stdin.close()
            procs.append((d, p))
            time.sleep(2.2)
        for d, p in procs:
            out, err = p.stdout.read(), p.stderr.read()
            p.wait(timeout=3600)
            if p.returncode != 0 or "Ep = " not in out:
                raise SystemExit(f"reference HMC chain failed ({p.returncode}):\n{out[-2000:]}\n{err[-2000:]}")
            sim = [f for f in os.listdir(d) if f.endswith("_SimData.txt")][0]
            with open(os.path.join(d, sim)) as f:
                chains.append(parse_hmc_output(out, f.read()))
    base = {key: HMC_STAT[key] for key in HMC_STAT}
    allc = [{key: prior[key] for key in ("Ep", "dEp", "gS", "dgS", "acceptance", "seconds")}] + chains
    n = len(allc)
    pooled = {
        "Ep": sum(ch["Ep"] for ch in allc) / n,
        "dEp": (sum(ch["dEp"] ** 2 for ch in allc)) ** 0.5 / n,
        "gS": sum(ch["gS"] for ch in allc) / n,
        "dgS": (sum(ch["dgS"] ** 2 for ch in allc)) ** 0.5 / n,
        "acceptance": sum(ch["acceptance"] for ch in allc) / n,
    }
    return dict(base, chains=allc, pooled=pooled, program="reference src/main.cpp (CPU, 1 rank), independent chains")


def make_md(name, nx, nt, sigma, m0, beta, tau, steps, mpi=None):
    exe = os.path.join(REF_DIR, f"sm_ref_{nx}x{nt}")
    S = nx * nt
    with tempfile.TemporaryDirectory() as d:
        run([exe, "gen", d, str(SEED_U), repr(sigma), str(SEED_PSI), str(SEED_CHI)])
        np.random.default_rng(SEED_P).standard_normal(2 * S).tofile(os.path.join(d, "P.bin"))
        args = [repr(m0), repr(beta), repr(tau), str(steps), "1e-10", "10000"]
        meta = json.loads(run([exe, "md", d, "1", "1"] + args, cwd=d))
        arrs = {k: np.fromfile(os.path.join(d, k + ".bin"), dtype=np.float64)
                for k in ["U", "chi", "P"] + MD_OUTS}
        arrs["ref_plaq"] = arrs["ref_plaq"][:2 * S]  # written as two identical planes
        if mpi and nx % 2 == 0 and nt % 2 == 0 and nx >= 4 and nt >= 4:
            meta2 = json.loads(run([mpi, "-n", "4", exe, "md", d, "2", "2"] + args, cwd=d, timeout=900))
            dec = {}
            for k in MD_OUTS:
                a = np.fromfile(os.path.join(d, k + ".bin"), dtype=np.float64)
                if k == "ref_plaq":
                    a = a[:2 * S]
                b = arrs[k]
                dec[k] = "bitwise" if np.array_equal(a.view(np.uint64), b.view(np.uint64)) \
                    else f"max_abs={np.abs(a - b).max():.3e}"
            for k in ("sp", "gauge_action", "H0", "H1"):
                dec[k] = meta2[k]
            meta["decomposition_2x2"] = dec
    meta.update({"sigma": sigma, "file": name + ".npz", "seed_P": SEED_P})
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **arrs)
    return meta


# Gauge-configuration files written by the reference's SaveConf (28-byte
# records) on a 1-rank and a 2x2 decomposition (MPI_Gatherv displacements),
# plus the field its readBinary reads back: name, Nx, Nt, sigma, ranks (rx, rt)
CONF_FIXTURES = [("conf8x8_hot", 8, 8, -1.0, (1, 1)), ("conf32x48_b3", 32, 48, 0.3246, (2, 2))]


def make_conf(name, nx, nt, sigma, ranks, mpirun):
    exe = os.path.join(REF_DIR, f"sm_ref_{nx}x{nt}")
    rx, rt = ranks
    with tempfile.TemporaryDirectory() as d:
        run([exe, "gen", d, str(SEED_U), repr(sigma), str(SEED_PSI), str(SEED_CHI)])
        cmd = [exe, "conf", d, str(rx), str(rt)]
        run(cmd if rx * rt == 1 else [mpirun, "-n", str(rx * rt)] + cmd, timeout=300)
        U = np.fromfile(os.path.join(d, "U.bin"), dtype=np.float64)
        with open(os.path.join(d, "ref_conf.ctxt"), "rb") as f:
            raw = f.read()
        with open(os.path.join(HERE, name + ".ctxt"), "wb") as f:
            f.write(raw)
        back = np.fromfile(os.path.join(d, "ref_conf_read.bin"), dtype=np.float64)
    np.savez_compressed(os.path.join(HERE, name + ".npz"), U=U, ref_conf_read=back)
    return {"Nx": nx, "Nt": nt, "sigma": sigma, "ranks_x": rx, "ranks_t": rt, "file": name + ".npz",
            "ctxt": name + ".ctxt", "bytes": len(raw), "sha256": hashlib.sha256(raw).hexdigest(),
            "program": "reference SaveConf then GaugeConf::readBinary (src/gauge_conf.cpp:378-423, 495-546)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mpi", action="store_true", help="also run 2x2 ranks (mpirun)")
    ap.add_argument("--large", nargs="+", default=None, metavar="NAME",
                    help="(re)make only these summary fixtures (LARGE names): 1024^2 ~4 min on one core, "
                         "4096^2 ~70 min on one core, 8192^2 ~2 h on 2x4 ranks")
    ap.add_argument("--spread", nargs=3, default=None, metavar=("NAME", "RX", "RT"),
                    help="rerun a finished large fixture's reference solve on RX x RT ranks and record the "
                         "reference's own decomposition spread in the manifest")
    ap.add_argument("--large-workdir", default="/tmp/sm_large",
                    help="parent of the per-fixture reference run directories (resumable)")
    ap.add_argument("--mpirun", default="/opt/conda/bin/mpirun")
    ap.add_argument("--md-only", action="store_true", help="regenerate only the MD fixtures")
    ap.add_argument("--hmc-stat", action="store_true", help="(re)run the reference HMC program (~2 min)")
    ap.add_argument("--hmc-log-dir", default=None, help="reuse a finished reference HMC run directory")
    ap.add_argument("--hmc-chains", type=int, default=0,
                    help="run this many more independent reference HMC chains in parallel (~4 min) into hmc_stat_chains")
    ap.add_argument("--conf-only", action="store_true", help="regenerate only the SaveConf fixtures")
    args = ap.parse_args()
    if args.spread:
        name, rx, rt = args.spread[0], int(args.spread[1]), int(args.spread[2])
        sp = large_spread(name, (rx, rt), args.large_workdir, args.mpirun)
        path = os.path.join(HERE, "manifest.json")
        with open(path) as f:
            manifest = json.load(f)
        manifest["large"][name].setdefault("reference_decomposition_spread", []).append(sp)
        with open(path, "w") as f:
            json.dump(manifest, f, indent=1, sort_keys=True)
        print(name, json.dumps(sp), file=sys.stderr)
        return
    if args.large:
        todo = [e for e in LARGE if e[0] in args.large]
        if len(todo) != len(args.large):
            raise SystemExit(f"unknown large fixture in {args.large}; known: {[e[0] for e in LARGE]}")
        subprocess.run(["make", "-C", os.path.join(REPO, "oracle"), "ref",
                        "REF_SIZES=" + " ".join(f"{e[1]}x{e[2]}" for e in todo)], check=True)
        path = os.path.join(HERE, "manifest.json")
        for name, nx, nt, sigma, m0, ranks in todo:
            meta = make_large(name, nx, nt, sigma, m0, ranks, os.path.join(args.large_workdir, name),
                              args.mpirun)
            with open(path) as f:  # re-read: several --large runs may be in flight
                manifest = json.load(f)
            manifest.setdefault("large", {})[name] = meta
            with open(path, "w") as f:
                json.dump(manifest, f, indent=1, sort_keys=True)
            print(name, json.dumps({k: meta[k] for k in ("cg_iters", "cg_true_relres", "cg_seconds")}),
                  file=sys.stderr)
        return
    if args.conf_only:
        sizes = sorted({f"{nx}x{nt}" for _, nx, nt, *_ in CONF_FIXTURES})
        subprocess.run(["make", "-C", os.path.join(REPO, "oracle"), "ref", "REF_SIZES=" + " ".join(sizes)],
                       check=True)
        path = os.path.join(HERE, "manifest.json")
        with open(path) as f:
            manifest = json.load(f)
        manifest["conf"] = {n: make_conf(n, nx, nt, sg, rk, args.mpirun) for n, nx, nt, sg, rk in CONF_FIXTURES}
        with open(path, "w") as f:
            json.dump(manifest, f, indent=1, sort_keys=True)
        return
    if args.hmc_chains:
        path = os.path.join(HERE, "manifest.json")
        with open(path) as f:
            manifest = json.load(f)
        manifest["hmc_stat_chains"] = make_hmc_stat_chains(args.hmc_chains, manifest["hmc_stat"])
        print(json.dumps(manifest["hmc_stat_chains"]["pooled"]), file=sys.stderr)
        with open(path, "w") as f:
            json.dump(manifest, f, indent=1, sort_keys=True)
        return
    if args.hmc_stat:
        path = os.path.join(HERE, "manifest.json")
        with open(path) as f:
            manifest = json.load(f)
        manifest["hmc_stat"] = make_hmc_stat(args.hmc_log_dir)
        print(json.dumps(manifest["hmc_stat"]), file=sys.stderr)
        with open(path, "w") as f:
            json.dump(manifest, f, indent=1, sort_keys=True)
        return
    if args.md_only:
        sizes = sorted({f"{nx}x{nt}" for _, nx, nt, *_ in MD_FIXTURES})
        subprocess.run(["make", "-C", os.path.join(REPO, "oracle"), "ref", "oracle",
                        "REF_SIZES=" + " ".join(sizes)], check=True)
        path = os.path.join(HERE, "manifest.json")
        with open(path) as f:
            manifest = json.load(f)
        manifest["md"] = {}
        for name, nx, nt, sigma, m0, beta, tau, steps in MD_FIXTURES:
            manifest["md"][name] = make_md(name, nx, nt, sigma, m0, beta, tau, steps,
                                           args.mpirun if args.mpi else None)
            print(name, json.dumps(manifest["md"][name]), file=sys.stderr)
        manifest["md_params"] = {"seed_P": SEED_P, "P": "numpy default_rng(seed_P).standard_normal(2S)",
                                 "cg": {"tol": 1e-10, "max_iter": 10000}}
        manifest["jackknife"] = make_jackknife()
        with open(path, "w") as f:
            json.dump(manifest, f, indent=1, sort_keys=True)
        return
    sizes = sorted({f"{nx}x{nt}" for _, nx, nt, _, _ in FIXTURES} |
                   {f"{nx}x{nt}" for _, nx, nt, *_ in MD_FIXTURES})
    subprocess.run(["make", "-C", os.path.join(REPO, "oracle"), "ref", "oracle",
                    "REF_SIZES=" + " ".join(sizes)], check=True)
    manifest = {"generator": "tests/golden/make_golden.py",
                "reference": "Fabian2598/SchwingerModel (unmodified src/, compiled by oracle/Makefile)",
                "layout": "two planes of interleaved complex<double>, n = x*Nt + t; force: two real planes",
                "seeds": {"U": SEED_U, "psi": SEED_PSI, "chi": SEED_CHI},
                "cg": {"tol": 1e-10, "max_iter": 10000, "rhs": "psi"},
                "fixtures": {}}
    for name, nx, nt, sigma, m0 in FIXTURES:
        exe = os.path.join(REF_DIR, f"sm_ref_{nx}x{nt}")
        with tempfile.TemporaryDirectory() as d:
            run([exe, "gen", d, str(SEED_U), repr(sigma), str(SEED_PSI), str(SEED_CHI)])
            meta = json.loads(run([exe, "fixture", d, "1", "1", repr(m0), "1e-10", "10000"]))
            arrs = {k: np.fromfile(os.path.join(d, k + ".bin"), dtype=np.float64)
                    for k in ["U", "psi", "chi"] + OUTS}
            if args.mpi and nx % 2 == 0 and nt % 2 == 0 and nx >= 4 and nt >= 4:
                for k in OUTS:
                    os.rename(os.path.join(d, k + ".bin"), os.path.join(d, k + ".1rank"))
                meta2 = json.loads(run([args.mpirun, "-n", "4", exe, "fixture", d, "2", "2",
                                        repr(m0), "1e-10", "10000"], timeout=600))
                dec = {}
                for k in OUTS:
                    a = np.fromfile(os.path.join(d, k + ".bin"), dtype=np.float64)
                    b = arrs[k]
                    dec[k] = "bitwise" if np.array_equal(a.view(np.uint64), b.view(np.uint64)) \
                        else f"max_abs={np.abs(a - b).max():.3e}"
                dec["cg_iters_2x2"] = meta2["cg_iters"]
                meta["decomposition_2x2"] = dec
        meta.update({"sigma": sigma, "file": name + ".npz"})
        np.savez_compressed(os.path.join(HERE, name + ".npz"), **arrs)
        manifest["fixtures"][name] = meta
        print(name, json.dumps(meta), file=sys.stderr)
    manifest["md"] = {}
    for name, nx, nt, sigma, m0, beta, tau, steps in MD_FIXTURES:
        manifest["md"][name] = make_md(name, nx, nt, sigma, m0, beta, tau, steps,
                                       args.mpirun if args.mpi else None)
    manifest["md_params"] = {"seed_P": SEED_P, "P": "numpy default_rng(seed_P).standard_normal(2S)",
                             "cg": {"tol": 1e-10, "max_iter": 10000}}
    manifest["jackknife"] = make_jackknife()
    manifest["conf"] = {n: make_conf(n, nx, nt, sg, rk, args.mpirun) for n, nx, nt, sg, rk in CONF_FIXTURES}
    old = os.path.join(HERE, "manifest.json")
    if os.path.exists(old):
        with open(old) as f:
            manifest["large"] = json.load(f).get("large", {})
    with open(os.path.join(HERE, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
