#!/usr/bin/env python3
"""CPU restatement (oracle/) vs the unmodified reference (oracle/_ref), one core each.

    python tools/cpu_ratio.py [--n 1024] [--cg 5]

Both run the same workload on the same host: D applies and CG iterations at
n x n (beta = 3 field, m0 = -0.1). The reference is run
as one MPI rank (its bench mode in oracle/ref_harness.cpp). Test/measurement
infrastructure only: prints one JSON line (SURVEY.md §8d "CPU reference timing":
state the restatement's ratio to the reference).
"""
import argparse
import ctypes
import json
import os
import subprocess
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1024)
    ap.add_argument("--cg", type=int, default=5)
    ap.add_argument("--applies", type=int, default=3)
    a = ap.parse_args()
    N, S = a.n, a.n * a.n
    seed_u, sigma, seed_chi, m0 = 4321, 0.3246, 91011, -0.1
    exe = os.path.join(REPO, "oracle", "_ref", f"sm_ref_{N}x{N}")
    env = dict(os.environ, HOSTNAME=os.environ.get("HOSTNAME", "localhost"))
    out = subprocess.run(["/opt/conda/bin/mpirun", "-n", "1", exe, "bench", "1", "1", str(seed_u), repr(sigma),
                          str(seed_chi), repr(m0), str(a.applies), str(a.cg)],
                         capture_output=True, text=True, timeout=600, env=env, check=True)
    ref = json.loads(out.stdout.strip().splitlines()[-1])

    import schwingermodel_amd as sm  # host-side field generators only (no GPU)
    o = ctypes.CDLL(os.path.join(REPO, "oracle", "liboracle.so"))
    vp, ci, cd = ctypes.c_void_p, ctypes.c_int, ctypes.c_double
    o.oracle_dirac.argtypes = [ci, ci, vp, vp, vp, vp, vp, vp, cd, ci]
    o.oracle_cg.argtypes = [ci, ci, vp, vp, vp, vp, vp, vp, cd, cd, ci, ctypes.POINTER(ci), ctypes.POINTER(cd)]
    U0, U1, p0, p1, y0, y1 = (np.empty(2 * S) for _ in range(6))
    sm.lib.sm_fill_gauge(seed_u, sigma, N, 0, N, 0, N, U0.ctypes.data, U1.ctypes.data)
    sm.lib.sm_fill_spinor(seed_chi, N, 0, N, 0, N, p0.ctypes.data, p1.ctypes.data)
    ptr = [v.ctypes.data for v in (U0, U1, p0, p1, y0, y1)]
    t = time.perf_counter()
    for _ in range(a.applies):
        o.oracle_dirac(N, N, *ptr, m0, 0)
    apply_s = (time.perf_counter() - t) / a.applies
    it, err = ctypes.c_int(), ctypes.c_double()
    t = time.perf_counter()
    o.oracle_cg(N, N, *ptr, m0, 0.0, a.cg, ctypes.byref(it), ctypes.byref(err))
    cg_s = time.perf_counter() - t
    port = {"apply_s": apply_s, "cg_it_per_s": it.value / cg_s}
    print(json.dumps({"N": N, "cores": 1, "reference": {"apply_s": ref["apply_s"], "cg_it_per_s": ref["cg_it_per_s"]},
                      "port": {k: round(v, 6) for k, v in port.items()},
                      "port_over_reference": {"apply": round(ref["apply_s"] / apply_s, 3),
                                              "cg": round(port["cg_it_per_s"] / ref["cg_it_per_s"], 3)}}))


if __name__ == "__main__":
    main()
