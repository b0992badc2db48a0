#!/usr/bin/env python3
"""Small-lattice CG latency probe (the HMC config-1 regime, 32^2 .. 512^2).

    python tools/small_cg.py [--sizes 32,64,128,256] [--paths twodir,recompute,sixkernel]

Per size and CG path: a full solve through sm_cg_dev (tol 1e-10, host status
polling included: wall-clock us per iteration) and a fixed-length device
pipeline (sm_cg_iterate, HIP events: device us per iteration).
"""
import argparse
import ctypes
import json
import os
import statistics
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

PATHS = {"sixkernel": 0, "twodir": 4, "recompute": 5}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="32,64,128,256")
    ap.add_argument("--paths", default="twodir,recompute,sixkernel")
    ap.add_argument("--m0", type=float, default=0.0)
    ap.add_argument("--sigma", type=float, default=0.4242)
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    import torch
    import schwingermodel_amd as sm
    vp = ctypes.c_void_p
    for N in (int(s) for s in a.sizes.split(",")):
        L = sm.Lattice(N, N)
        V = L.V
        s = torch.cuda.Stream()
        torch.cuda.set_stream(s)
        sm.check(sm.lib.sm_set_stream(L.ctx, vp(s.cuda_stream)))
        U = torch.empty(4 * V, dtype=torch.float64)
        p = torch.empty(4 * V, dtype=torch.float64)
        Un, pn = U.numpy(), p.numpy()
        sm.lib.sm_fill_gauge(4321, a.sigma, N, 0, N, 0, N, Un.ctypes.data, Un[2 * V:].ctypes.data)
        sm.lib.sm_fill_spinor(91011, N, 0, N, 0, N, pn.ctypes.data, pn[2 * V:].ctypes.data)
        dU, dp = U.cuda(), p.cuda()
        x = torch.empty_like(dp)
        sm.check(sm.lib.sm_upload_gauge_dev(L.ctx, vp(dU.data_ptr())))
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for path in a.paths.split(","):
            if sm.lib.sm_tune_cg(L.ctx, PATHS[path], 0) != 0:
                print(json.dumps({"N": N, "path": path, "error": sm.lib.sm_last_error().decode()}))
                continue
            walls, its = [], 0
            res = sm.CGResult()
            for _ in range(a.reps):
                torch.cuda.synchronize()
                t = time.perf_counter()
                sm.check(sm.lib.sm_cg_dev(L.ctx, vp(dp.data_ptr()), vp(x.data_ptr()), a.m0, 1e-10, 10000,
                                          ctypes.byref(res)))
                walls.append(time.perf_counter() - t)
                its = res.iterations
            wall = statistics.median(walls)
            dev = None
            if path != "small":
                sm.check(sm.lib.sm_cg_begin(L.ctx, vp(dp.data_ptr()), vp(x.data_ptr()), a.m0, 0.0))
                sm.check(sm.lib.sm_cg_iterate(L.ctx, 5))
                e0.record(s)
                sm.check(sm.lib.sm_cg_iterate(L.ctx, a.iters))
                e1.record(s)
                e1.synchronize()
                dev = e0.elapsed_time(e1) * 1e3 / a.iters
            print(json.dumps({"N": N, "path": path, "iterations": its, "converged": res.converged,
                              "solve_ms": round(wall * 1e3, 3), "wall_us_per_it": round(wall * 1e6 / max(its, 1), 2),
                              "device_us_per_it": None if dev is None else round(dev, 2)}), flush=True)
        L.close()


if __name__ == "__main__":
    main()
