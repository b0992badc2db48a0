#!/usr/bin/env python3
"""Recompute-Ad CG pass time per site across lattice shapes (one GPU, one
shard): does the pass stream more efficiently on long rows (Nt) or on large
lattices? Each shape runs with its table geometry and with a common one
(4 waves x 32 rows), HIP events over --passes passes after --warmup passes,
back to back (no idle between shapes, so no start-of-solve clock transient).

    python tools/shape_probe.py [--shapes 4096x4096,4096x8192,8192x4096,8192x8192] [--passes 200]
"""
import argparse
import ctypes
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="4096x4096,4096x8192,8192x4096,8192x8192,4096x4096")
    ap.add_argument("--passes", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=30)
    a = ap.parse_args()
    import torch
    import bench
    rt = {"world": 1, "rank": 0, "device": 0, "transport": "rccl"}
    s = torch.cuda.Stream()
    torch.cuda.set_stream(s)
    rt["stream"] = s
    for shape in a.shapes.split(","):
        Nx, Nt = map(int, shape.split("x"))
        sh = bench.Shard(rt, Nx, Nt, 0.2374)
        sm = sh.sm
        for geo in ("table", "4x32"):
            sm.check(sm.lib.sm_tune_cg(sh.L.ctx, 5, 0))
            if geo != "table":
                sm.check(sm.lib.sm_tune_cg_geometry(sh.L.ctx, 4, 32))
            sm.check(sm.lib.sm_cg_link_angles(sh.L.ctx, 1, None))
            sm.check(sm.lib.sm_cg_begin(sh.L.ctx, sh.p(sh.phi), sh.p(sh.x), -0.06, 0.0))
            for _ in range(20):  # keep the chip busy right before the passes
                sm.check(sm.lib.sm_dirac_dev(sh.L.ctx, sh.p(sh.phi), sh.p(sh.out), -0.06, 0))
            sm.check(sm.lib.sm_cg_iterate(sh.L.ctx, a.warmup))
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            sm.check(sm.lib.sm_cg_iterate(sh.L.ctx, a.passes))
            e1.record(s)
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / a.passes
            V = Nx * Nt
            print(json.dumps({"shape": shape, "geometry": geo, "us_per_pass": round(us, 2),
                              "ps_per_site": round(us * 1e6 / V, 2),
                              "alg_TBps": round(144 * V / (us * 1e-6) / 1e12, 3)}), flush=True)
        sh.close()
        del sh
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
