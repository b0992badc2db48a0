#!/usr/bin/env python3
"""Real-loop A/B of recompute-Ad CG launch geometries at the BASELINE shard shapes.

One shard of Nx x Nt on one GPU; for each candidate (waves per block, rows per
block, link angles) the library's own CG loop (sm_cg_begin / sm_cg_iterate, the
scalar kernel or redundant scalars included) is timed with events on the ctx
stream; candidates are interleaved over rounds and the median is printed.

    python tools/tune_shapes.py 4096x512:1,48,0 4096x512:4,32,0 4096x4096:4,64,1,1,0 ...
(optional 4th / 5th values: t-strip blocks and balanced x-chunks, sm_tune_cg_strip)
"""
import argparse
import ctypes
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("cands", nargs="+", help="NxxNt:wpb,xchunk,angles[,strip[,balanced]] (wpb/xchunk 0 = the default)")
    ap.add_argument("--iters", type=int, default=40)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    import torch
    import schwingermodel_amd as sm
    vp = ctypes.c_void_p
    shapes = {}
    for c in a.cands:
        shp, cfg = c.split(":")
        shapes.setdefault(shp, []).append(tuple(int(v) for v in cfg.split(",")))
    for shp, cands in shapes.items():
        Nx, Nt = (int(v) for v in shp.split("x"))
        L = sm.Lattice(Nx, Nt)
        V = L.V
        s = torch.cuda.Stream()
        torch.cuda.set_stream(s)
        sm.check(sm.lib.sm_set_stream(L.ctx, vp(s.cuda_stream)))
        U = torch.empty(4 * V, dtype=torch.float64)
        p = torch.empty(4 * V, dtype=torch.float64)
        Un, pn = U.numpy(), p.numpy()
        sm.lib.sm_fill_gauge(4321, 0.2374, Nt, 0, Nx, 0, Nt, Un.ctypes.data, Un[2 * V:].ctypes.data)
        sm.lib.sm_fill_spinor(91011, Nt, 0, Nx, 0, Nt, pn.ctypes.data, pn[2 * V:].ctypes.data)
        dU, dp = U.cuda(), p.cuda()
        x = torch.empty_like(dp)
        sm.check(sm.lib.sm_upload_gauge_dev(L.ctx, vp(dU.data_ptr())))
        sm.check(sm.lib.sm_tune_cg(L.ctx, 5, 0))
        res = {c: [] for c in cands}
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for _ in range(a.rounds):
            for c in cands:
                wpb, xc, ang = c[:3]
                strip, bal = (tuple(c[3:]) + (0, 0))[:2]
                L2 = L
                sm.check(sm.lib.sm_tune_cg_strip(L2.ctx, strip, bal))
                if wpb or xc:
                    sm.check(sm.lib.sm_tune_cg_geometry(L2.ctx, wpb, xc))
                sm.check(sm.lib.sm_cg_link_angles(L2.ctx, ang, None))
                sm.check(sm.lib.sm_cg_begin(L2.ctx, vp(dp.data_ptr()), vp(x.data_ptr()), -0.06, 0.0))
                sm.check(sm.lib.sm_cg_iterate(L2.ctx, 4))
                e0.record(s)
                sm.check(sm.lib.sm_cg_iterate(L2.ctx, a.iters))
                e1.record(s)
                e1.synchronize()
                res[c].append(e0.elapsed_time(e1) / a.iters)
        for c in cands:
            med = statistics.median(res[c])
            print(json.dumps({"shape": shp, "wpb": c[0], "xchunk": c[1], "angles": c[2],
                              "strip": c[3] if len(c) > 3 else 0, "balanced": c[4] if len(c) > 4 else 0,
                              "ms_per_it": round(med, 5),
                              "ps_per_site": round(med * 1e9 / V, 3), "all": [round(v, 5) for v in res[c]]}),
                  flush=True)
        L.close()
        del dU, dp, x


if __name__ == "__main__":
    main()
