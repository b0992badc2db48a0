#!/usr/bin/env python3
"""A/B of CG-iteration configurations in ONE process (interleaved rounds).

    python tools/tune_cg.py [--n 4096] [--xchunk 16,32,64] [--iters 20] [--rounds 3]
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
    ap.add_argument("--n", type=int, default=4096)
    ap.add_argument("--xchunk", default="16,32,64,128")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--sixkernel", action="store_true")
    ap.add_argument("--paths", default="recompute", help="comma list of twodir (stored Ad), recompute, sixkernel")
    a = ap.parse_args()
    import torch
    import schwingermodel_amd as sm
    N = a.n
    L = sm.Lattice(N, N)
    V = L.V
    s = torch.cuda.Stream()
    torch.cuda.set_stream(s)
    vp = ctypes.c_void_p
    sm.check(sm.lib.sm_set_stream(L.ctx, vp(s.cuda_stream)))
    U = torch.empty(4 * V, dtype=torch.float64)
    p = torch.empty(4 * V, dtype=torch.float64)
    Un, pn = U.numpy(), p.numpy()
    sm.lib.sm_fill_gauge(4321, 0.2374, N, 0, N, 0, N, Un.ctypes.data, Un[2 * V:].ctypes.data)
    sm.lib.sm_fill_spinor(91011, N, 0, N, 0, N, pn.ctypes.data, pn[2 * V:].ctypes.data)
    dU, dp = U.cuda(), p.cuda()
    x = torch.empty_like(dp)
    sm.check(sm.lib.sm_upload_gauge_dev(L.ctx, vp(dU.data_ptr())))
    configs = [(p, int(c)) for p in a.paths.split(",") for c in a.xchunk.split(",")]
    if a.sixkernel:
        configs.append(("sixkernel", 0))
    res = {c: [] for c in configs}
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(a.rounds):
        for c in configs:
            sm.check(sm.lib.sm_tune_cg(L.ctx, {"twodir": 4, "recompute": 5, "sixkernel": 0}[c[0]], c[1]))
            sm.check(sm.lib.sm_cg_begin(L.ctx, vp(dp.data_ptr()), vp(x.data_ptr()), -0.06, 0.0))
            sm.check(sm.lib.sm_cg_iterate(L.ctx, 3))
            e0.record(s)
            sm.check(sm.lib.sm_cg_iterate(L.ctx, a.iters))
            e1.record(s)
            e1.synchronize()
            res[c].append(e0.elapsed_time(e1) / a.iters)
    for c in configs:
        med = statistics.median(res[c])
        print(json.dumps({"path": c[0], "xchunk": c[1], "ms_per_it": round(med, 4), "it_per_s": round(1e3 / med, 1)}))


if __name__ == "__main__":
    main()
