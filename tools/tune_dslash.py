#!/usr/bin/env python3
"""A/B sweep of the dslash launch geometry in ONE process, interleaved rounds
(cdna_hip_programming.md §5.4 rule 24), plus a device-copy ceiling.

    python tools/tune_dslash.py [--n 4096] [--rounds 5] [--applies 20]
Prints one JSON line per config: median / min microseconds and algorithmic GB/s.
"""
import argparse
import ctypes
import itertools
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=4096)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--applies", type=int, default=20)
    ap.add_argument("--bt", default="64,128,256")
    ap.add_argument("--xchunk", default="16,32,64,128")
    ap.add_argument("--remap", default="0,1")
    ap.add_argument("--variant", default="0,1,2")
    ap.add_argument("--dagger", type=int, default=0)
    a = ap.parse_args()
    import torch
    import schwingermodel_amd as sm
    N = a.n
    L = sm.Lattice(N, N)
    V = L.V
    s = torch.cuda.Stream()
    torch.cuda.set_stream(s)
    sm.check(sm.lib.sm_set_stream(L.ctx, ctypes.c_void_p(s.cuda_stream)))
    U = torch.empty(4 * V, dtype=torch.float64)
    p = torch.empty(4 * V, dtype=torch.float64)
    Un, pn = U.numpy(), p.numpy()
    sm.lib.sm_fill_gauge(4321, 0.2374, N, 0, N, 0, N, Un.ctypes.data, Un[2 * V:].ctypes.data)
    sm.lib.sm_fill_spinor(91011, N, 0, N, 0, N, pn.ctypes.data, pn[2 * V:].ctypes.data)
    dU, dp = U.cuda(), p.cuda()
    out = torch.empty_like(dp)
    sm.check(sm.lib.sm_upload_gauge_dev(L.ctx, ctypes.c_void_p(dU.data_ptr())))
    vp = ctypes.c_void_p
    configs = list(itertools.product([int(x) for x in a.bt.split(",")],
                                     [int(x) for x in a.xchunk.split(",")],
                                     [int(x) for x in a.remap.split(",")],
                                     [int(x) for x in a.variant.split(",")]))
    res = {c: [] for c in configs}
    copy_t = []
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for r in range(a.rounds):
        for c in configs:
            sm.check(sm.lib.sm_tune(L.ctx, c[0], c[1], c[2], c[3]))
            for _ in range(3):
                sm.check(sm.lib.sm_dirac_dev(L.ctx, vp(dp.data_ptr()), vp(out.data_ptr()), -0.06, a.dagger))
            ev0.record(s)
            for _ in range(a.applies):
                sm.check(sm.lib.sm_dirac_dev(L.ctx, vp(dp.data_ptr()), vp(out.data_ptr()), -0.06, a.dagger))
            ev1.record(s)
            ev1.synchronize()
            res[c].append(ev0.elapsed_time(ev1) * 1e3 / a.applies)
        # streaming ceilings: out = psi + U over 2V complex (96 B/site, the
        # dslash byte mix), out = psi (64 B/site), torch copy_ (64 B/site)
        for key, fn in (("stream2r1w", lambda: sm.lib.sm_bench_stream(L.ctx, 1, 2 * V, vp(dp.data_ptr()), vp(dU.data_ptr()), vp(out.data_ptr()), 0)),
                        ("stream1r1w", lambda: sm.lib.sm_bench_stream(L.ctx, 0, 2 * V, vp(dp.data_ptr()), None, vp(out.data_ptr()), 0)),
                        ("torch_copy", lambda: out.copy_(dp))):
            fn()
            ev0.record(s)
            for _ in range(a.applies):
                fn()
            ev1.record(s)
            ev1.synchronize()
            copy_t.append((key, ev0.elapsed_time(ev1) * 1e3 / a.applies))
    for c in configs:
        med = statistics.median(res[c])
        print(json.dumps({"bt": c[0], "xchunk": c[1], "remap": c[2], "variant": c[3], "median_us": round(med, 2),
                          "min_us": round(min(res[c]), 2), "GBps": round(96 * V / med / 1e3, 1)}))
    for key, bps in (("stream2r1w", 96), ("stream1r1w", 64), ("torch_copy", 64)):
        cm = statistics.median([t for k, t in copy_t if k == key])
        print(json.dumps({key + "_median_us": round(cm, 2), "GBps": round(bps * V / cm / 1e3, 1)}))


if __name__ == "__main__":
    main()
