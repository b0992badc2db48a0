#!/usr/bin/env python3
"""Cost of the t-shard machinery per CG pass, on ONE GPU.

For each lattice the same recompute-Ad CG runs on a plain one-shard context
and on an RCCL loopback context (sm_create_loopback: the whole lattice as
one shard driven through the multi-GPU code path -- 4-deep faces packed and
sent to itself with ncclSend/ncclRecv on the comm stream, interior / edge
launches split over two streams, the local partial sum, ncclAllReduce of the
six scalars and the scalar kernel). The difference per iteration is what a
t-shard pays on top of its own stencil work, minus the xGMI wire time.

    python tools/loopback_probe.py [--shapes 4096x512,4096x1024] [--iters 200] [--rounds 3]
Prints one JSON line per (shape, context): ms per CG iteration and us per
Dirac apply (medians over rounds).
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="4096x512,4096x1024,4096x2048,4096x4096")
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--applies", type=int, default=50)
    ap.add_argument("--m0", type=float, default=-0.06)
    ap.add_argument("--sigma", type=float, default=0.2374)
    ap.add_argument("--geom", default="", help="waves per block,rows per block of the CG pass (sm_tune_cg_geometry)")
    ap.add_argument("--contexts", default="one,loopback,peer",
                    help="one (plain shard), loopback (RCCL to itself), peer (the peer transport to itself)")
    a = ap.parse_args()
    import torch
    import schwingermodel_amd as sm
    vp = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    s = torch.cuda.Stream()
    torch.cuda.set_stream(s)
    for shape in a.shapes.split(","):
        Nx, Nt = (int(v) for v in shape.split("x"))
        V = Nx * Nt
        U = torch.empty(4 * V, dtype=torch.float64)
        chi = torch.empty(4 * V, dtype=torch.float64)
        Un, cn = U.numpy(), chi.numpy()
        sm.lib.sm_fill_gauge(4321, a.sigma, Nt, 0, Nx, 0, Nt, Un.ctypes.data, Un[2 * V:].ctypes.data)
        sm.lib.sm_fill_spinor(91011, Nt, 0, Nx, 0, Nt, cn.ctypes.data, cn[2 * V:].ctypes.data)
        dU, phi = U.cuda(), chi.cuda()
        x = torch.empty_like(phi)
        make = {"one": lambda: sm.Lattice(Nx, Nt), "loopback": lambda: sm.Lattice(Nx, Nt, loopback=True),
                "peer": lambda: sm.Lattice(Nx, Nt, loopback="peer")}
        ctxs = {k: make[k]() for k in a.contexts.split(",")}
        times = {k: [] for k in ctxs}
        host = {k: [] for k in ctxs}  # host seconds to ENQUEUE the timed iterations (host-bound if ~ the GPU time)
        for L in ctxs.values():
            sm.check(sm.lib.sm_set_stream(L.ctx, ctypes.c_void_p(s.cuda_stream)))
            sm.check(sm.lib.sm_upload_gauge_dev(L.ctx, vp(dU)))
            sm.check(sm.lib.sm_tune_cg(L.ctx, 5, 0))
            if a.geom:
                sm.check(sm.lib.sm_tune_cg_geometry(L.ctx, *(int(v) for v in a.geom.split(","))))
            sm.check(sm.lib.sm_cg_link_angles(L.ctx, -1, None))
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for _ in range(a.rounds):
            for k, L in ctxs.items():
                sm.check(sm.lib.sm_cg_begin(L.ctx, vp(phi), vp(x), a.m0, 0.0))
                sm.check(sm.lib.sm_cg_iterate(L.ctx, a.warmup))
                e0.record(s)
                th = time.perf_counter()
                sm.check(sm.lib.sm_cg_iterate(L.ctx, a.iters))
                host[k].append((time.perf_counter() - th) * 1e3 / a.iters)
                e1.record(s)
                e1.synchronize()
                times[k].append(e0.elapsed_time(e1) / a.iters)
                res = sm.CGResult()
                sm.check(sm.lib.sm_cg_finish(L.ctx, ctypes.byref(res)))
                if res.converged or res.iterations != a.warmup + a.iters - 1:
                    raise SystemExit(f"{k} {shape}: {res.iterations} iterations, converged={res.converged}")
        # the Dirac apply (1-deep spin-projected faces, interior / edge split)
        out = torch.empty_like(phi)
        ap = {k: [] for k in ctxs}
        for _ in range(a.rounds):
            for k, L in ctxs.items():
                for _ in range(3):
                    sm.check(sm.lib.sm_dirac_dev(L.ctx, vp(phi), vp(out), a.m0, 0))
                e0.record(s)
                for _ in range(a.applies):
                    sm.check(sm.lib.sm_dirac_dev(L.ctx, vp(phi), vp(out), a.m0, 0))
                e1.record(s)
                e1.synchronize()
                ap[k].append(e0.elapsed_time(e1) * 1e3 / a.applies)
        for k, L in ctxs.items():
            print(json.dumps({"shape": shape, "context": k, "geom": a.geom or "default", "ms_per_iter": round(statistics.median(times[k]), 4),
                              "min": round(min(times[k]), 4), "iters": a.iters,
                              "host_enqueue_ms_per_iter": round(statistics.median(host[k]), 4),
                              "apply_us": round(statistics.median(ap[k]), 2)}), flush=True)
            L.close()
        del dU, phi, x


if __name__ == "__main__":
    main()
