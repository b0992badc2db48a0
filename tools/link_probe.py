#!/usr/bin/env python3
"""Recompute-Ad CG pass with complex links (32 B/site) against one-double link
codes (16 B/site, sm_linkcode.h) per shard shape, one GPU, one shard, table
geometry: interleaved rounds, HIP events over --passes passes after --warmup
passes, a few Dirac applies right before each (no idle, no clock transient).
Decides the shard-size threshold of the code form (sm_capi.cpp link_angles).

    python tools/link_probe.py [--shapes 4096x512,4096x1024,...] [--rounds 3]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="1024x1024,2048x2048,4096x512,4096x1024,8192x1024,4096x2048,4096x4096")
    ap.add_argument("--passes", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=30)
    ap.add_argument("--rounds", type=int, default=3)
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
        res = {0: [], 1: []}
        for _ in range(a.rounds):
            for on in (0, 1):
                sm.check(sm.lib.sm_tune_cg(sh.L.ctx, 5, 0))
                sm.check(sm.lib.sm_cg_link_angles(sh.L.ctx, on, None))
                sm.check(sm.lib.sm_cg_begin(sh.L.ctx, sh.p(sh.phi), sh.p(sh.x), -0.06, 0.0))
                for _ in range(20):
                    sm.check(sm.lib.sm_dirac_dev(sh.L.ctx, sh.p(sh.phi), sh.p(sh.out), -0.06, 0))
                sm.check(sm.lib.sm_cg_iterate(sh.L.ctx, a.warmup))
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                sm.check(sm.lib.sm_cg_iterate(sh.L.ctx, a.passes))
                e1.record(s)
                torch.cuda.synchronize()
                res[on].append(round(e0.elapsed_time(e1) * 1e3 / a.passes, 2))
        print(json.dumps({"shape": shape, "us_per_pass_complex": res[0], "us_per_pass_codes": res[1]}), flush=True)
        sh.close()
        del sh
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
