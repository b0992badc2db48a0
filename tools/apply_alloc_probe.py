#!/usr/bin/env python3
"""Dirac apply at 4096^2 with the caller's input / output fields in tensors of
their own size or as the start of 2 GiB tensors (the placement effect of
schwingermodel_amd/csrc/sm_capi.cpp stream_alloc_bytes), interleaved in one
process; HIP events over --n applies on the launch stream.

    python tools/apply_alloc_probe.py [--rounds 3] [--n 100]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--n", type=int, default=100)
    a = ap.parse_args()
    import torch
    import bench
    rt = {"world": 1, "rank": 0, "device": 0, "transport": "rccl"}
    s = torch.cuda.Stream()
    torch.cuda.set_stream(s)
    rt["stream"] = s
    cfg = bench.CONFIGS[3]
    sh = bench.Shard(rt, cfg["Nx"], cfg["Nt"], cfg["sigma"])
    sm, m0, V = sh.sm, cfg["m0"], sh.V
    big_in = torch.empty((2 << 30) // 8, dtype=torch.float64, device="cuda")
    big_out = torch.empty((2 << 30) // 8, dtype=torch.float64, device="cuda")
    big_in[:4 * V].copy_(sh.phi)
    layouts = {"own_size": (sh.phi, sh.out), "in_2GiB": (big_in[:4 * V], big_out[:4 * V])}
    for r in range(a.rounds):
        for name, (fin, fout) in layouts.items():
            for _ in range(10):
                sm.check(sm.lib.sm_dirac_dev(sh.L.ctx, sh.p(fin), sh.p(fout), m0, 0))
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(a.n):
                sm.check(sm.lib.sm_dirac_dev(sh.L.ctx, sh.p(fin), sh.p(fout), m0, 0))
            e1.record(s)
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / a.n
            print(json.dumps({"round": r, "layout": name, "lib": os.environ.get("SM_LIB_PATH", "product"),
                              "apply_us": round(us, 2), "GBps": round(96 * V / us / 1e3, 1)}), flush=True)
    sh.close()


if __name__ == "__main__":
    main()
