#!/usr/bin/env python3
"""Per-pass duration of the first CG passes at 4096^2 (HIP events around each
pass on the launch stream), after different preludes: the GPU idle for 2 s,
100 Dirac applies just before (bench.py's order), and with the link angles
off. Shows the start-of-solve transient that a short timed window (the
driver's --steps 20 --warmup 5) falls into.

    python tools/cg_transient.py [--passes 200]
"""
import argparse
import ctypes
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--passes", type=int, default=200)
    a = ap.parse_args()
    import torch
    import bench
    rt = {"world": 1, "rank": 0, "device": 0, "transport": "rccl"}
    s = torch.cuda.Stream()
    torch.cuda.set_stream(s)
    rt["stream"] = s
    cfg = bench.CONFIGS[3]
    sh = bench.Shard(rt, cfg["Nx"], cfg["Nt"], cfg["sigma"])
    sm = sh.sm
    m0 = cfg["m0"]
    for prelude in ("idle", "applies", "idle_noangles", "applies"):
        sm.check(sm.lib.sm_cg_link_angles(sh.L.ctx, 0 if prelude.endswith("noangles") else 1, None))
        sm.check(sm.lib.sm_cg_begin(sh.L.ctx, sh.p(sh.phi), sh.p(sh.x), m0, 0.0))
        torch.cuda.synchronize()
        if prelude.startswith("idle"):
            time.sleep(2.0)
        else:
            for _ in range(100):
                sm.check(sm.lib.sm_dirac_dev(sh.L.ctx, sh.p(sh.phi), sh.p(sh.out), m0, 0))
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(a.passes + 1)]
        ev[0].record(s)
        for i in range(a.passes):
            sm.check(sm.lib.sm_cg_iterate(sh.L.ctx, 1))
            ev[i + 1].record(s)
        torch.cuda.synchronize()
        us = [round(ev[i].elapsed_time(ev[i + 1]) * 1e3, 1) for i in range(a.passes)]
        print(json.dumps({"prelude": prelude, "us_per_pass": us,
                          "mean_5_25": round(sum(us[5:25]) / 20, 1),
                          "mean_last100": round(sum(us[-100:]) / 100, 1)}), flush=True)
    sh.close()


if __name__ == "__main__":
    main()
