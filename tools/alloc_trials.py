#!/usr/bin/env python3
"""CG pass speed per placement of its streamed buffers, many contexts in ONE
process (round 4): is the fast / slow state a property of
the allocation rule or of where the driver happens to put the memory?

For each trial: set SM_TEST_OPTS=pad_alloc=<mode> (read at context creation,
sm_capi.cpp apply_test_opts), build bench.py's 4096^2 shard, time 200 CG
iterations after 20 warmup ones (the bench's own timing), destroy. With
--hold, every other trial keeps a 4 GiB torch allocation alive until the end,
so later contexts land on other physical memory.

    python tools/alloc_trials.py --modes 1,0,4 --rounds 3 [--hold] [--probe N]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--modes", default="1,0,4")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--hold", action="store_true")
    ap.add_argument("--probe", type=int, default=1,
                    help="place_probe for the trials (1: no placement probe, so each trial is one placement)")
    a = ap.parse_args()
    import torch
    import bench
    torch.cuda.set_device(0)
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    rt = {"world": 1, "rank": 0, "device": 0, "stream": stream, "transport": "rccl"}
    cfg = bench.CONFIGS[3]
    held = []
    k = 0
    for r in range(a.rounds):
        for m in (int(x) for x in a.modes.split(",")):
            os.environ["SM_TEST_OPTS"] = f"pad_alloc={m},place_probe={a.probe}"
            sh = bench.Shard(rt, cfg["Nx"], cfg["Nt"], cfg["sigma"])
            t, bps = bench.time_cg_steps(rt, sh, cfg["m0"], "recompute", 20, a.steps)
            sh.close()
            del sh
            print(json.dumps({"round": r, "trial": k, "pad_alloc": m, "place_probe": a.probe,
                              "it_per_s": round(a.steps / t, 1),
                              "ms_per_step": round(1e3 * t / a.steps, 4), "held_GiB": 4 * len(held)}), flush=True)
            if a.hold and k % 2 == 0:
                held.append(torch.empty(1 << 29, dtype=torch.float64, device="cuda"))
            k += 1
    os.environ.pop("SM_TEST_OPTS", None)


if __name__ == "__main__":
    main()
