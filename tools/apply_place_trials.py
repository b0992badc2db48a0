#!/usr/bin/env python3
"""Is the Dirac apply placement-sensitive like the CG pass (round 4)?

One 4096^2 context (U generated on the device), then K candidate (in, out)
field pairs, each field in its own allocation (plain own-size, or >= 2 GiB
with the contiguous flag: --mode), all held at once. Interleaved rounds time
N applies on each pair (device synchronise around them, wall clock); the
first round is discarded. Prints the median us per apply of each pair.

    python tools/apply_place_trials.py --pairs 8 --mode contig2g
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
    ap.add_argument("--pairs", type=int, default=8)
    ap.add_argument("--applies", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--mode", choices=["own", "contig2g"], default="contig2g")
    a = ap.parse_args()
    import schwingermodel_amd as sm
    rt = ctypes.CDLL("libamdhip64.so.7")
    rt.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
    rt.hipExtMallocWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
    rt.hipMemset.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t]
    rt.hipDeviceSynchronize.argtypes = []
    N = 4096
    fb = 32 * N * N
    L = sm.Lattice(N, N)
    sm.check(sm.lib.sm_fill_gauge_dev(L.ctx, 4321, 0.2374))
    pairs = []
    for k in range(a.pairs):
        pr = []
        for _ in range(2):
            p = ctypes.c_void_p()
            if a.mode == "own":
                assert rt.hipMalloc(ctypes.byref(p), fb) == 0
            else:
                assert rt.hipExtMallocWithFlags(ctypes.byref(p), 2 << 30, 4) == 0  # hipDeviceMallocContiguous
            assert rt.hipMemset(p, 0, fb) == 0
            pr.append(p)
        pairs.append(pr)
    t = [[] for _ in pairs]
    for r in range(a.rounds):
        for k, (pin, pout) in enumerate(pairs):
            assert rt.hipDeviceSynchronize() == 0
            t0 = time.perf_counter()
            for _ in range(a.applies):
                sm.check(sm.lib.sm_dirac_dev(L.ctx, pin, pout, -0.06, 0))
            sm.check(sm.lib.sm_synchronize(L.ctx))
            if r:
                t[k].append((time.perf_counter() - t0) / a.applies * 1e6)
    us = [round(statistics.median(x), 1) for x in t]
    print(json.dumps({"mode": a.mode, "pairs": a.pairs, "us_per_apply": us, "min": min(us), "max": max(us)}))
    L.close()


if __name__ == "__main__":
    main()
