#!/usr/bin/env python3
"""The product's placement probe over many contexts in one process.

    python tools/probe_trials.py [--n 8] [--hold 5] [--nx 4096 --nt 4096]

Creates --n contexts of the bench shape one after another, keeping the last
--hold alive (so later ones land elsewhere in physical memory), and prints
each context's sm_placement_report as one JSON line: the CG pass time of the
initial placement and after each buffer's search, and the buffers moved.
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
    ap.add_argument("--n", type=int, default=8)
    ap.add_argument("--hold", type=int, default=5)
    ap.add_argument("--nx", type=int, default=4096)
    ap.add_argument("--nt", type=int, default=4096)
    a = ap.parse_args()
    import schwingermodel_amd as sm
    names = ("x", "d1", "d0", "d2")
    held = []
    for i in range(a.n):
        L = sm.Lattice(a.nx, a.nt)
        us = (ctypes.c_double * 16)()
        n, k = ctypes.c_int(0), ctypes.c_int(0)
        sm.check(sm.lib.sm_placement_report(L.ctx, us, ctypes.byref(n), ctypes.byref(k)))
        print(json.dumps({"context": i, "us_per_pass": [round(us[j], 1) for j in range(n.value)],
                          "moved": [names[b] for b in range(4) if k.value >> b & 1],
                          "sweeps": (n.value - 1) // 4}), flush=True)
        held.append(L)
        if len(held) > a.hold:
            held.pop(0).close()
    for L in held:
        L.close()


if __name__ == "__main__":
    main()
