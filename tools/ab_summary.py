#!/usr/bin/env python3
"""Summarise an A/B run of tools/gpu_r03_ab.sh: CG it/s and ms per step of the
interleaved base / new bench.py runs, and the new build's CG-pass counter
bytes (FETCH_SIZE x 2 + WRITE_SIZE, gfx950 rule) per site.

    python tools/ab_summary.py TAG [--out profiles/....jsonl]
"""
import csv
import glob
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
G = os.path.join(REPO, "gpurun_out")


def last_json(path):
    with open(path) as f:
        for line in reversed(f.read().splitlines()):
            if line.startswith("{"):
                return json.loads(line)
    return None


def pmc(tag, counter, kernel_part="cg_ra_kernel<0, 1,"):
    f = os.path.join(G, f"abpmc_{'f' if counter == 'FETCH_SIZE' else 'w'}_{tag}", "run_counter_collection.csv")
    if not os.path.exists(f):
        return None
    vals = []
    with open(f) as fh:
        for r in csv.DictReader(fh):
            if kernel_part in r["Kernel_Name"] and r["Counter_Name"] == counter:
                vals.append(float(r["Counter_Value"]))
    return sum(vals) / len(vals) if vals else None


def main():
    tag = sys.argv[1]
    out = sys.argv[sys.argv.index("--out") + 1] if "--out" in sys.argv else None
    rows = []
    for side in ("base", "new"):
        for p in sorted(glob.glob(os.path.join(G, f"ab_{side}_*_{tag}.log"))):
            d = last_json(p)
            if d:
                rows.append({"tag": tag, "side": side, "run": os.path.basename(p), "it_per_s": d["value"],
                             "ms_per_step": d["ms_per_step"], "apply_us": d.get("dirac_apply_us")})
    for side in ("base", "new"):
        v = [r["it_per_s"] for r in rows if r["side"] == side]
        if v:
            print(f"{side}: {', '.join(f'{x:.1f}' for x in v)}  mean {sum(v) / len(v):.1f}")
    fs, ws = pmc(tag, "FETCH_SIZE"), pmc(tag, "WRITE_SIZE")
    summ = None
    if fs is not None and ws is not None:
        V = 4096 * 4096
        summ = {"tag": tag, "cg_pass_xp1_read_B_per_site": round(2 * fs * 1024 / V, 2),
                "cg_pass_xp1_write_B_per_site": round(ws * 1024 / V, 2),
                "cg_pass_xp1_B_per_site": round((2 * fs + ws) * 1024 / V, 2)}
        print(summ)
    if out:
        with open(os.path.join(REPO, out), "a") as f:
            for r in rows:
                f.write(json.dumps(r) + "\n")
            if summ:
                f.write(json.dumps(summ) + "\n")


if __name__ == "__main__":
    main()
