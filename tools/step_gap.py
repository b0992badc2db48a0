#!/usr/bin/env python3
"""Where a CG step's time goes: kernel durations against the gaps between them.

    python tools/step_gap.py gpurun_out/<dir>/run_kernel_trace.csv [--kernel cg_ra_kernel] [--last 200]

Takes the last N launches of the named kernel (the timed CG passes of a
bench.py run) and prints, over the span from the first one's start to the last
one's end: the summed kernel time, the summed idle gaps between consecutive
launches of ANY kernel on the device, and the other kernels in that span. The
span per pass is the rocprof-side counterpart of bench.py's ms_per_step.
"""
import argparse
import csv
import json
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--kernel", default="cg_ra_kernel")
    ap.add_argument("--last", type=int, default=200)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
    sel = [i for i, k in enumerate(ks) if a.kernel in k[2]][-a.last:]
    if not sel:
        raise SystemExit(f"no {a.kernel} launches in {a.trace}")
    lo, hi = sel[0], sel[-1]
    span = ks[hi][1] - ks[lo][0]
    durs = [ks[i][1] - ks[i][0] for i in sel]
    others = {}
    gaps = []
    for i in range(lo, hi + 1):
        if i > lo:
            gaps.append(max(0, ks[i][0] - ks[i - 1][1]))
        if a.kernel not in ks[i][2]:
            n = ks[i][2].split("(")[0][:60]
            others[n] = others.get(n, 0) + ks[i][1] - ks[i][0]
    n = len(sel)
    out = {
        "kernel": a.kernel, "passes": n,
        "span_us_per_pass": round(span / n / 1e3, 2),
        "kernel_us_per_pass": round(sum(durs) / n / 1e3, 2),
        "kernel_us_median": round(statistics.median(durs) / 1e3, 2),
        "gap_us_per_pass": round(sum(gaps) / n / 1e3, 2),
        "gap_us_median": round(statistics.median(gaps) / 1e3, 2) if gaps else 0,
        "gap_us_max": round(max(gaps) / 1e3, 2) if gaps else 0,
        "other_kernels_us_per_pass": {k: round(v / n / 1e3, 2) for k, v in others.items()},
    }
    print(json.dumps(out))


if __name__ == "__main__":
    main()
