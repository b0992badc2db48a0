#!/usr/bin/env python3
"""Timeline of the last few CG passes from a rocprofv3 kernel trace.

    python tools/trace_pass.py gpurun_out/lbtrace/run_kernel_trace.csv [--last 24]

Prints each kernel's start (us, relative to the first one shown), duration,
end and queue, so the critical path of a sharded pass (edge launch, face
exchange, interior launch, scalar step) can be read off directly.
"""
import argparse
import csv


def short(name):
    n = name.split("(")[0]
    return n.replace("void ", "").replace("sm::", "")[:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--last", type=int, default=24)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r.get("Queue_Id", "?"))
                 for r in rows))
    ks = ks[-a.last:]
    t0 = ks[0][0]
    for s, e, n, q in ks:
        print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f} {(e - t0) / 1e3:9.1f}  q{q:>3}  {short(n)}")


if __name__ == "__main__":
    main()
