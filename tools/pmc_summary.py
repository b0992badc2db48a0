#!/usr/bin/env python3
"""Per-launch counter averages of one kernel from a rocprofv3 --pmc run.

    python tools/pmc_summary.py <counter_collection.csv> [--kernel cg_ra_kernel] [--sites 16777216]

Prints one JSON line: the kernel's launch count and, per counter, the mean
value per launch (and per site when --sites is given). TCC_EA0_RDREQ counts
the L2's memory-side read requests; on gfx950 a wide streaming read is
tallied as 64 B per request (MI355X_MICROARCH.md §HBM), so bytes = 2 x 64 x
RDREQ for the 128-B lines our 16-B-per-lane loads fetch.
"""
import argparse
import collections
import csv
import json


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--kernel", default="cg_ra_kernel")
    ap.add_argument("--sites", type=int, default=0)
    ap.add_argument("--label", default="")
    a = ap.parse_args()
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    with open(a.csv) as f:
        for r in csv.DictReader(f):
            if a.kernel not in r["Kernel_Name"]:
                continue
            key = (r.get("Dispatch_Id") or r.get("Correlation_Id"), r["Kernel_Name"])
            per[key][r["Counter_Name"]] += float(r["Counter_Value"])
    n = len(per)
    tot = collections.defaultdict(float)
    for d in per.values():
        for k, v in d.items():
            tot[k] += v
    out = {"label": a.label, "kernel": a.kernel, "launches": n,
           "per_launch": {k: v / n for k, v in sorted(tot.items())} if n else {}}
    if a.sites and n:
        out["per_site"] = {k: v / n / a.sites for k, v in sorted(tot.items())}
        hit, miss = tot.get("TCC_HIT_sum"), tot.get("TCC_MISS_sum")
        if hit is not None and miss is not None and hit + miss > 0:
            out["l2_hit_rate"] = hit / (hit + miss)
        if "TCC_EA0_RDREQ_sum" in tot:
            out["read_bytes_per_site"] = 128.0 * tot["TCC_EA0_RDREQ_sum"] / n / a.sites
    print(json.dumps(out))


if __name__ == "__main__":
    main()
