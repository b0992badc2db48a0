#!/usr/bin/env python3
"""Turn rocprofv3 outputs (gpurun_out/prof_*) into the judged summaries under profiles/.

    python tools/summarize_prof.py --round r01 [--out-dir gpurun_out] [--nx 4096 --nt 4096]

Reads
  <out>/prof_stats/run_kernel_stats.csv        (rocprofv3 --kernel-trace --stats)
  <out>/prof_fetch/run_counter_collection.csv  (rocprofv3 --pmc FETCH_SIZE)
  <out>/prof_write/run_counter_collection.csv  (rocprofv3 --pmc WRITE_SIZE)
and writes
  profiles/<round>_kernel_stats.csv   (verbatim copy of the stats summary)
  profiles/<round>_dslash_pmc.json    (per-launch HBM bytes of every kernel)

HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE are in
KiB; on gfx950 FETCH_SIZE reports exactly half of a wide (16 B/lane)
coalesced stream, so reads = 2 x FETCH_SIZE (our copy kernel is the
calibration: it reports 1/2 of its known byte count), writes = WRITE_SIZE.
"""
import argparse
import collections
import csv
import json
import os
import shutil

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def per_kernel(path, counter):
    agg = collections.defaultdict(list)
    with open(path) as f:
        for r in csv.DictReader(f):
            if r["Counter_Name"] == counter:
                agg[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in agg.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--round", required=True)
    ap.add_argument("--out-dir", default=os.path.join(REPO, "gpurun_out"))
    ap.add_argument("--nx", type=int, default=4096)
    ap.add_argument("--nt", type=int, default=4096)
    ap.add_argument("--tag", default="")
    ap.add_argument("--suffix", default="", help="input dirs prof_stats<suffix> etc. (tools/gpu_round.sh writes _<tag>)")
    ap.add_argument("--build-id", default=None,
                    help="sm_build_id() of the profiled library (default: the in-tree libsm_hip.so, which is the "
                         "one gpurun shipped as long as nothing was rebuilt since)")
    a = ap.parse_args()
    if a.build_id is None:
        import ctypes
        lib = ctypes.CDLL(os.path.join(REPO, "schwingermodel_amd", "libsm_hip.so"))
        lib.sm_build_id.restype = ctypes.c_char_p
        a.build_id = lib.sm_build_id().decode()
    pdir = os.path.join(REPO, "profiles")
    os.makedirs(pdir, exist_ok=True)
    tag = f"{a.round}{a.tag}"
    stats = os.path.join(a.out_dir, "prof_stats" + a.suffix, "run_kernel_stats.csv")
    if os.path.exists(stats):
        shutil.copy(stats, os.path.join(pdir, f"{tag}_kernel_stats.csv"))
    fetch = per_kernel(os.path.join(a.out_dir, "prof_fetch" + a.suffix, "run_counter_collection.csv"), "FETCH_SIZE")
    write = per_kernel(os.path.join(a.out_dir, "prof_write" + a.suffix, "run_counter_collection.csv"), "WRITE_SIZE")
    avg_ns = {}
    if os.path.exists(stats):
        with open(stats) as f:
            for r in csv.DictReader(f):
                avg_ns[r["Name"]] = float(r["AverageNs"])
    sites = a.nx * a.nt
    kernels = {}
    for k in sorted(set(fetch) | set(write)):
        rd = 2 * 1024 * fetch.get(k, 0.0)
        wr = 1024 * write.get(k, 0.0)
        e = {"read_bytes": rd, "write_bytes": wr, "hbm_bytes": rd + wr,
             "bytes_per_site": (rd + wr) / sites}
        if k in avg_ns:
            e["avg_ns"] = avg_ns[k]
            e["hbm_GBps"] = (rd + wr) / avg_ns[k]
        kernels[k] = e
    dslash = [k for k in kernels if "dslash_kernel" in k and "<0, 0>" in k]
    # the CG pass behind bench.py's value: one shard, x rows, fused multiply-
    # adds, in-kernel scalars off, link angles, ticketed tail (sm_cgra.hip)
    # (link codes: UC 2 packed flag bytes, 145 B/site; UC 1 flag words, 148; any march-schedule suffix)
    cg_bytes = {2: 145, 1: 148}
    cgk, cg_uc = [], None
    for uc in (2, 1):
        cgk = [k for k in kernels if f"cg_ra_kernel<0, 1, 2, 0, {uc}, 1" in k]
        if cgk:
            cg_uc = uc
            break
    out = {"Nx": a.nx, "Nt": a.nt, "build_id": a.build_id,
           "source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, separate passes",
           "correction": "reads = 2 x FETCH_SIZE KiB (gfx950), writes = WRITE_SIZE KiB",
           "algorithmic_bytes_per_launch": 96 * sites,
           "dslash_kernel": dslash[0] if dslash else None,
           "hbm_bytes_per_launch": kernels[dslash[0]]["hbm_bytes"] if dslash else None,
           "cg_pass_kernel": cgk[0] if cgk else None,
           "cg_pass_algorithmic_bytes_per_launch": cg_bytes[cg_uc] * sites if cgk else None,
           "cg_pass_hbm_bytes_per_launch": kernels[cgk[0]]["hbm_bytes"] if cgk else None,
           "kernels": kernels}
    with open(os.path.join(pdir, f"{tag}_dslash_pmc.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps({k: round(v["bytes_per_site"], 2) for k, v in kernels.items()}, indent=1))


if __name__ == "__main__":
    main()
