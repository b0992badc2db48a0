#!/usr/bin/env python3
"""Clocks and power under sustained load: the 4096^2 CG pass and the Dirac
apply, each run for a few seconds, with HIP events every --chunk launches and
`amd-smi metric` (read-only: power, clocks) sampled from a side process.
Answers whether the sustained CG pass is clock/power limited (the start of a
solve runs faster passes than its steady state, profiles/r03_q_cg_transient.jsonl).

    python tools/clock_probe.py [--seconds 3.5] [--chunk 100]
"""
import argparse
import json
import os
import subprocess
import sys
import threading
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


class Sampler(threading.Thread):
    def __init__(self):
        super().__init__(daemon=True)
        self.samples, self.stop = [], threading.Event()

    def run(self):
        while not self.stop.is_set():
            t = time.perf_counter()
            try:
                out = subprocess.run(["amd-smi", "metric", "-g", "0", "-p", "-c", "--json"], capture_output=True,
                                     text=True, timeout=20).stdout
                self.samples.append({"t": round(t, 3), "smi": json.loads(out)})
            except Exception as e:  # noqa: BLE001
                self.samples.append({"t": round(t, 3), "err": str(e)[:200]})
                time.sleep(0.5)


def compact(s):
    """power and the gfx / mem clocks out of one amd-smi JSON sample."""
    if "smi" not in s:
        return s
    d = s["smi"]
    d = d[0] if isinstance(d, list) else d
    d = d.get("gpu_data", [d])[0] if isinstance(d, dict) and "gpu_data" in d else d
    out = {"t": s["t"]}
    pw = d.get("power", {})
    for k in ("socket_power", "current_socket_power", "average_socket_power"):
        if k in pw:
            out["power"] = pw[k]
    clk = d.get("clock", {})
    for name in ("gfx_0", "mem_0", "fclk_0", "socclk_0"):
        if name in clk:
            out[name] = clk[name].get("clk", clk[name])
    if len(out) == 1:
        out["raw"] = json.dumps(d)[:1500]
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=3.5)
    ap.add_argument("--chunk", type=int, default=100)
    ap.add_argument("--shape", default="4096x4096", help="NxxNt of the lattice (config 3's field and m0)")
    ap.add_argument("--no-apply", action="store_true")
    a = ap.parse_args()
    import torch
    import bench
    rt = {"world": 1, "rank": 0, "device": 0, "transport": "rccl"}
    s = torch.cuda.Stream()
    torch.cuda.set_stream(s)
    rt["stream"] = s
    cfg = bench.CONFIGS[3]
    Nx, Nt = map(int, a.shape.split("x"))
    sh = bench.Shard(rt, Nx, Nt, cfg["sigma"])
    sm, m0 = sh.sm, cfg["m0"]
    scale = Nx * Nt / 4096 ** 2

    def run(kind, launch, per_launch_s):
        n_chunks = max(2, int(a.seconds / (per_launch_s * a.chunk)))
        smp = Sampler()
        time.sleep(1.0)
        smp.start()
        time.sleep(1.5)  # idle samples first
        t0 = time.perf_counter()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(n_chunks + 1)]
        ev[0].record(s)
        for i in range(n_chunks):
            launch(a.chunk)
            ev[i + 1].record(s)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        time.sleep(1.5)
        smp.stop.set()
        smp.join(30)
        us = [round(ev[i].elapsed_time(ev[i + 1]) * 1e3 / a.chunk, 1) for i in range(n_chunks)]
        print(json.dumps({"kind": kind, "shape": a.shape, "chunk": a.chunk, "us_per_launch": us, "load_start": round(t0, 3),
                          "load_end": round(t1, 3), "smi": [compact(x) for x in smp.samples]}), flush=True)

    def cg(n):
        sm.check(sm.lib.sm_cg_iterate(sh.L.ctx, n))

    def apply(n):
        for _ in range(n):
            sm.check(sm.lib.sm_dirac_dev(sh.L.ctx, sh.p(sh.phi), sh.p(sh.out), m0, 0))

    sm.check(sm.lib.sm_cg_link_angles(sh.L.ctx, 1, None))
    sm.check(sm.lib.sm_cg_begin(sh.L.ctx, sh.p(sh.phi), sh.p(sh.x), m0, 0.0))
    torch.cuda.synchronize()
    run("cg_pass", cg, 450e-6 * scale)
    if not a.no_apply:
        run("dirac_apply", apply, 285e-6 * scale)
    sh.close()


if __name__ == "__main__":
    main()
