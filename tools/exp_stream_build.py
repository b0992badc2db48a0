#!/usr/bin/env python3
"""Counter-only variants of the CG pass: where its reads above the algorithmic bytes go, per stream.

    python tools/exp_stream_build.py            # builds tools/exp/libsm_hip_s_<v>.so for every variant

Each variant is the product's sm_cgra.hip with ONE stream's row loads pinned
to the tile's first row (x0), so that stream costs one row per tile instead
of a row per march step: the pass's memory-side reads (rocprofv3 --pmc
TCC_EA0_RDREQ_sum) then drop by that stream's algorithmic bytes plus whatever
it read above them. The results are WRONG -- the libraries exist only to
count read requests under SM_LIB_PATH; they never replace the product
library. Variants (reads per site of the product, packed codes):
  d1   d_{j-1}  (32 B + its x-halo rows)      d2   d_{j-2}  (32 B)
  u    link codes + flag bytes (17 B)         x    x (16 B: half the rows per pass)
and the x-halo variants d1h, d2h, uh, allh: only the rows a tile reads beyond
its own chunk (4 + 4 of d_{j-1}, 2 + 2 of d_{j-2}, 4 + 3 of the links) clamped
to its edge rows, which it reads anyway.
The other objects are the product's (build/sm_hip/, from schwingermodel_amd/build.py).
"""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from schwingermodel_amd import build as B  # noqa: E402

SRC = os.path.join(B.CSRC, "sm_cgra.hip")
D1 = "const double2 *p = S1.p + (long)wrap(phys(min(xr, xe + 3))) * S1.xs;"
D2 = "const double2 *p = S2.p + (long)wrap(phys(min(max(xr, x0 - 2), xe + 1))) * S2.xs;"
UX = "const int X = phys(min(xr, xe + 2));"
# the x-halo variants: only the rows outside the tile's own [x0, xe) clamped to its edge rows (read anyway)
D1H = (D1, "const double2 *p = S1.p + (long)wrap(phys(min(max(xr, x0), xe - 1))) * S1.xs;  // exp_stream_build")
D2H = (D2, "const double2 *p = S2.p + (long)wrap(phys(min(max(xr, x0), xe - 1))) * S2.xs;  // exp_stream_build")
UH = (UX, "const int X = phys(min(max(xr, x0 + 1), xe - 1));  // exp_stream_build")
PATCHES = {
    "d1": [("const double2 *p = S1.p + (long)wrap(phys(min(xr, xe + 3))) * S1.xs;",
            "const double2 *p = S1.p + (long)x0 * S1.xs;  // exp_stream_build")],
    "d2": [("const double2 *p = S2.p + (long)wrap(phys(min(max(xr, x0 - 2), xe + 1))) * S2.xs;",
            "const double2 *p = S2.p + (long)x0 * S2.xs;  // exp_stream_build")],
    "u": [("const int X = phys(min(xr, xe + 2));", "const int X = x0 + 0 * xr;  // exp_stream_build")],
    "x": [("const long n = (long)wrap(phys(min(max(xr, x0), xe - 1))) * Wt + cx;",
           "const long n = (long)x0 * Wt + cx;  // exp_stream_build")],
    "d1h": [D1H], "d2h": [D2H], "uh": [UH], "allh": [D1H, D2H, UH],
}


def main():
    B.build_library(verbose=False)
    src = open(SRC).read()
    outdir = os.path.join(REPO, "tools", "exp")
    os.makedirs(outdir, exist_ok=True)
    objdir = os.path.join(REPO, "build", "sm_hip")
    others = [os.path.join(objdir, s + ".o") for s in B.SOURCES if s != "sm_cgra.hip"]
    others.append(os.path.join(objdir, "sm_build_id.cpp.o"))
    for v, pats in PATCHES.items():
        s = src
        for old, new in pats:
            assert s.count(old) == 1, (v, old)
            s = s.replace(old, new)
        vsrc = os.path.join(REPO, "build", f"exp_sm_cgra_s_{v}.hip")
        with open(vsrc, "w") as f:
            f.write(s)
        obj = vsrc + ".o"
        subprocess.run([B.HIPCC] + B.CFLAGS + ["-I", B.CSRC, "-c", vsrc, "-o", obj], check=True)
        so = os.path.join(outdir, f"libsm_hip_s_{v}.so")
        subprocess.run([B.HIPCC, f"--offload-arch={B.ARCH}", obj] + others + ["-o", so] + B.LDFLAGS, check=True)
        print(so)


if __name__ == "__main__":
    main()
