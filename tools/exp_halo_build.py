#!/usr/bin/env python3
"""Counter-only variants of the CG pass: which streams' t-halo lines cost HBM reads.

    python tools/exp_halo_build.py            # builds tools/exp/libsm_hip_<v>.so for every variant

Each variant is the product's sm_cgra.hip with ONE textual change: the halo
lanes of a wave (the 4 + 4 lanes outside its 56 owned columns) load the named
streams from their own wave's nearest owned column instead of the neighbour
wave's, so those loads touch no line outside the owned ones. The results are
WRONG (the stencil's halo values are garbage) -- the libraries exist only to
count the pass's memory-side read requests (rocprofv3 --pmc TCC_EA0_RDREQ_sum)
under SM_LIB_PATH; they never replace the product library. Variants:
  d1   d_{j-1}        d2   d_{j-2}        uc   link codes + flag bytes
  x    x              all  all four
The other objects are the product's (build/sm_hip/, from schwingermodel_amd/build.py).
"""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from schwingermodel_amd import build as B  # noqa: E402

SRC = os.path.join(B.CSRC, "sm_cgra.hip")
OWN = "    const int c = g * RW - RH + lane;\n"
PATCHES = {
    "d1": [("rsrc<SH>(a.d1, a.f1, c, a)", "rsrc<SH>(a.d1, a.f1, co, a)")],
    "d2": [("rsrc<SH>(a.d2, a.f2, c, a)", "rsrc<SH>(a.d2, a.f2, co, a)")],
    "uc": [("return rsrc<SH>(a.Ua, a.fUa, c, a);", "return rsrc<SH>(a.Ua, a.fUa, co, a);"),
           ("            int cw = c % a.Wt;\n            if (cw < 0) cw += a.Wt;\n            SB = a.Ub + cw;",
            "            int cw = co % a.Wt;\n            if (cw < 0) cw += a.Wt;\n            SB = a.Ub + cw;")],
    "x": [("const int cx = c < 0 ? 0 : (c >= Wt ? Wt - 1 : c);", "const int cx = co < 0 ? 0 : (co >= Wt ? Wt - 1 : co);")],
}
PATCHES["all"] = PATCHES["d1"] + PATCHES["d2"] + PATCHES["uc"] + PATCHES["x"]


def main():
    B.build_library(verbose=False)
    src = open(SRC).read()
    assert OWN in src
    base = src.replace(OWN, OWN + "    const int co = min(max(c, g * RW), g * RW + RW - 1);  // exp_halo_build\n")
    outdir = os.path.join(REPO, "tools", "exp")
    os.makedirs(outdir, exist_ok=True)
    objdir = os.path.join(REPO, "build", "sm_hip")
    others = [os.path.join(objdir, s + ".o") for s in B.SOURCES if s != "sm_cgra.hip"]
    others.append(os.path.join(objdir, "sm_build_id.cpp.o"))
    for v, pats in PATCHES.items():
        s = base
        for old, new in pats:
            assert old in s, (v, old)
            s = s.replace(old, new)
        vsrc = os.path.join(REPO, "build", f"exp_sm_cgra_{v}.hip")
        with open(vsrc, "w") as f:
            f.write(s)
        obj = vsrc + ".o"
        subprocess.run([B.HIPCC] + B.CFLAGS + ["-I", B.CSRC, "-c", vsrc, "-o", obj], check=True)
        so = os.path.join(outdir, f"libsm_hip_{v}.so")
        subprocess.run([B.HIPCC, f"--offload-arch={B.ARCH}", obj] + others + ["-o", so] + B.LDFLAGS, check=True)
        print(so)


if __name__ == "__main__":
    main()
