"""The link-angle CG pass rebuilds U = (cos theta, sin theta) with
schwingermodel_amd/csrc/sm_sincos.h. The header is plain C as well: compiled
here for the host (gcc, explicit fmas, no contraction), it must stay within
1 ulp of glibc's sin / cos over [-pi, pi], including the quadrant boundaries."""
import os
import subprocess

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

DRIVER = r"""
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include "sm_sincos.h"
static double ulps(double a, double b) {
    if (a == b) return 0.0;
    const double u = nextafter(fabs(b), INFINITY) - fabs(b);
    return fabs(a - b) / u;
}
int main(void) {
    double ms = 0.0, mc = 0.0;
    const double special[] = {M_PI, -M_PI, 0.0, -0.0, M_PI / 2, -M_PI / 2, M_PI / 4, -M_PI / 4,
                              3 * M_PI / 4, -3 * M_PI / 4, 1e-300, -1e-20};
    const long n = 2000000;
    srand48(7);
    for (long i = 0; i < n; ++i) {
        double th = i < 12 ? special[i] : (drand48() * 2.0 - 1.0) * M_PI;
        if (i >= 12 && i < 1000) th = nextafter(((i % 5) - 2) * M_PI_2, (i & 1) ? INFINITY : -INFINITY);
        double c, s;
        sm_cos_sin_pi(th, &c, &s);
        const double es = ulps(s, sin(th)), ec = ulps(c, cos(th));
        if (es > ms) ms = es;
        if (ec > mc) mc = ec;
    }
    printf("%.6f %.6f\n", ms, mc);
    return 0;
}
"""


def test_link_sincos_within_one_ulp(tmp_path):
    src = tmp_path / "drv.c"
    src.write_text(DRIVER)
    exe = tmp_path / "drv"
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-I", os.path.join(REPO, "schwingermodel_amd", "csrc"),
                    str(src), "-o", str(exe), "-lm"], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split()
    ms, mc = float(out[0]), float(out[1])
    assert ms <= 1.0 and mc <= 1.0, (ms, mc)
