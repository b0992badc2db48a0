"""The compact-link CG pass stores each U(1) link as one double and rebuilds it
with schwingermodel_amd/csrc/sm_linkcode.h. The header is plain C as well:
compiled here for the host (gcc, explicit fma, no contraction) it runs the
device's arithmetic (sqrt and fma are correctly rounded on both). Over unit
links of every quadrant, the axes and the diagonal ties, the rebuilt link is
within 3 ulp per component of the stored one and within 3.5e-16 absolute."""
import os
import subprocess

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

DRIVER = r"""
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include "sm_linkcode.h"
static double ulps(double a, double b) {
    if (a == b) return 0.0;
    const double u = nextafter(fabs(b), INFINITY) - fabs(b);
    return fabs(a - b) / u;
}
int main(void) {
    double mu = 0.0, ma = 0.0;
    long bad_sign = 0;
    const double special[] = {0.0, -0.0, M_PI, -M_PI, M_PI / 2, -M_PI / 2, M_PI / 4, -M_PI / 4,
                              3 * M_PI / 4, -3 * M_PI / 4, 1e-300, -1e-20};
    const long n = 4000000;
    srand48(11);
    for (long i = 0; i < n; ++i) {
        double th = i < 12 ? special[i] : (drand48() * 2.0 - 1.0) * M_PI;
        if (i >= 12 && i < 4000) th = nextafter(((i % 9) - 4) * M_PI_4, (i & 1) ? INFINITY : -INFINITY);
        const double c = cos(th), s = sin(th);
        double c2, s2;
        sm_link_decode(sm_link_encode(c, s), &c2, &s2);
        /* ulps against the larger of the component and 2^-53 (a link's scale is 1) */
        const double uc = fabs(c) > 0x1p-2 ? ulps(c2, c) : fabs(c2 - c) / 0x1p-55;
        const double us = fabs(s) > 0x1p-2 ? ulps(s2, s) : fabs(s2 - s) / 0x1p-55;
        if (uc > mu) mu = uc;
        if (us > mu) mu = us;
        const double a = fmax(fabs(c2 - c), fabs(s2 - s));
        if (a > ma) ma = a;
        if ((c != 0.0 && signbit(c2) != signbit(c)) || (s != 0.0 && signbit(s2) != signbit(s))) ++bad_sign;
    }
    printf("%.6f %.6e %ld\n", mu, ma, bad_sign);
    return 0;
}
"""


def test_link_code_round_trip(tmp_path):
    src = tmp_path / "drv.c"
    src.write_text(DRIVER)
    exe = tmp_path / "drv"
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-I", os.path.join(REPO, "schwingermodel_amd", "csrc"),
                    str(src), "-o", str(exe), "-lm"], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split()
    mu, ma, bad_sign = float(out[0]), float(out[1]), int(out[2])
    assert mu <= 3.0, mu
    assert ma <= 3.5e-16, ma
    assert bad_sign == 0
