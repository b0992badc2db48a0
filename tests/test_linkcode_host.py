"""The compact-link CG pass stores each U(1) link as its smaller component v
(a double, exact) plus a 16-bit flag word (which component v is, the sign of
the other one, and a signed ulp offset k of the other one from the decoder's
root sqrt(1 - v^2)); schwingermodel_amd/csrc/sm_linkcode.h. The header is plain
C as well and is compiled here for the host (gcc, explicit fma, no contraction).

The host build is NOT bit-for-bit the device's: the device seeds the square
root with the hardware reciprocal square root (v_rsq_f64, __builtin_amdgcn_rsq),
the host with 1 / sqrt (SM_LC_HOST_SEED_PERTURB models a seed off by a relative
2^-22 either way). Exactness does not depend on the seed: the encoder measures
k against the SAME root the decoder forms, so on each side the pair round-trips
bitwise; the device's own round trip is checked on the device
(tests/test_gpu_parity.py, test_link_codes_*). Here, for each seed model:
  * unit links of every quadrant, the axes, the diagonal ties, tiny angles:
    encodable, rebuilt bitwise, |k| <= 3;
  * links off the unit circle by 1 + j 2^-53 (|j| <= 40) and links after
    20000 steps of the leapfrog's link update U <- U exp(i y) (src/hmc.cpp:70,
    rounded every step, never re-unitarised): encodable and rebuilt bitwise;
  * links off the circle by 1e-9 (|k| far beyond 8191), NaN and Inf: not
    encodable (the pass then reads the complex links);
  * the packed form's flag nibble (k in [-2, 1]) round-trips every flag word
    it accepts and refuses every other.
"""
import os
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

DRIVER = r"""
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include "sm_linkcode.h"
static long kmax = 0, inexact = 0, rejected = 0;
/* encode + decode; counts links that are encodable but not rebuilt bitwise, and not encodable */
static int trip(double c, double s) {
    double v, c2, s2;
    uint16_t f;
    if (!sm_link_encode(c, s, &v, &f)) { ++rejected; return 0; }
    sm_link_decode(v, f, &c2, &s2);
    if (sm_lc_bits(c2) != sm_lc_bits(c) || sm_lc_bits(s2) != sm_lc_bits(s)) ++inexact;
    const long k = labs((long)((int16_t)f >> 2));
    if (k > kmax) kmax = k;
    if (sm_link_code_ok(c, s) != 1) ++inexact;
    return 1;
}
int main(void) {
    const double special[] = {0.0, -0.0, M_PI, -M_PI, M_PI / 2, -M_PI / 2, M_PI / 4, -M_PI / 4,
                              3 * M_PI / 4, -3 * M_PI / 4, 1e-300, -1e-20};
    const long n = 4000000;
    srand48(11);
    for (long i = 0; i < n; ++i) {
        double th = i < 12 ? special[i] : (drand48() * 2.0 - 1.0) * M_PI;
        if (i >= 12 && i < 4000) th = nextafter(((i % 9) - 4) * M_PI_4, (i & 1) ? INFINITY : -INFINITY);
        trip(cos(th), sin(th));
    }
    const long unit_kmax = kmax, unit_rejected = rejected;
    /* off the circle by 1 + j 2^-53 */
    for (long i = 0; i < 400000; ++i) {
        const double th = (drand48() * 2.0 - 1.0) * M_PI, f = 1.0 + (double)(i % 81 - 40) * 0x1p-53;
        trip(cos(th) * f, sin(th) * f);
    }
    /* the leapfrog's update U <- U (cos y, sin y), 20000 steps on 2000 links */
    for (long l = 0; l < 2000; ++l) {
        const double th = (drand48() * 2.0 - 1.0) * M_PI;
        double c = cos(th), s = sin(th);
        for (int st = 0; st < 20000; ++st) {
            const double y = (drand48() - 0.5) * 0.4, cy = cos(y), sy = sin(y);
            const double c1 = c * cy - s * sy, s1 = c * sy + s * cy;
            c = c1;
            s = s1;
        }
        trip(c, s);
    }
    const long drift_rejected = rejected - unit_rejected;
    /* never encodable: far off the circle, NaN, Inf */
    long far_ok = 0;
    for (long i = 0; i < 1000; ++i) {
        const double th = (drand48() * 2.0 - 1.0) * M_PI;
        double v;
        uint16_t f;
        far_ok += sm_link_encode(cos(th) * (1.0 + 1e-9), sin(th) * (1.0 + 1e-9), &v, &f);
    }
    double v;
    uint16_t f;
    far_ok += sm_link_encode(0.0 / 0.0, 0.5, &v, &f) + sm_link_encode(0.5, INFINITY, &v, &f);
    far_ok += sm_link_code_ok(0.0 / 0.0, 0.5) + sm_link_code_ok(2.0, 2.0);
    /* the packed flags: every nibble round-trips, offsets outside [-2, 1] do not pack */
    long nib_bad = 0;
    for (int k = -8191; k <= 8191; ++k)
        for (unsigned lo = 0; lo < 4; ++lo) {
            const uint16_t f = (uint16_t)(((uint32_t)(int32_t)k << 2) | lo);
            const uint8_t nb = sm_lc_nibble(f);
            if (k >= -2 && k <= 1) nib_bad += nb > 15 || sm_lc_flags_of_nibble(nb) != f;
            else nib_bad += nb != 0xff;
        }
    printf("%ld %ld %ld %ld %ld %ld %ld\n", unit_kmax, unit_rejected, drift_rejected, inexact, kmax, far_ok, nib_bad);
    return 0;
}
"""


@pytest.mark.parametrize("perturb", [None, "0x1p-22", "-0x1p-22"], ids=["exact_seed", "seed_hi", "seed_lo"])
def test_link_code_round_trip(tmp_path, perturb):
    src = tmp_path / "drv.c"
    src.write_text(DRIVER)
    exe = tmp_path / "drv"
    cmd = ["gcc", "-O2", "-ffp-contract=off", "-I", os.path.join(REPO, "schwingermodel_amd", "csrc"),
           str(src), "-o", str(exe), "-lm"]
    if perturb:
        cmd.insert(1, f"-DSM_LC_HOST_SEED_PERTURB={perturb}")
    subprocess.run(cmd, check=True)
    out = [int(v) for v in subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split()]
    unit_kmax, unit_rejected, drift_rejected, inexact, kmax, far_ok, nib_bad = out
    print(f"unit links |k| <= {unit_kmax}; largest |k| over all encodable links {kmax}")
    assert unit_rejected == 0 and unit_kmax <= 3, out
    assert drift_rejected == 0, out          # 20000 leapfrog updates stay in the 14-bit range
    assert inexact == 0, out                 # every encodable link is rebuilt bitwise
    assert kmax <= 8191, out
    assert far_ok == 0, out                  # 1e-9 off the circle, NaN, Inf: never encodable
    assert nib_bad == 0, out                 # flag nibbles: exact for k in [-2, 1], refused otherwise
