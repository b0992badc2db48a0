// sm_linkcode.h -- one double per U(1) link for the compact-link CG pass
// (sm_cgra.hip, UC): 8 instead of 16 B per link, decoded with one square root.
//
// A unit link U = (c, s) is stored as its smaller component v (s if |s| <= |c|,
// else c) with two flags in the two lowest mantissa bits: bit 1 = v is the
// cosine, bit 0 = the other component is negative. The decoder takes v as
// stored and rebuilds the other one as +-sqrt(1 - v^2), formed as
// sqrt(fma(-v, v, 1)). Because |v| <= 1/sqrt(2), 1 - v^2 >= 1/2 and the
// square root's sensitivity to v is |v| / sqrt(1 - v^2) <= 1. For a link ON
// the unit circle the rebuilt link is within 3 ulp (3.5e-16 absolute) per
// component (the flags move v by <= 2 ulp, the fma and the square root round
// once each; tests/test_linkcode_host.py). A link OFF the circle by
// delta = | |U|^2 - 1 | comes back with its larger component moved by a further
// ~delta / (2 |w|) <= 0.71 delta, because the decoder puts it back on the circle.
//
// So the guarantee is enforced link by link instead of assumed: the device
// kernel that builds the codes (sm_cgra.hip link_code_kernel) decodes every
// code with this same function and counts the links whose rebuilt components
// differ from the stored ones by more than SM_LINKCODE_TOL = 2^-51 (4.4e-16,
// 4 ulp of a component in [1/2, 1)). One such link anywhere and the field keeps
// the complex-link passes (sm_capi.cpp ensure_link_angles). Fresh exp(i theta)
// links (src/gauge_conf.cpp:23-29, the generator here) all pass: the config-3
// field generated on the device comes back within 2^-51 exactly (its links sit
// a few ulp off the circle; tests/test_gpu_parity.py). Links pushed off the
// circle by more than ~1.6e-15 in |U|^2 never pass (their larger component
// moves by >= delta / 2 - 3.5e-16), which is where many leapfrog updates
// (U <- U exp(i eps P), rounded each time) eventually take a field.
// Plain C as well, so tests/test_linkcode_host.py runs the same code on the
// host (with a perturbed reciprocal-square-root seed to model v_rsq_f64);
// tests/test_gpu_parity.py checks the device's own decode.
#pragma once

#include <stdint.h>
#include <string.h>

#define SM_LINKCODE_TOL 0x1p-51  // per component, absolute: the acceptance bound above

#ifdef __HIPCC__
#define SM_LINKCODE_FN __host__ __device__ __forceinline__
#else
#define SM_LINKCODE_FN static inline
#endif

SM_LINKCODE_FN uint64_t sm_lc_bits(double v) {
    uint64_t b;
    memcpy(&b, &v, sizeof b);
    return b;
}

SM_LINKCODE_FN double sm_lc_double(uint64_t b) {
    double v;
    memcpy(&v, &b, sizeof v);
    return v;
}

SM_LINKCODE_FN double sm_link_encode(double c, double s) {
    const int cosv = __builtin_fabs(s) > __builtin_fabs(c);  // store the cosine (the sine is the larger)
    const double v = cosv ? c : s, w = cosv ? s : c;
    const uint64_t f = ((uint64_t)cosv << 1) | (uint64_t)(__builtin_signbit(w) != 0);
    const uint64_t b = sm_lc_bits(v);
    // nearest bit pattern whose low two bits are f: |change| <= 2 in the
    // magnitude bits (sign-magnitude, so it moves v by <= 2 ulp)
    const uint64_t d = (f - b) & 3u;
    const uint64_t mag = b & 0x7fffffffffffffffull;
    const uint64_t e = (d == 3 && mag != 0) ? b - 1 : b + d;
    return sm_lc_double(e);
}

// sqrt(a) for a in [1/2, 1] (no scaling, no special cases): the hardware
// reciprocal square root (~2^-23 relative) on the device, 1 / sqrt on the host,
// then one Goldschmidt step (error ~2^-46) and one Newton correction of the
// root (~2^-92 before rounding): within 1 ulp, ~8 operations against ~18 for
// the general correctly rounded square root.
SM_LINKCODE_FN double sm_lc_sqrt_half1(double a) {
#ifdef __HIP_DEVICE_COMPILE__
    const double y = __builtin_amdgcn_rsq(a);
#else
    double y = 1.0 / __builtin_sqrt(a);
#ifdef SM_LC_HOST_SEED_PERTURB  // tests: a seed off by a relative 2^-22 or so, like the device's
    y *= 1.0 + (SM_LC_HOST_SEED_PERTURB);
#endif
#endif
    double g = a * y, h = 0.5 * y;
    const double r = __builtin_fma(-h, g, 0.5);
    g = __builtin_fma(g, r, g);
    h = __builtin_fma(h, r, h);
    const double d = __builtin_fma(-g, g, a);
    return __builtin_fma(d, h, g);
}

SM_LINKCODE_FN void sm_link_decode(double e, double *c_out, double *s_out) {
    const uint64_t b = sm_lc_bits(e);
    const double r = sm_lc_sqrt_half1(__builtin_fma(-e, e, 1.0));
    const double w = (b & 1u) ? -r : r;
    const int cosv = (int)((b >> 1) & 1u);
    *c_out = cosv ? e : w;
    *s_out = cosv ? w : e;
}

// 1 iff the code e of link (c, s) decodes to within SM_LINKCODE_TOL of it in
// both components (0 for NaN / Inf links).
SM_LINKCODE_FN int sm_link_code_ok(double c, double s, double e) {
    double c2, s2;
    sm_link_decode(e, &c2, &s2);
    const double err = __builtin_fmax(__builtin_fabs(c2 - c), __builtin_fabs(s2 - s));
    return err <= SM_LINKCODE_TOL && c - c == 0.0 && s - s == 0.0;
}
