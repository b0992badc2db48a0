// sm_linkcode.h -- exact compact U(1) links for the recompute-Ad CG pass
// (sm_cgra.hip, UC): 10 instead of 16 B per link, decoded with one square
// root, and BITWISE the stored link.
//
// A link U = (c, s) is stored as
//   v  (double): its smaller component (s if |s| <= |c|, else c), exactly as
//      stored, all 64 bits;
//   f  (uint16): bit 0 = the other component w is negative, bit 1 = v is the
//      cosine, bits 2..15 = a signed 14-bit count k of ulps between |w| and the
//      decoder's root r = sqrt(1 - v^2) (formed as sqrt(fma(-v, v, 1))).
// The decoder rebuilds |w| as the double whose bit pattern is bits(r) + k
// (positive doubles are ordered like their bit patterns, so this counts ulps
// across a binade boundary too, e.g. |w| = 1.0 against r = 1 - 2^-53), then
// sets its sign from bit 0. Encoder and decoder evaluate r with the SAME
// function, so every encodable link decodes to its stored bits exactly. A
// link is encodable iff both components are finite and |k| <= 8191: for a
// unit link k is 0..3 (r is within 1 ulp of the true root and |w| within a few
// ulps of it); a link pushed off the unit circle by delta = | |U|^2 - 1 |
// has |k| ~ delta / (2 |w| 2^-53), so 8191 covers delta up to ~1e-12. The
// reference's leapfrog multiplies U by exp(i eps P) every MD step
// (src/hmc.cpp:70-100) without re-unitarising, so |U| takes a random walk of
// ~0.55 sqrt(steps) ulps (a numpy model of the update: 379 ulps at most after
// 20000 steps of 200 000 links); it reaches the 14-bit range only after ~10^7
// steps. Round 4's codes kept v's two flag bits in its mantissa and accepted a
// link within 2^-51 of its stored components, so the first ~20 trajectories
// of an HMC pushed fields out of range (the pass then read complex links) and
// the pass's operator differed from D D^dag by a few ulps.
//
// Device layout (sm_capi.cpp ensure_link_angles): one allocation holds the
// codes v of both planes (2V doubles: U_t plane, then U_x plane), the flags f
// (2V uint16, same order) and the packed form's flag bytes (V bytes, below);
// the t-shard ghost faces likewise (16 Nx doubles, 16 Nx uint16, 8 Nx bytes).
// The pass reads v and either the flag words (20 B/site of links) or, when
// every offset of the field lies in [-2, 1] -- fresh exp(i theta) fields --
// the flag bytes (17 B/site).
// Plain C as well, so tests/test_linkcode_host.py runs the same code on the
// host (with a perturbed reciprocal-square-root seed to model v_rsq_f64; the
// host pair is exact for the host's own root, as the device pair is for the
// device's); tests/test_gpu_parity.py checks the device's own round trip.
#pragma once

#include <stdint.h>
#include <string.h>

#define SM_LINKCODE_KMAX 8191  // largest |k| a flag word holds (14-bit signed)

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

// sqrt(a) for a in ~[1/2, 1] (no scaling, no special cases): the hardware
// reciprocal square root (~2^-23 relative) on the device, 1 / sqrt on the host,
// then one Goldschmidt step (error ~2^-46) and one Newton correction of the
// root (~2^-92 before rounding): within 1 ulp, ~8 operations against ~18 for
// the general correctly rounded square root. Exactness of the codes does not
// depend on this accuracy (the offset k absorbs it), only their range does.
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

// The decoder's root for code v.
SM_LINKCODE_FN double sm_lc_root(double v) { return sm_lc_sqrt_half1(__builtin_fma(-v, v, 1.0)); }

// Code (v, f) of link (c, s); returns 1 iff the link is encodable (then the
// decoder gives back c and s bitwise), else 0 with f = 0.
SM_LINKCODE_FN int sm_link_encode(double c, double s, double *v_out, uint16_t *f_out) {
    const int cosv = __builtin_fabs(s) > __builtin_fabs(c);  // store the cosine (the sine is the larger)
    const double v = cosv ? c : s, w = cosv ? s : c;
    *v_out = v;
    *f_out = 0;
    if (!(c - c == 0.0 && s - s == 0.0)) return 0;  // NaN / Inf
    const int64_t k = (int64_t)sm_lc_bits(__builtin_fabs(w)) - (int64_t)sm_lc_bits(sm_lc_root(v));
    if (k < -SM_LINKCODE_KMAX || k > SM_LINKCODE_KMAX) return 0;
    *f_out = (uint16_t)(((uint32_t)(int32_t)k << 2) | ((uint32_t)cosv << 1) | (uint32_t)(__builtin_signbit(w) != 0));
    return 1;
}

SM_LINKCODE_FN void sm_link_decode(double v, uint16_t f, double *c_out, double *s_out) {
    const int64_t k = (int64_t)((int16_t)f >> 2);  // arithmetic shift: the signed offset
    const uint64_t wb = (uint64_t)((int64_t)sm_lc_bits(sm_lc_root(v)) + k) | ((uint64_t)(f & 1u) << 63);
    const double w = sm_lc_double(wb);
    const int cosv = (int)((f >> 1) & 1u);
    *c_out = cosv ? v : w;
    *s_out = cosv ? w : v;
}

// Packed form for fields whose every offset k lies in [-2, 1] (fresh
// exp(i theta) fields: |k| <= 1 measured): a link's flag word as a nibble
// (bit 0 sign of w, bit 1 v is the cosine, bits 2..3 k as 2-bit two's
// complement), the U_t nibble and the U_x nibble of a site in ONE byte --
// 17 instead of 20 B/site of links. sm_lc_nibble returns 0xff for a flag word
// that does not fit.
SM_LINKCODE_FN uint8_t sm_lc_nibble(uint16_t f) {
    const int k = (int16_t)f >> 2;
    return (k < -2 || k > 1) ? (uint8_t)0xff : (uint8_t)((f & 3u) | (((unsigned)k & 3u) << 2));
}

SM_LINKCODE_FN uint16_t sm_lc_flags_of_nibble(unsigned nib) {
    const int k = (int)((nib >> 2) & 3u) - (int)((nib >> 1) & 4u);  // sign-extend the 2-bit k
    return (uint16_t)((nib & 3u) | ((uint32_t)(int32_t)k << 2));
}

// 1 iff link (c, s) is encodable and its code decodes to it bitwise.
SM_LINKCODE_FN int sm_link_code_ok(double c, double s) {
    double v, c2, s2;
    uint16_t f;
    if (!sm_link_encode(c, s, &v, &f)) return 0;
    sm_link_decode(v, f, &c2, &s2);
    return sm_lc_bits(c2) == sm_lc_bits(c) && sm_lc_bits(s2) == sm_lc_bits(s);
}
