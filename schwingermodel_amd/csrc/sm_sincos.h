// sm_sincos.h -- cos and sin of an angle in [-pi, pi] for the link-angle CG
// pass (sm_cgra.hip, UC): U(1) links rebuilt from their stored angles.
//
// Two-constant Cody-Waite reduction to r in [-pi/4, pi/4] (the quadrant
// q = rint(2 theta / pi) is at most 2 in size, so q * PIO2_HI is exact inside
// the fma), fdlibm's __kernel_sin / __kernel_cos polynomials on r, and the
// quadrant rotation: within 1 ulp of glibc's sin / cos over [-pi, pi]
// (tests/test_sincos_host.py compiles this same header for the host), ~25 fp64
// operations against ~60 for a general-argument sincos. Plain C as well, so
// the host test runs the exact device arithmetic (explicit fmas, no contraction).
//
// The polynomial coefficients and the cos-kernel's compensated sum below are
// those of fdlibm's k_sin.c / k_cos.c, which carry this notice:
//
//   Copyright (C) 1993 by Sun Microsystems, Inc. All rights reserved.
//
//   Developed at SunSoft, a Sun Microsystems, Inc. business.
//   Permission to use, copy, modify, and distribute this
//   software is freely granted, provided that this notice
//   is preserved.
#pragma once

#ifdef __HIPCC__
#define SM_SINCOS_FN __host__ __device__ __forceinline__
#else
#define SM_SINCOS_FN static inline
#endif

SM_SINCOS_FN void sm_cos_sin_pi(double th, double *c_out, double *s_out) {
    const double q = __builtin_rint(th * 0.63661977236758134308);
    double r = __builtin_fma(-q, 1.57079632679489655800e+00, th);
    r = __builtin_fma(-q, 6.12323399573676603587e-17, r);
    const double z = r * r;
    const double ps =
        __builtin_fma(z, __builtin_fma(z, __builtin_fma(z, __builtin_fma(z, 1.58969099521155010221e-10,
                                                                          -2.50507602534068634195e-08),
                                                        2.75573137070700676789e-06),
                                       -1.98412698298579493134e-04),
                      8.33333333332248946124e-03);
    const double rz = r * z;
    const double sn = __builtin_fma(rz, __builtin_fma(z, ps, -1.66666666666666324348e-01), r);
    const double pc =
        z * __builtin_fma(z, __builtin_fma(z, __builtin_fma(z, __builtin_fma(z, __builtin_fma(z,
                                                                             -1.13596475577881948265e-11,
                                                                             2.08757232129817482790e-09),
                                                                             -2.75573143513906633035e-07),
                                                            2.48015872894767294178e-05),
                                           -1.38888888888741095749e-03),
                          4.16666666666666019037e-02);
    const double hz = 0.5 * z, w = 1.0 - hz;
    const double zpc = z * pc;
    const double cs = w + (((1.0 - w) - hz) + zpc);
    const int k = (int)q & 3;  // theta = k pi/2 + r: (cos r, sin r) turned by k quarter turns
    const double c = (k & 1) ? sn : cs, sv = (k & 1) ? cs : sn;
    *c_out = (k == 1 || k == 2) ? -c : c;
    *s_out = (k >= 2) ? -sv : sv;
}
