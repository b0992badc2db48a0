/*
 * sm_fields.h -- counter-based synthetic field generator (host C, header-only).
 *
 * Every value is a pure function of (seed, global site, stream), so each
 * t-shard / GPU / CPU process generates exactly its own slice of the same
 * global field with no communication (SURVEY.md §8d "Seeds").
 *
 *   gauge   U_mu(n) = exp(i theta),  theta ~ N(0, sigma^2)   (sigma > 0)
 *                                    theta ~ U(-pi, pi]       (sigma < 0: "hot")
 *                                    theta = 0                (sigma == 0: "cold")
 *   spinor  psi_a(n) = (g1 + i g2) / sqrt(2),  g ~ N(0,1)  -- the
 *           distribution of HMC::RandomCHI, src/hmc.cpp:19-28.
 *
 * Layout: two planes of interleaved complex<double>, local site index
 * n = (x - x0)*Wt + t, covering global rows [x0, x0+nx) and global t in
 * [t0, t0+Wt) of a lattice with Nt_global (one rank's block,
 * include/mpi_setup.h:20-22).
 *
 * The scalar generator functions are also compiled for the device
 * (sm_gauge.hip draws HMC momenta and pseudofermion sources on the GPU).
 * There log/sincos are the device math library's, which may differ from
 * glibc in the last bit: device-drawn fields are the same distribution, not
 * bit-identical to host-drawn ones.
 */
#ifndef SM_FIELDS_H
#define SM_FIELDS_H
#ifndef _GNU_SOURCE
#define _GNU_SOURCE 1
#endif
#include <math.h>
#include <stdint.h>

#if defined(__HIPCC__)
#define SM_FIELDS_HD __host__ __device__
#else
#define SM_FIELDS_HD
#endif

SM_FIELDS_HD static inline uint64_t sm_mix64(uint64_t z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

/* Uniform in (0, 1], 53 random bits, from (seed, stream, index). */
SM_FIELDS_HD static inline double sm_uniform(uint64_t seed, uint64_t stream, uint64_t idx) {
    uint64_t k = sm_mix64(sm_mix64(seed ^ (0xD1B54A32D192ED03ull * (stream + 1))) + idx);
    return (double)((k >> 11) + 1) * (1.0 / 9007199254740992.0);
}

/* Box-Muller pair of independent N(0,1) draws for (seed, stream pair, index). */
SM_FIELDS_HD static inline void sm_gauss2(uint64_t seed, uint64_t stream, uint64_t idx,
                             double *g1, double *g2) {
    const double two_pi = 6.283185307179586476925286766559;
    double u1 = sm_uniform(seed, 2 * stream, idx);
    double u2 = sm_uniform(seed, 2 * stream + 1, idx);
    double rad = sqrt(-2.0 * log(u1));
    /* glibc sincos explicitly: g++ merges cos+sin into sincos, whose last bit
     * can differ from separate calls; one entry point for every compiler. */
    double s, c;
    sincos(two_pi * u2, &s, &c);
    *g1 = rad * c;
    *g2 = rad * s;
}

/* Per-trajectory key of the HMC draws (momenta, sources, accept/reject). */
SM_FIELDS_HD static inline uint64_t sm_traj_seed(uint64_t seed, uint64_t traj) {
    return sm_mix64(seed ^ sm_mix64(traj ^ 0x6A09E667F3BCC909ull));
}

/* Stream ids: gauge theta 0/1 (Gaussian pairs) and 16/17 (hot); spinor
 * planes 4/5; HMC momenta 6 (one Box-Muller pair = both links of a site);
 * Metropolis uniform 7 (uniform stream 7, index 0). */
#define SM_STREAM_MOMENTA 6
#define SM_STREAM_ACCEPT 7

/* Gauge link of global site ng: exp(i theta), theta per sigma (see top). */
SM_FIELDS_HD static inline void sm_gauge_link(uint64_t seed, double sigma, uint64_t ng, int mu,
                                              double *re, double *im) {
    const double pi = 3.141592653589793238462643383279;
    double th, g1, g2;
    if (sigma > 0.0) {
        sm_gauss2(seed, (uint64_t)mu, ng, &g1, &g2);
        th = sigma * g1;
    } else if (sigma < 0.0) {
        th = pi * (2.0 * sm_uniform(seed, 16 + (uint64_t)mu, ng) - 1.0);
    } else {
        th = 0.0;
    }
    sincos(th, im, re);
}

static inline void sm_fields_fill_gauge(uint64_t seed, double sigma, int Nt_global, int x0,
                                        int nx, int t0, int Wt, double *U0, double *U1) {
    for (int x = 0; x < nx; x++) {
        for (int t = 0; t < Wt; t++) {
            const uint64_t ng = (uint64_t)(x0 + x) * (uint64_t)Nt_global + (uint64_t)(t0 + t);
            const long n = (long)x * Wt + t;
            for (int mu = 0; mu < 2; mu++) {
                double *U = mu ? U1 : U0;
                sm_gauge_link(seed, sigma, ng, mu, &U[2 * n], &U[2 * n + 1]);
            }
        }
    }
}

static inline void sm_fields_fill_spinor(uint64_t seed, int Nt_global, int x0, int nx, int t0,
                                         int Wt, double *p0, double *p1) {
    const double s = 0.70710678118654752440084436210485;
    for (int x = 0; x < nx; x++) {
        for (int t = 0; t < Wt; t++) {
            const uint64_t ng = (uint64_t)(x0 + x) * (uint64_t)Nt_global + (uint64_t)(t0 + t);
            const long n = (long)x * Wt + t;
            double g1, g2;
            sm_gauss2(seed, 4, ng, &g1, &g2);
            p0[2 * n] = s * g1;
            p0[2 * n + 1] = s * g2;
            sm_gauss2(seed, 5, ng, &g1, &g2);
            p1[2 * n] = s * g1;
            p1[2 * n + 1] = s * g2;
        }
    }
}

#endif
