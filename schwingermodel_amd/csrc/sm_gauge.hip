// sm_gauge.hip -- gauge-field kernels of the molecular-dynamics step on gfx950
// (SURVEY.md §8f rows 1-3): plaquette field and sums, staples + gauge force,
// the fused momentum / link update of the leapfrog, the momentum kinetic
// energy, and device draws of momenta, pseudofermion sources and gauge fields.
//
// All are single-pass streaming kernels over the shard (HBM-bound, a few bytes
// of neighbour reuse per site that the L2 absorbs); the CG solves they sit
// between dominate an MD step by orders of magnitude. What matters here is
// bit-exact parity with the reference's expressions (same complex-multiply
// order, -ffp-contract=off) and that U, P and F never leave the device.
//
// Neighbour links across the t-shard boundary come from the 2-deep U faces
// ([col -2,-1,Wt,Wt+1][plane][x], exchanged by exchange_ghost_U after every
// link update); one shard wraps periodically in place.
#include "sm_device.h"
#include "sm_fields.h"

#include <float.h>

namespace sm {

struct GArgs {
    const double2 *U;    // 2V: plane 0 U_t, plane 1 U_x
    const double2 *fU;   // 2-deep U faces (nshard > 1)
    long V;
    int Nx, Wt, nshard;
};

// U_plane(x, t = c) for c in [-1, Wt]; x already in [0, Nx).
__device__ __forceinline__ double2 ulink(const GArgs &a, int p, int x, int c) {
    if (c >= 0 && c < a.Wt) return a.U[(long)x * a.Wt + c + p * a.V];
    if (a.nshard == 1) return a.U[(long)x * a.Wt + (c < 0 ? c + a.Wt : c - a.Wt) + p * a.V];
    const int fc = c < 0 ? c + 2 : c - a.Wt + 2;  // face slot of columns -2,-1,Wt,Wt+1
    return a.fU[((long)fc * 2 + p) * a.Nx + x];
}

// ---- plaquette: U_01(n) = U_0(n) U_1(n+0) U*_0(n+1) U*_1(n) ----------------
// src/gauge_conf.cpp:45-49; sums as MeasureSp_HMC (:430-440) and
// Compute_gaugeAction (:444-453): partial.x = sum Re U_01,
// partial.y = sum beta Re(1 - U_01).
__global__ void __launch_bounds__(256) plaquette_kernel(GArgs a, double beta, double2 *field,
                                                        double2 *partials) {
    __shared__ double2 sh[4];
    double2 acc = make_double2(0.0, 0.0);
    for (long n = (long)blockIdx.x * blockDim.x + threadIdx.x; n < a.V; n += (long)gridDim.x * blockDim.x) {
        const int x = (int)(n / a.Wt), t = (int)(n - (long)x * a.Wt);
        const int xp = x + 1 == a.Nx ? 0 : x + 1;
        const double2 P = cmul(cmul(cmul(a.U[n], ulink(a, 1, x, t + 1)), cconj(ulink(a, 0, xp, t))),
                               cconj(a.U[n + a.V]));
        if (field) field[n] = P;
        acc.x += P.x;
        acc.y += beta * (1.0 - P.x);
    }
    const double2 s = block_sum(acc, sh);
    if (threadIdx.x == 0) partials[blockIdx.x] = s;
}

// ---- staples and gauge force (src/gauge_conf.cpp:95-125; src/hmc.cpp:31-40) --
//   S_0(n) = U_1(n) U_0(n+1) U*_1(n+0) + U*_1(n-1) U_0(n-1) U_1(n-1+0)
//   S_1(n) = U_0(n) U_1(n+0) U*_0(n+1) + U*_0(n-0) U_1(n-0) U_0(n+1-0)
//   F_mu(n) += -beta Im(U_mu(n) conj(S_mu(n)))
// (0 = t direction, 1 = x direction; "n+1" is x+1, "n+0" is t+1.)
__global__ void __launch_bounds__(256) staple_force_kernel(GArgs a, double beta, double *F,
                                                           double2 *staples) {
    for (long n = (long)blockIdx.x * blockDim.x + threadIdx.x; n < a.V; n += (long)gridDim.x * blockDim.x) {
        const int x = (int)(n / a.Wt), t = (int)(n - (long)x * a.Wt);
        const int xp = x + 1 == a.Nx ? 0 : x + 1, xm = x == 0 ? a.Nx - 1 : x - 1;
        const double2 u0 = a.U[n], u1 = a.U[n + a.V];
        const double2 S0 = cadd(cmul(cmul(u1, ulink(a, 0, xp, t)), cconj(ulink(a, 1, x, t + 1))),
                                cmul(cmul(cconj(ulink(a, 1, xm, t)), ulink(a, 0, xm, t)), ulink(a, 1, xm, t + 1)));
        const double2 S1 = cadd(cmul(cmul(u0, ulink(a, 1, x, t + 1)), cconj(ulink(a, 0, xp, t))),
                                cmul(cmul(cconj(ulink(a, 0, x, t - 1)), ulink(a, 1, x, t - 1)), ulink(a, 0, xp, t - 1)));
        if (staples) {
            staples[n] = S0;
            staples[n + a.V] = S1;
        }
        if (F) {
            F[n] += -beta * cmul(u0, cconj(S0)).y;
            F[n + a.V] += -beta * cmul(u1, cconj(S1)).y;
        }
    }
}

// ---- leapfrog link / momentum update (src/hmc.cpp:63-101) --------------------
//   do_p:  P += eps * F
//   U *= exp(i coef P): std::exp of (+-0, coef*P) is glibc cexp = (cos y, sin y)
//          for |y| > DBL_MIN and (1, y) below (s_cexp_template.c); then the
//          plain complex product. coef = eps (full step) or 0.5*eps (half).
__global__ void __launch_bounds__(256) md_update_kernel(long n2, double2 *U, double *P, const double *F,
                                                        double eps, int do_p, double coef) {
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n2; i += (long)gridDim.x * blockDim.x) {
        double p = P[i];
        if (do_p) {
            p += eps * F[i];
            P[i] = p;
        }
        const double y = coef * p;
        double s, c;
        if (fabs(y) > DBL_MIN) {
            sincos(y, &s, &c);
        } else {
            s = y;
            c = 1.0;
        }
        U[i] = cmul(U[i], make_double2(c, s));
    }
}

// ---- momentum kinetic energy: sum_n 0.5 P_0^2 + 0.5 P_1^2 (src/hmc.cpp:107-111)
__global__ void __launch_bounds__(256) kinetic_kernel(long V, const double *P, double2 *partials) {
    __shared__ double2 sh[4];
    double2 acc = make_double2(0.0, 0.0);
    for (long n = (long)blockIdx.x * blockDim.x + threadIdx.x; n < V; n += (long)gridDim.x * blockDim.x) {
        acc.x += 0.5 * P[n] * P[n];
        acc.x += 0.5 * P[n + V] * P[n + V];
    }
    const double2 s = block_sum(acc, sh);
    if (threadIdx.x == 0) partials[blockIdx.x] = s;
}

// ---- device draws (counter-based, keyed by the GLOBAL site: every sharding
// draws the same global field) ------------------------------------------------
struct DrawArgs {
    uint64_t seed;
    long V;
    int Nx, Wt, t0, Ntg;
};

__device__ __forceinline__ uint64_t global_site(const DrawArgs &a, long n, int &x, int &t) {
    x = (int)(n / a.Wt);
    t = (int)(n - (long)x * a.Wt);
    return (uint64_t)x * (uint64_t)a.Ntg + (uint64_t)(a.t0 + t);
}

// HMC::RandomPI (src/hmc.cpp:5-16): Pi_mu(n) ~ N(0, 1).
__global__ void __launch_bounds__(256) draw_momenta_kernel(DrawArgs a, double *P) {
    for (long n = (long)blockIdx.x * blockDim.x + threadIdx.x; n < a.V; n += (long)gridDim.x * blockDim.x) {
        int x, t;
        const uint64_t ng = global_site(a, n, x, t);
        double g1, g2;
        sm_gauss2(a.seed, SM_STREAM_MOMENTA, ng, &g1, &g2);
        P[n] = g1;
        P[n + a.V] = g2;
    }
}

// HMC::RandomCHI (src/hmc.cpp:19-28): Re, Im ~ N(0, 1/2) per spin component
// (same streams and scaling as the host spinor generator).
__global__ void __launch_bounds__(256) draw_source_kernel(DrawArgs a, double2 *chi) {
    const double s = 0.70710678118654752440084436210485;
    for (long n = (long)blockIdx.x * blockDim.x + threadIdx.x; n < a.V; n += (long)gridDim.x * blockDim.x) {
        int x, t;
        const uint64_t ng = global_site(a, n, x, t);
        double g1, g2;
        sm_gauss2(a.seed, 4, ng, &g1, &g2);
        chi[n] = make_double2(s * g1, s * g2);
        sm_gauss2(a.seed, 5, ng, &g1, &g2);
        chi[n + a.V] = make_double2(s * g1, s * g2);
    }
}

// Gauge field of the host generator (sm_fields_fill_gauge), drawn in place.
__global__ void __launch_bounds__(256) draw_gauge_kernel(DrawArgs a, double sigma, double2 *U) {
    for (long n = (long)blockIdx.x * blockDim.x + threadIdx.x; n < a.V; n += (long)gridDim.x * blockDim.x) {
        int x, t;
        const uint64_t ng = global_site(a, n, x, t);
        for (int mu = 0; mu < 2; ++mu) {
            double re, im;
            sm_gauge_link(a.seed, sigma, ng, mu, &re, &im);
            U[n + mu * a.V] = make_double2(re, im);
        }
    }
}

// ---- launchers -----------------------------------------------------------------
namespace {
GArgs gargs(const Geometry &g, int nshard, const double2 *U, const double2 *fU) {
    GArgs a;
    a.U = U;
    a.fU = fU;
    a.V = g.V;
    a.Nx = g.Nx;
    a.Wt = g.Wt;
    a.nshard = nshard;
    return a;
}
DrawArgs dargs(const Geometry &g, uint64_t seed) {
    DrawArgs a;
    a.seed = seed;
    a.V = g.V;
    a.Nx = g.Nx;
    a.Wt = g.Wt;
    a.t0 = g.t0;
    a.Ntg = g.Ntg;
    return a;
}
unsigned grid_for(long n) {
    long nb = (n + 255) / 256;
    return (unsigned)(nb > 4096 ? 4096 : (nb < 1 ? 1 : nb));
}
}  // namespace

int gauge_reduce_blocks(const Geometry &g) { return reduce_blocks(g.V); }

void launch_plaquette(hipStream_t s, const Geometry &g, int nshard, const double2 *U, const double2 *fU,
                      double beta, double2 *field, double2 *partials) {
    hipLaunchKernelGGL(plaquette_kernel, dim3(gauge_reduce_blocks(g)), dim3(256), 0, s, gargs(g, nshard, U, fU),
                       beta, field, partials);
}

void launch_staple_force(hipStream_t s, const Geometry &g, int nshard, const double2 *U, const double2 *fU,
                         double beta, double *F, double2 *staples) {
    hipLaunchKernelGGL(staple_force_kernel, dim3(grid_for(g.V)), dim3(256), 0, s, gargs(g, nshard, U, fU), beta,
                       F, staples);
}

void launch_md_update(hipStream_t s, const Geometry &g, double2 *U, double *P, const double *F, double eps,
                      int do_p, double coef) {
    hipLaunchKernelGGL(md_update_kernel, dim3(grid_for(2 * g.V)), dim3(256), 0, s, 2 * g.V, U, P, F, eps, do_p,
                       coef);
}

void launch_kinetic(hipStream_t s, const Geometry &g, const double *P, double2 *partials) {
    hipLaunchKernelGGL(kinetic_kernel, dim3(gauge_reduce_blocks(g)), dim3(256), 0, s, g.V, P, partials);
}

void launch_draw_momenta(hipStream_t s, const Geometry &g, uint64_t seed, double *P) {
    hipLaunchKernelGGL(draw_momenta_kernel, dim3(grid_for(g.V)), dim3(256), 0, s, dargs(g, seed), P);
}

void launch_draw_source(hipStream_t s, const Geometry &g, uint64_t seed, double2 *chi) {
    hipLaunchKernelGGL(draw_source_kernel, dim3(grid_for(g.V)), dim3(256), 0, s, dargs(g, seed), chi);
}

void launch_draw_gauge(hipStream_t s, const Geometry &g, uint64_t seed, double sigma, double2 *U) {
    hipLaunchKernelGGL(draw_gauge_kernel, dim3(grid_for(g.V)), dim3(256), 0, s, dargs(g, seed), sigma, U);
}

}  // namespace sm
