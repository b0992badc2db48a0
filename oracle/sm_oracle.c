/*
 * sm_oracle.c -- CPU ORACLE (test infrastructure only; see sm_oracle.h).
 *
 * Clean-room restatement of the reference hot path from HMC_doc.pdf eqs.
 * (34)-(38) and the CG on pp. 5-6, with every expression evaluated in the
 * same order and with the same (non-fused) complex arithmetic as the
 * reference's std::complex<double> code, so that results are bit-identical.
 * Build with -ffp-contract=off (oracle/Makefile) -- x86-64 baseline g++ -O3,
 * which built the reference, never contracts to FMA.
 */
#include "sm_oracle.h"
#include <math.h>
#include <pthread.h>
#include <stdlib.h>

typedef struct { double re, im; } cplx;

static inline cplx C(double re, double im) { cplx z = {re, im}; return z; }
static inline cplx ld(const double *p, long i) { return C(p[2 * i], p[2 * i + 1]); }
static inline void st(double *p, long i, cplx z) { p[2 * i] = z.re; p[2 * i + 1] = z.im; }
static inline cplx cadd(cplx a, cplx b) { return C(a.re + b.re, a.im + b.im); }
static inline cplx csub(cplx a, cplx b) { return C(a.re - b.re, a.im - b.im); }
static inline cplx cneg(cplx a) { return C(-a.re, -a.im); }
static inline cplx cconj(cplx a) { return C(a.re, -a.im); }
/* GCC's expansion of complex*complex: (ac - bd, ad + bc), no contraction. */
static inline cplx cmul(cplx a, cplx b) {
    return C(a.re * b.re - a.im * b.im, a.re * b.im + a.im * b.re);
}
/* real * complex (libstdc++ operator*(const T&, const complex<T>&)). */
static inline cplx rmul(double s, cplx a) { return C(s * a.re, s * a.im); }

/* I_number = (0, 1), src/dirac_operator.cpp:3; -I_number = (-0, -1). */
static const cplx I_num = {0.0, 1.0};
static const cplx mI_num = {-0.0, -1.0};

void oracle_cdiv(double a, double b, double c, double d, double *re, double *im) {
    /* libgcc2.c __divdc3 as shipped with GCC 11 (Smith's method, no scaling). */
    double denom, ratio, x, y;
    if (fabs(c) < fabs(d)) {
        ratio = c / d;
        denom = (c * ratio) + d;
        x = ((a * ratio) + b) / denom;
        y = ((b * ratio) - a) / denom;
    } else {
        ratio = d / c;
        denom = (d * ratio) + c;
        x = ((b * ratio) + a) / denom;
        y = (b - (a * ratio)) / denom;
    }
    /* NaN recovery branch of __divdc3 is never taken for finite CG scalars. */
    *re = x;
    *im = y;
}

/* Neighbour sources for one t-domain: either periodic wrap inside the array
 * or explicit faces (t-sharded domain). */
typedef struct {
    int Nx, Wt, t0, Ntg;
    const double *U0, *U1, *in0, *in1;
    const double *lo0, *lo1, *loU, *hi0, *hi1;
} dom_t;

/* Site kernel: reference src/dirac_operator.cpp:31-43 (D) and :255-267 (D^dagger). */
static void dirac_site(const dom_t *g, int x, int t, double m0, int dagger,
                       double *out0, double *out1) {
    const int Wt = g->Wt, Nx = g->Nx;
    const long n = (long)x * Wt + t;
    const long nxp = (long)((x + 1) % Nx) * Wt + t;          /* RightPB[2n+1] */
    const long nxm = (long)((x - 1 + Nx) % Nx) * Wt + t;     /* LeftPB[2n+1]  */
    cplx p0 = ld(g->in0, n), p1 = ld(g->in1, n);
    cplx pt0, pt1, pm0, pm1, Utm;                             /* psi(n+t), psi(n-t), U_t(n-t) */
    if (t + 1 < Wt) { pt0 = ld(g->in0, n + 1); pt1 = ld(g->in1, n + 1); }
    else if (g->hi0) { pt0 = ld(g->hi0, x); pt1 = ld(g->hi1, x); }
    else { pt0 = ld(g->in0, n + 1 - Wt); pt1 = ld(g->in1, n + 1 - Wt); }
    if (t > 0) { pm0 = ld(g->in0, n - 1); pm1 = ld(g->in1, n - 1); Utm = ld(g->U0, n - 1); }
    else if (g->lo0) { pm0 = ld(g->lo0, x); pm1 = ld(g->lo1, x); Utm = ld(g->loU, x); }
    else { pm0 = ld(g->in0, n - 1 + Wt); pm1 = ld(g->in1, n - 1 + Wt); Utm = ld(g->U0, n - 1 + Wt); }
    cplx px0 = ld(g->in0, nxp), px1 = ld(g->in1, nxp);
    cplx pxm0 = ld(g->in0, nxm), pxm1 = ld(g->in1, nxm);
    cplx Ut = ld(g->U0, n), Ux = ld(g->U1, n), Uxm = ld(g->U1, nxm);
    /* SignR/SignL, include/dirac_operator.h:51-58: -1 only for mu=0 at the
     * global t boundary (antiperiodic fermions); complex +-1. */
    const int tg = g->t0 + t;
    cplx SR0 = C(tg == g->Ntg - 1 ? -1.0 : 1.0, 0.0), SR1 = C(1.0, 0.0);
    cplx SL0 = C(tg == 0 ? -1.0 : 1.0, 0.0), SL1 = C(1.0, 0.0);
    cplx a = cmul(Ut, SR0), b = cmul(Ux, SR1);
    cplx c = cmul(cconj(Utm), SL0), e = cmul(cconj(Uxm), SL1);
    const double mass = m0 + 2;
    cplx s0, s1;
    if (!dagger) {
        /* (D psi)_0 = (m0+2) psi_0 - 1/2 [A + B + C + E], src/dirac_operator.cpp:31-36 */
        cplx A = cmul(a, csub(pt0, pt1));
        cplx B = cmul(b, cadd(px0, cmul(I_num, px1)));
        cplx Cc = cmul(c, cadd(pm0, pm1));
        cplx E = cmul(e, csub(pxm0, cmul(I_num, pxm1)));
        s0 = csub(rmul(mass, p0), rmul(0.5, cadd(cadd(cadd(A, B), Cc), E)));
        /* (D psi)_1, src/dirac_operator.cpp:38-43 */
        A = cmul(a, cadd(cneg(pt0), pt1));
        B = cmul(b, cadd(cmul(mI_num, px0), px1));
        Cc = cmul(c, cadd(pm0, pm1));
        E = cmul(e, cadd(cmul(I_num, pxm0), pxm1));
        s1 = csub(rmul(mass, p1), rmul(0.5, cadd(cadd(cadd(A, B), Cc), E)));
    } else {
        /* D^dagger, src/dirac_operator.cpp:255-267: backward hops first. */
        cplx Cc = cmul(c, csub(pm0, pm1));
        cplx E = cmul(e, cadd(pxm0, cmul(I_num, pxm1)));
        cplx A = cmul(a, cadd(pt0, pt1));
        cplx B = cmul(b, csub(px0, cmul(I_num, px1)));
        s0 = csub(rmul(mass, p0), rmul(0.5, cadd(cadd(cadd(Cc, E), A), B)));
        Cc = cmul(c, cadd(cneg(pm0), pm1));
        E = cmul(e, cadd(cmul(mI_num, pxm0), pxm1));
        A = cmul(a, cadd(pt0, pt1));
        B = cmul(b, cadd(cmul(I_num, px0), px1));
        s1 = csub(rmul(mass, p1), rmul(0.5, cadd(cadd(cadd(Cc, E), A), B)));
    }
    st(out0, n, s0);
    st(out1, n, s1);
}

static void dirac_rows(const dom_t *g, int xb, int xe, double m0, int dagger,
                       double *out0, double *out1) {
    for (int x = xb; x < xe; x++)
        for (int t = 0; t < g->Wt; t++) dirac_site(g, x, t, m0, dagger, out0, out1);
}

void oracle_dirac_local(int Nx, int Wt, int t0, int Nt_global,
                        const double *U0, const double *U1,
                        const double *in0, const double *in1,
                        const double *lo_psi0, const double *lo_psi1, const double *lo_U0,
                        const double *hi_psi0, const double *hi_psi1,
                        double *out0, double *out1, double m0, int dagger) {
    dom_t g = {Nx, Wt, t0, Nt_global, U0, U1, in0, in1,
               lo_psi0, lo_psi1, lo_U0, hi_psi0, hi_psi1};
    dirac_rows(&g, 0, Nx, m0, dagger, out0, out1);
}

void oracle_dirac(int Nx, int Nt, const double *U0, const double *U1,
                  const double *in0, const double *in1, double *out0, double *out1,
                  double m0, int dagger) {
    oracle_dirac_local(Nx, Nt, 0, Nt, U0, U1, in0, in1, 0, 0, 0, 0, 0,
                       out0, out1, m0, dagger);
}

typedef struct {
    const dom_t *g;
    int xb, xe, dagger;
    double m0;
    double *out0, *out1;
} job_t;

static void *dirac_job(void *p) {
    job_t *j = (job_t *)p;
    dirac_rows(j->g, j->xb, j->xe, j->m0, j->dagger, j->out0, j->out1);
    return 0;
}

void oracle_dirac_mt(int Nx, int Nt, const double *U0, const double *U1,
                     const double *in0, const double *in1, double *out0, double *out1,
                     double m0, int dagger, int nthreads) {
    dom_t g = {Nx, Nt, 0, Nt, U0, U1, in0, in1, 0, 0, 0, 0, 0};
    if (nthreads < 1) nthreads = 1;
    if (nthreads > Nx) nthreads = Nx;
    pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * nthreads);
    job_t *jobs = (job_t *)malloc(sizeof(job_t) * nthreads);
    for (int i = 0; i < nthreads; i++) {
        jobs[i].g = &g;
        jobs[i].xb = (int)((long)Nx * i / nthreads);
        jobs[i].xe = (int)((long)Nx * (i + 1) / nthreads);
        jobs[i].dagger = dagger;
        jobs[i].m0 = m0;
        jobs[i].out0 = out0;
        jobs[i].out1 = out1;
        pthread_create(&th[i], 0, dirac_job, &jobs[i]);
    }
    for (int i = 0; i < nthreads; i++) pthread_join(th[i], 0);
    free(th);
    free(jobs);
}

void oracle_ddag(int Nx, int Nt, const double *U0, const double *U1,
                 const double *in0, const double *in1, double *tmp0, double *tmp1,
                 double *out0, double *out1, double m0) {
    /* src/dirac_operator.cpp:477-480: D(D^dagger psi) through DTEMP. */
    oracle_dirac(Nx, Nt, U0, U1, in0, in1, tmp0, tmp1, m0, 1);
    oracle_dirac(Nx, Nt, U0, U1, tmp0, tmp1, out0, out1, m0, 0);
}

void oracle_force(int Nx, int Nt, const double *U0, const double *U1,
                  const double *l0, const double *l1, const double *r0, const double *r1,
                  double *F0, double *F1) {
    /* src/dirac_operator.cpp:493-506, eqs. (37)-(38). */
    for (int x = 0; x < Nx; x++) {
        for (int t = 0; t < Nt; t++) {
            const long n = (long)x * Nt + t;
            const long nt = (long)x * Nt + (t + 1) % Nt;      /* RightPB[2n]   */
            const long nx = (long)((x + 1) % Nx) * Nt + t;    /* RightPB[2n+1] */
            cplx SR0 = C(t == Nt - 1 ? -1.0 : 1.0, 0.0), SR1 = C(1.0, 0.0);
            cplx U = ld(U0, n), V = ld(U1, n);
            cplx L0 = ld(l0, n), L1 = ld(l1, n), R0 = ld(r0, n), R1 = ld(r1, n);
            /* mu = 0 */
            cplx P = cmul(cmul(cmul(U, SR0), cconj(csub(L0, L1))),
                          csub(ld(r0, nt), ld(r1, nt)));
            cplx Q = cmul(cmul(cmul(cconj(U), SR0), cconj(cadd(ld(l0, nt), ld(l1, nt)))),
                          cadd(R0, R1));
            F0[n] = csub(P, Q).im;
            /* mu = 1 */
            P = cmul(cmul(cmul(V, SR1), csub(cconj(L0), cmul(I_num, cconj(L1)))),
                     cadd(ld(r0, nx), cmul(I_num, ld(r1, nx))));
            Q = cmul(cmul(cmul(cconj(V), SR1),
                          cadd(cconj(ld(l0, nx)), cmul(I_num, cconj(ld(l1, nx))))),
                     cadd(cneg(R0), cmul(I_num, R1)));
            F1[n] = cadd(P, Q).im;
        }
    }
}

void oracle_dot(long S, const double *x0, const double *x1, const double *y0,
                const double *y1, double *out) {
    cplx z = C(0.0, 0.0);
    for (long n = 0; n < S; n++) {
        z = cadd(z, cmul(ld(x0, n), cconj(ld(y0, n))));
        z = cadd(z, cmul(ld(x1, n), cconj(ld(y1, n))));
    }
    out[0] = z.re;
    out[1] = z.im;
}

int oracle_cg(int Nx, int Nt, const double *U0, const double *U1,
              const double *phi0, const double *phi1, double *x0, double *x1,
              double m0, double tol, int max_iter, int *iters, double *err_out) {
    /* src/conjugate_gradient.cpp:4-66 */
    const long S = (long)Nx * Nt;
    double *buf = (double *)calloc((size_t)(10 * 2 * S), sizeof(double));
    double *r0 = buf, *r1 = r0 + 2 * S, *d0 = r1 + 2 * S, *d1 = d0 + 2 * S;
    double *A0 = d1 + 2 * S, *A1 = A0 + 2 * S, *T0 = A1 + 2 * S, *T1 = T0 + 2 * S;
    double z[2];
    int k = 0, conv = 0;
    double err = 0.0, err_sqr;
    for (long i = 0; i < 2 * S; i++) { x0[i] = phi0[i]; x1[i] = phi1[i]; }   /* x = phi */
    oracle_ddag(Nx, Nt, U0, U1, x0, x1, T0, T1, A0, A1, m0);
    for (long n = 0; n < S; n++) {
        st(r0, n, csub(ld(phi0, n), ld(A0, n)));
        st(r1, n, csub(ld(phi1, n), ld(A1, n)));
    }
    for (long i = 0; i < 2 * S; i++) { d0[i] = r0[i]; d1[i] = r1[i]; }
    oracle_dot(S, r0, r1, r0, r1, z);
    cplx rn = C(z[0], z[1]);
    oracle_dot(S, phi0, phi1, phi0, phi1, z);
    const double phi_norm2 = sqrt(z[0]);
    while (k < max_iter) {
        oracle_ddag(Nx, Nt, U0, U1, d0, d1, T0, T1, A0, A1, m0);
        oracle_dot(S, d0, d1, A0, A1, z);
        cplx alpha;
        oracle_cdiv(rn.re, rn.im, z[0], z[1], &alpha.re, &alpha.im);
        for (long n = 0; n < S; n++) {
            st(x0, n, cadd(ld(x0, n), cmul(alpha, ld(d0, n))));
            st(x1, n, cadd(ld(x1, n), cmul(alpha, ld(d1, n))));
            st(r0, n, csub(ld(r0, n), cmul(alpha, ld(A0, n))));
            st(r1, n, csub(ld(r1, n), cmul(alpha, ld(A1, n))));
        }
        oracle_dot(S, r0, r1, r0, r1, z);
        err_sqr = z[0];
        err = sqrt(err_sqr);
        if (err < tol * phi_norm2) { conv = 1; k++; break; }
        cplx beta;
        oracle_cdiv(err_sqr, 0.0, rn.re, rn.im, &beta.re, &beta.im);
        for (long n = 0; n < S; n++) {
            st(d0, n, cadd(cmul(ld(d0, n), beta), ld(r0, n)));
            st(d1, n, cadd(cmul(ld(d1, n), beta), ld(r1, n)));
        }
        rn = C(err_sqr, 0.0);
        k++;
    }
    free(buf);
    *iters = k;
    *err_out = err;
    return conv;
}

/* ===================== gauge field / molecular dynamics =====================
 * the rest of the MD force step and the HMC
 * Hamiltonian, restated from src/gauge_conf.cpp and src/hmc.cpp in the
 * reference's evaluation order (single domain; the reference's MPI variants
 * compute the same expressions with halo values, bitwise equal). */
#include <complex.h>
#include <float.h>

/* U_01(n) = U_0(n) U_1(n+0) U*_0(n+1) U*_1(n), src/gauge_conf.cpp:45-49. */
static cplx plaq_site(int Nx, int Nt, const double *U0, const double *U1, int x, int t) {
    const long n = (long)x * Nt + t;
    const long nt = (long)x * Nt + (t + 1) % Nt;     /* RightPB[2n]   */
    const long nx = (long)((x + 1) % Nx) * Nt + t;   /* RightPB[2n+1] */
    return cmul(cmul(cmul(ld(U0, n), ld(U1, nt)), cconj(ld(U0, nx))), cconj(ld(U1, n)));
}

void oracle_plaquette(int Nx, int Nt, const double *U0, const double *U1, double *P) {
    for (int x = 0; x < Nx; x++)
        for (int t = 0; t < Nt; t++) st(P, (long)x * Nt + t, plaq_site(Nx, Nt, U0, U1, x, t));
}

void oracle_plaquette_sums(int Nx, int Nt, const double *U0, const double *U1, double beta,
                           double *sp, double *action) {
    /* MeasureSp_HMC (src/gauge_conf.cpp:430-440) and Compute_gaugeAction
     * (:444-453): sequential sums over n. */
    double s = 0.0, a = 0.0;
    for (int x = 0; x < Nx; x++)
        for (int t = 0; t < Nt; t++) {
            const cplx p = plaq_site(Nx, Nt, U0, U1, x, t);
            s += p.re;
            a += beta * (1.0 - p.re);   /* beta * real(1.0 - P) */
        }
    *sp = s;
    *action = a;
}

void oracle_staples(int Nx, int Nt, const double *U0, const double *U1, double *S0, double *S1) {
    /* Compute_Staple, src/gauge_conf.cpp:95-125 (size == 1 branch). */
    for (int x = 0; x < Nx; x++)
        for (int t = 0; t < Nt; t++) {
            const long n = (long)x * Nt + t;
            const int xp = (x + 1) % Nx, xm = (x - 1 + Nx) % Nx;
            const int tp = (t + 1) % Nt, tm = (t - 1 + Nt) % Nt;
            const long x1 = (long)xp * Nt + t, x_1 = (long)xm * Nt + t;
            const long t1 = (long)x * Nt + tp, t_1 = (long)x * Nt + tm;
            const long x_1_t1 = (long)xm * Nt + tp, x1_t_1 = (long)xp * Nt + tm;
            /* mu = 0: U_1(n) U_0(n+1) U*_1(n+0) + U*_1(n-1) U_0(n-1) U_1(n-1+0) */
            st(S0, n, cadd(cmul(cmul(ld(U1, n), ld(U0, x1)), cconj(ld(U1, t1))),
                           cmul(cmul(cconj(ld(U1, x_1)), ld(U0, x_1)), ld(U1, x_1_t1))));
            /* mu = 1: U_0(n) U_1(n+0) U*_0(n+1) + U*_0(n-0) U_1(n-0) U_0(n+1-0) */
            st(S1, n, cadd(cmul(cmul(ld(U0, n), ld(U1, t1)), cconj(ld(U0, x1))),
                           cmul(cmul(cconj(ld(U0, t_1)), ld(U1, t_1)), ld(U0, x1_t_1))));
        }
}

void oracle_gauge_force(int Nx, int Nt, const double *U0, const double *U1, double beta,
                        double *F0, double *F1) {
    /* HMC::Force_G, src/hmc.cpp:31-40: F += -beta Im(U conj(staple)). */
    const long S = (long)Nx * Nt;
    double *St = (double *)malloc(sizeof(double) * 4 * S);
    oracle_staples(Nx, Nt, U0, U1, St, St + 2 * S);
    for (long n = 0; n < S; n++) {
        F0[n] += -beta * cmul(ld(U0, n), cconj(ld(St, n))).im;
        F1[n] += -beta * cmul(ld(U1, n), cconj(ld(St + 2 * S, n))).im;
    }
    free(St);
}

int oracle_md_force(int Nx, int Nt, const double *U0, const double *U1, const double *phi0,
                    const double *phi1, double m0, double beta, double tol, int max_iter,
                    double *F0, double *F1, int *iters) {
    /* HMC::Force, src/hmc.cpp:44-60: psi = (DD^dag)^-1 phi (x0 = phi),
     * F = phi_dag_partialD_phi(U, psi, D^dag psi) + gauge force. The
     * ill-conditioned-conf save on CG failure is not restated. */
    const long S = (long)Nx * Nt;
    double *buf = (double *)malloc(sizeof(double) * 8 * S);
    double *ps0 = buf, *ps1 = buf + 2 * S, *T0 = buf + 4 * S, *T1 = buf + 6 * S;
    double err;
    const int conv = oracle_cg(Nx, Nt, U0, U1, phi0, phi1, ps0, ps1, m0, tol, max_iter, iters, &err);
    oracle_dirac(Nx, Nt, U0, U1, ps0, ps1, T0, T1, m0, 1);
    oracle_force(Nx, Nt, U0, U1, ps0, ps1, T0, T1, F0, F1);
    oracle_gauge_force(Nx, Nt, U0, U1, beta, F0, F1);
    free(buf);
    return conv;
}

/* U *= exp(i coef P) with std::exp(complex) = glibc cexp of (+-0, coef*P):
 * (cos y, sin y) for |y| > DBL_MIN, (1, y) below (s_cexp_template.c). */
static void link_update(long S, double *U, const double *P, double coef) {
    for (long n = 0; n < S; n++) {
        const double complex w = cexp(CMPLX(0.0, coef * P[n]));
        st(U, n, cmul(ld(U, n), C(creal(w), cimag(w))));
    }
}

int oracle_leapfrog(int Nx, int Nt, double *U0, double *U1, double *P0, double *P1,
                    const double *phi0, const double *phi1, double m0, double beta, double tau,
                    int md_steps, double tol, int max_iter, long *cg_iters) {
    /* HMC::Leapfrog, src/hmc.cpp:63-101, on the copies (U, P updated in place),
     * including its loop bound: forces are evaluated md_steps - 1 times. */
    const long S = (long)Nx * Nt;
    const double eps = tau / (md_steps * 1.0);
    double *F = (double *)malloc(sizeof(double) * 2 * S);
    int ok = 1, it;
    long total = 0;
    link_update(S, U0, P0, 0.5 * eps);
    link_update(S, U1, P1, 0.5 * eps);
    ok &= oracle_md_force(Nx, Nt, U0, U1, phi0, phi1, m0, beta, tol, max_iter, F, F + S, &it);
    total += it;
    for (int step = 1; step < md_steps - 1; step++) {
        for (long n = 0; n < S; n++) {
            P0[n] += eps * F[n];
            P1[n] += eps * F[S + n];
        }
        link_update(S, U0, P0, eps);
        link_update(S, U1, P1, eps);
        ok &= oracle_md_force(Nx, Nt, U0, U1, phi0, phi1, m0, beta, tol, max_iter, F, F + S, &it);
        total += it;
    }
    for (long n = 0; n < S; n++) {
        P0[n] += eps * F[n];
        P1[n] += eps * F[S + n];
    }
    link_update(S, U0, P0, 0.5 * eps);
    link_update(S, U1, P1, 0.5 * eps);
    free(F);
    *cg_iters = total;
    return ok;
}

double oracle_hamiltonian(int Nx, int Nt, const double *U0, const double *U1, const double *P0,
                          const double *P1, const double *phi0, const double *phi1, double m0,
                          double beta, double tol, int max_iter, int *iters) {
    /* HMC::Hamiltonian + HMC::Action, src/hmc.cpp:104-148:
     * H = sum 0.5 Pi^2 + (beta sum Re(1 - U_01) + Re dot((DD^dag)^-1 phi, phi)). */
    const long S = (long)Nx * Nt;
    double K = 0.0;
    for (long n = 0; n < S; n++) {
        K += 0.5 * P0[n] * P0[n];
        K += 0.5 * P1[n] * P1[n];
    }
    double sp, action, err, z[2];
    oracle_plaquette_sums(Nx, Nt, U0, U1, beta, &sp, &action);
    double *x = (double *)malloc(sizeof(double) * 4 * S);
    oracle_cg(Nx, Nt, U0, U1, phi0, phi1, x, x + 2 * S, m0, tol, max_iter, iters, &err);
    oracle_dot(S, x, x + 2 * S, phi0, phi1, z);
    free(x);
    action += z[0];
    return K + action;
}
