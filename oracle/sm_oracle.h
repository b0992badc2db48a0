/*
 * sm_oracle.h -- CPU ORACLE (test infrastructure only).
 *
 * A plain-C restatement of the reference's hot path, used ONLY by tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg as the checker.
 * Nothing in the product (schwingermodel_amd/, include/sm_hip.h) links or
 * calls this code.
 *
 * Reference: Fabian2598/SchwingerModel (read-only at /root/reference).
 *   D_phi                 src/dirac_operator.cpp:24-44   (eq. 34 of HMC_doc.pdf)
 *   D_dagger_phi          src/dirac_operator.cpp:247-268 (eqs. 35-36)
 *   D_D_dagger_phi        src/dirac_operator.cpp:477-480
 *   phi_dag_partialD_phi  src/dirac_operator.cpp:486-506 (eqs. 37-38)
 *   conjugate_gradient    src/conjugate_gradient.cpp:4-66
 *   dot                   include/variables.h:181-192
 *   periodic_boundary     include/dirac_operator.h:35-62 (signs / neighbours)
 *   Compute_Plaquette01   src/gauge_conf.cpp:41-85; MeasureSp_HMC :430-440;
 *   Compute_gaugeAction   :444-453; Compute_Staple :89-373
 *   HMC::Force_G / Force  src/hmc.cpp:31-60; Leapfrog :63-101;
 *   HMC::Action / Hamiltonian :104-148
 *
 * Parity is PINNED: tests/test_oracle_golden.py checks every function here
 * bit-for-bit against fixtures produced by the unmodified reference sources
 * (oracle/ref_harness.cpp + oracle/Makefile, generator tests/golden/make_golden.py).
 *
 * Data layout = the reference's: a field is two planes (mu0, mu1) of
 * complex<double>, each plane S = Nx*Nt complex numbers stored as interleaved
 * (re, im) doubles, site index n = x*Nt + t (t fastest), src/variables.cpp:10-12.
 */
#ifndef SM_ORACLE_H
#define SM_ORACLE_H

#ifdef __cplusplus
extern "C" {
#endif

/* Wilson-Dirac apply on the full periodic lattice (single domain).
 * dagger = 0: D (src/dirac_operator.cpp:29-44); 1: D^dagger (:253-268). */
void oracle_dirac(int Nx, int Nt, const double *U0, const double *U1,
                  const double *in0, const double *in1, double *out0, double *out1,
                  double m0, int dagger);

/* Local (t-sharded) apply: this domain owns global t in [t0, t0+Wt) for all x.
 * lo_* hold psi / U_t at local t = -1 (one complex per x, per spin plane),
 * hi_* hold psi at local t = Wt. Passing NULL faces means the domain is the
 * whole t-range and wraps periodically (then Wt == Nt_global, t0 == 0). */
void oracle_dirac_local(int Nx, int Wt, int t0, int Nt_global,
                        const double *U0, const double *U1,
                        const double *in0, const double *in1,
                        const double *lo_psi0, const double *lo_psi1, const double *lo_U0,
                        const double *hi_psi0, const double *hi_psi1,
                        double *out0, double *out1, double m0, int dagger);

/* D D^dagger psi via a caller-provided scratch field (the reference's DTEMP). */
void oracle_ddag(int Nx, int Nt, const double *U0, const double *U1,
                 const double *in0, const double *in1, double *tmp0, double *tmp1,
                 double *out0, double *out1, double m0);

/* Fermion-force bilinear; F0, F1 are real planes of S doubles. */
void oracle_force(int Nx, int Nt, const double *U0, const double *U1,
                  const double *l0, const double *l1, const double *r0, const double *r1,
                  double *F0, double *F1);

/* dot(x, y) = sum_n x0 conj(y0) + x1 conj(y1), sequential order of
 * include/variables.h:185-188. out[0] = re, out[1] = im. */
void oracle_dot(long S, const double *x0, const double *x1, const double *y0,
                const double *y1, double *out);

/* libgcc (GCC 11) __divdc3: the complex division std::complex<double> uses. */
void oracle_cdiv(double a, double b, double c, double d, double *re, double *im);

/* CG on D D^dagger exactly as src/conjugate_gradient.cpp:4-66.
 * Returns 1 converged / 0 not. *iters = loop passes executed (DD^dagger
 * applications inside the loop); *err = final sqrt(Re<r,r>). */
int oracle_cg(int Nx, int Nt, const double *U0, const double *U1,
              const double *phi0, const double *phi1, double *x0, double *x1,
              double m0, double tol, int max_iter, int *iters, double *err);

/* Threaded D apply for the CPU-baseline timing (same arithmetic, rows split
 * over nthreads pthreads). */
void oracle_dirac_mt(int Nx, int Nt, const double *U0, const double *U1,
                     const double *in0, const double *in1, double *out0, double *out1,
                     double m0, int dagger, int nthreads);

/* ---- gauge field and molecular dynamics (single domain) ---- */
/* Per-site plaquette U_01(n); P is S complex (interleaved). */
void oracle_plaquette(int Nx, int Nt, const double *U0, const double *U1, double *P);
/* sp = sum Re U_01 (MeasureSp_HMC), action = sum beta Re(1 - U_01), sequential. */
void oracle_plaquette_sums(int Nx, int Nt, const double *U0, const double *U1, double beta,
                           double *sp, double *action);
/* Staples of both directions (Compute_Staple), S0/S1 complex planes. */
void oracle_staples(int Nx, int Nt, const double *U0, const double *U1, double *S0, double *S1);
/* F += -beta Im(U conj(staple)) (HMC::Force_G). */
void oracle_gauge_force(int Nx, int Nt, const double *U0, const double *U1, double beta,
                        double *F0, double *F1);
/* HMC::Force: CG solve, D^dag, fermion bilinear, gauge force. Returns CG convergence. */
int oracle_md_force(int Nx, int Nt, const double *U0, const double *U1, const double *phi0,
                    const double *phi1, double m0, double beta, double tol, int max_iter,
                    double *F0, double *F1, int *iters);
/* HMC::Leapfrog on (U, P) in place; returns 1 if every CG converged. */
int oracle_leapfrog(int Nx, int Nt, double *U0, double *U1, double *P0, double *P1,
                    const double *phi0, const double *phi1, double m0, double beta, double tau,
                    int md_steps, double tol, int max_iter, long *cg_iters);
/* HMC::Hamiltonian(U, P, phi). */
double oracle_hamiltonian(int Nx, int Nt, const double *U0, const double *U1, const double *P0,
                          const double *P1, const double *phi0, const double *phi1, double m0,
                          double beta, double tol, int max_iter, int *iters);

#ifdef __cplusplus
}
#endif
#endif
