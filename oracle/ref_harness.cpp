// ref_harness.cpp -- TEST INFRASTRUCTURE ONLY (never shipped in the product).
//
// Drives the UNMODIFIED reference sources (compiled in place from
// /root/reference/src by oracle/Makefile, output only into oracle/_ref/) on
// fixed inputs, to produce golden vectors and a CPU timing baseline.
// Setup mirrors src/main.cpp:13-78 (MPI_Init -> initializeMPI ->
// allocate_lattice_arrays -> periodic_boundary); the lattice size is the
// reference's compile-time NS/NT (-DCONFIG_H -DNS=.. -DNT=..).
//
// Modes
//   fixture <dir> <ranks_x> <ranks_t> <m0> <tol> <max_iter>
//       reads <dir>/U.bin psi.bin chi.bin (global fields, two planes of
//       interleaved complex<double>, n = x*Nt + t), writes ref_Dpsi.bin,
//       ref_Ddagchi.bin, ref_DDdagpsi.bin, ref_force.bin (psi, chi),
//       ref_cgx.bin (CG on phi = psi) and prints one JSON line.
//   gen <dir> <seed_U> <sigma> <seed_psi> <seed_chi>
//       writes <dir>/U.bin psi.bin chi.bin from the synthetic generator
//       (sm_fields.h) for the compiled-in lattice (single process).
//   bench <ranks_x> <ranks_t> <seed_U> <sigma> <seed_psi> <m0> <napply> <ncg>
//       generates the synthetic fields per rank (sm_fields.h), times napply
//       D_phi applies and ncg CG iterations (tol = 0), prints one JSON line.
//   conf <dir> <ranks_x> <ranks_t>
//       reads U.bin, stores it with the reference's SaveConf into
//       <dir>/ref_conf.ctxt (src/gauge_conf.cpp:378-423: MPI_Gatherv to rank 0,
//       28-byte records), reads that file back with GaugeConf::readBinary
//       (:495-546, MPI_Scatterv) and writes the field it read as ref_conf_read.bin.
//   md <dir> <ranks_x> <ranks_t> <m0> <beta> <tau> <md_steps> <tol> <max_iter>
//       reads U.bin, chi.bin and P.bin (momenta: two real planes) and runs the
//       reference's gauge / molecular-dynamics code on them: plaquette field,
//       Sp, gauge action, staples, Force_G alone, Force (fermion + gauge) at
//       U, Hamiltonian(U, P, phi = D chi), Leapfrog(phi) -> (U', P') and
//       Hamiltonian(U', P', phi). HMC's members are private, so hmc.h is
//       included with `private` mapped to `public` (this TU only; the class
//       layout is unchanged).
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iomanip>
#include <iostream>
#include <random>
#include <sstream>
#include <string>
#include <vector>

#include "conjugate_gradient.h"
#include "gauge_conf.h"
#include "mpi_setup.h"
#include "sm_fields.h"
#define private public
#include "hmc.h"
#undef private

static long g_ddag_calls = 0;
extern "C" void __real__Z14D_D_dagger_phiRK6spinorS1_RS_RKd(const spinor &, const spinor &,
                                                             spinor &, const double &);
// Counts D_D_dagger_phi calls made by conjugate_gradient (linked with
// -Wl,--wrap=_Z14D_D_dagger_phiRK6spinorS1_RS_RKd): CG iterations = calls - 1.
extern "C" void __wrap__Z14D_D_dagger_phiRK6spinorS1_RS_RKd(const spinor &U, const spinor &phi,
                                                             spinor &Dphi, const double &m0) {
    g_ddag_calls++;
    __real__Z14D_D_dagger_phiRK6spinorS1_RS_RKd(U, phi, Dphi, m0);
}

static void setup(int rx, int rt) {
    MPI_Comm_size(MPI_COMM_WORLD, &mpi::size);
    MPI_Comm_rank(MPI_COMM_WORLD, &mpi::rank);
    mpi::ranks_x = rx;
    mpi::ranks_t = rt;
    initializeMPI();
    allocate_lattice_arrays();
    periodic_boundary();
    // The reference's scratch globals are default-sized to the full lattice
    // on every rank (src/variables.cpp:68-69, include/variables.h:59). The
    // operators only touch maxSize elements of them, so shrink them to the
    // rank's block: 8192^2 on 8 ranks otherwise holds 32 GiB of scratch.
    DTEMP = spinor(mpi::maxSize);
    TEMP = spinor(mpi::maxSize);
}

static int x_begin() { return mpi::coords[0] * mpi::width_x; }
static int t_begin() { return mpi::coords[1] * mpi::width_t; }

// Read this rank's block of a global two-plane real field (re_field).
static bool read_block_real(const std::string &path, re_field &s) {
    FILE *f = fopen(path.c_str(), "rb");
    if (!f) return false;
    std::vector<double> g((size_t)2 * LV::Ntot);
    size_t got = fread(g.data(), sizeof(double), g.size(), f);
    fclose(f);
    if (got != g.size()) return false;
    for (int x = 0; x < mpi::width_x; x++)
        for (int t = 0; t < mpi::width_t; t++) {
            long ng = (long)(x_begin() + x) * LV::Nt + t_begin() + t;
            int n = x * mpi::width_t + t;
            s.mu0[n] = g[ng];
            s.mu1[n] = g[LV::Ntot + ng];
        }
    return true;
}

// Read this rank's block of a global two-plane complex field.
static bool read_block(const std::string &path, spinor &s) {
    FILE *f = fopen(path.c_str(), "rb");
    if (!f) return false;
    std::vector<double> g((size_t)4 * LV::Ntot);
    size_t got = fread(g.data(), sizeof(double), g.size(), f);
    fclose(f);
    if (got != g.size()) return false;
    for (int x = 0; x < mpi::width_x; x++)
        for (int t = 0; t < mpi::width_t; t++) {
            long ng = (long)(x_begin() + x) * LV::Nt + t_begin() + t;
            int n = x * mpi::width_t + t;
            s.mu0[n] = c_double(g[2 * ng], g[2 * ng + 1]);
            s.mu1[n] = c_double(g[2 * LV::Ntot + 2 * ng], g[2 * LV::Ntot + 2 * ng + 1]);
        }
    return true;
}

// Gather per-rank blocks of (plane0, plane1) with `ncomp` doubles per site to
// rank 0 and write the global field.
static void write_global(const std::string &path, const double *p0, const double *p1, int ncomp) {
    const int blk = mpi::maxSize * ncomp;
    std::vector<double> mine((size_t)2 * blk);
    memcpy(mine.data(), p0, sizeof(double) * blk);
    memcpy(mine.data() + blk, p1, sizeof(double) * blk);
    std::vector<double> all;
    std::vector<int> coords((size_t)2 * mpi::size);
    int my[2] = {mpi::coords[0], mpi::coords[1]};
    MPI_Gather(my, 2, MPI_INT, coords.data(), 2, MPI_INT, 0, MPI_COMM_WORLD);
    if (mpi::rank == 0) all.resize((size_t)2 * blk * mpi::size);
    MPI_Gather(mine.data(), 2 * blk, MPI_DOUBLE, all.data(), 2 * blk, MPI_DOUBLE, 0, MPI_COMM_WORLD);
    if (mpi::rank != 0) return;
    std::vector<double> g((size_t)2 * ncomp * LV::Ntot);
    for (int r = 0; r < mpi::size; r++) {
        const double *b = all.data() + (size_t)2 * blk * r;
        int xb = coords[2 * r] * mpi::width_x, tb = coords[2 * r + 1] * mpi::width_t;
        for (int x = 0; x < mpi::width_x; x++)
            for (int t = 0; t < mpi::width_t; t++) {
                long ng = (long)(xb + x) * LV::Nt + tb + t;
                int n = x * mpi::width_t + t;
                for (int c = 0; c < ncomp; c++) {
                    g[(size_t)ncomp * ng + c] = b[(size_t)ncomp * n + c];
                    g[(size_t)ncomp * LV::Ntot + (size_t)ncomp * ng + c] = b[blk + (size_t)ncomp * n + c];
                }
            }
    }
    FILE *f = fopen(path.c_str(), "wb");
    fwrite(g.data(), sizeof(double), g.size(), f);
    fclose(f);
}

static void write_spinor(const std::string &path, const spinor &s) {
    write_global(path, reinterpret_cast<const double *>(s.mu0), reinterpret_cast<const double *>(s.mu1), 2);
}

static int run_fixture(const std::string &dir, double m0, double tol, int max_iter) {
    spinor U(mpi::maxSize), psi(mpi::maxSize), chi(mpi::maxSize);
    int ok = read_block(dir + "/U.bin", U) && read_block(dir + "/psi.bin", psi) &&
             read_block(dir + "/chi.bin", chi);
    if (!ok) {
        if (mpi::rank == 0) fprintf(stderr, "cannot read inputs in %s\n", dir.c_str());
        return 1;
    }
    spinor Dpsi(mpi::maxSize), Ddchi(mpi::maxSize), DDpsi(mpi::maxSize), x(mpi::maxSize);
    D_phi(U, psi, Dpsi, m0);
    D_dagger_phi(U, chi, Ddchi, m0);
    D_D_dagger_phi(U, psi, DDpsi, m0);
    re_field F = phi_dag_partialD_phi(U, psi, chi);
    c_double z1 = dot(chi, Dpsi), z2 = dot(Ddchi, psi);
    CG::tol = tol;
    CG::max_iter = max_iter;
    long before = g_ddag_calls;
    double t0 = MPI_Wtime();
    int conv = conjugate_gradient(U, psi, x, m0);
    double t1 = MPI_Wtime();
    long cg_calls = g_ddag_calls - before;
    // final true residual |psi - DD^dag x| / |psi|
    spinor Ax(mpi::maxSize), res(mpi::maxSize);
    D_D_dagger_phi(U, x, Ax, m0);
    for (int n = 0; n < mpi::maxSize; n++) {
        res.mu0[n] = psi.mu0[n] - Ax.mu0[n];
        res.mu1[n] = psi.mu1[n] - Ax.mu1[n];
    }
    double rr = std::real(dot(res, res)), pp = std::real(dot(psi, psi));
    write_spinor(dir + "/ref_Dpsi.bin", Dpsi);
    write_spinor(dir + "/ref_Ddagchi.bin", Ddchi);
    write_spinor(dir + "/ref_DDdagpsi.bin", DDpsi);
    write_spinor(dir + "/ref_cgx.bin", x);
    write_global(dir + "/ref_force.bin", F.mu0, F.mu1, 1);
    if (mpi::rank == 0) {
        printf("{\"Nx\": %d, \"Nt\": %d, \"ranks_x\": %d, \"ranks_t\": %d, \"m0\": %.17g, "
               "\"cg_converged\": %d, \"cg_iters\": %ld, \"cg_true_relres\": %.17g, "
               "\"cg_seconds\": %.6f, "
               "\"dot_chi_Dpsi\": [%.17g, %.17g], \"dot_Ddagchi_psi\": [%.17g, %.17g]}\n",
               LV::Nx, LV::Nt, mpi::ranks_x, mpi::ranks_t, m0, conv, cg_calls - 1,
               sqrt(rr / pp), t1 - t0, z1.real(), z1.imag(), z2.real(), z2.imag());
    }
    return 0;
}

static int run_md(const std::string &dir, double m0, double beta, double tau, int md_steps,
                  double tol, int max_iter) {
    GaugeConf G;
    spinor chi(mpi::maxSize);
    re_field P(mpi::maxSize);
    if (!(read_block(dir + "/U.bin", G.Conf) && read_block(dir + "/chi.bin", chi) &&
          read_block_real(dir + "/P.bin", P))) {
        if (mpi::rank == 0) fprintf(stderr, "cannot read md inputs in %s\n", dir.c_str());
        return 1;
    }
    CG::tol = tol;
    CG::max_iter = max_iter;
    G.Compute_Plaquette01();
    const double sp = G.MeasureSp_HMC(), gS = G.Compute_gaugeAction(beta);
    write_global(dir + "/ref_plaq.bin", reinterpret_cast<const double *>(G.Plaquette01),
                 reinterpret_cast<const double *>(G.Plaquette01), 2);
    G.Compute_Staple();
    write_spinor(dir + "/ref_staple.bin", G.Staples);
    HMC h(G, md_steps, tau, 0, 1, 0, beta, LV::Nx, LV::Nt, m0, 0);
    h.PConf = P;
    spinor phi(mpi::maxSize);
    D_phi(G.Conf, chi, phi, m0);
    write_spinor(dir + "/ref_phi.bin", phi);
    // gauge force alone (Forces zeroed first)
    for (int n = 0; n < mpi::maxSize; n++) h.Forces.mu0[n] = h.Forces.mu1[n] = 0.0;
    h.Force_G(h.GConf);
    write_global(dir + "/ref_gforce.bin", h.Forces.mu0, h.Forces.mu1, 1);
    long c0 = g_ddag_calls;
    h.Force(h.GConf, phi);
    long force_iters = g_ddag_calls - c0 - 1;
    write_global(dir + "/ref_mdforce.bin", h.Forces.mu0, h.Forces.mu1, 1);
    const double H0 = h.Hamiltonian(h.GConf, h.PConf, phi);
    c0 = g_ddag_calls;
    h.Leapfrog(phi);
    long lf_calls = g_ddag_calls - c0;
    write_spinor(dir + "/ref_U1.bin", h.GConf_copy.Conf);
    write_global(dir + "/ref_P1.bin", h.PConf_copy.mu0, h.PConf_copy.mu1, 1);
    const double H1 = h.Hamiltonian(h.GConf_copy, h.PConf_copy, phi);
    if (mpi::rank == 0)
        printf("{\"Nx\": %d, \"Nt\": %d, \"ranks_x\": %d, \"ranks_t\": %d, \"m0\": %.17g, "
               "\"beta\": %.17g, \"tau\": %.17g, \"md_steps\": %d, \"sp\": %.17g, "
               "\"gauge_action\": %.17g, \"force_cg_iters\": %ld, \"leapfrog_ddag_calls\": %ld, "
               "\"H0\": %.17g, \"H1\": %.17g, \"dH\": %.17g, \"cg_convergence\": %d}\n",
               LV::Nx, LV::Nt, mpi::ranks_x, mpi::ranks_t, m0, beta, tau, md_steps, sp, gS,
               force_iters, lf_calls, H0, H1, H1 - H0, h.CG_convergence);
    return 0;
}

static int run_conf(const std::string &dir) {
    GaugeConf G;
    if (!read_block(dir + "/U.bin", G.Conf)) {
        if (mpi::rank == 0) fprintf(stderr, "cannot read U in %s\n", dir.c_str());
        return 1;
    }
    SaveConf(G, dir + "/ref_conf.ctxt");
    MPI_Barrier(MPI_COMM_WORLD);
    GaugeConf H;
    H.readBinary(dir + "/ref_conf.ctxt");
    write_spinor(dir + "/ref_conf_read.bin", H.Conf);
    return 0;
}

static int run_bench(unsigned long long seedU, double sigma, unsigned long long seedP, double m0,
                     int napply, int ncg) {
    spinor U(mpi::maxSize), psi(mpi::maxSize), out(mpi::maxSize), x(mpi::maxSize);
    // Per-rank block of the same global synthetic fields the GPU bench uses.
    {
        std::vector<double> u0(2 * (size_t)mpi::maxSize), u1(u0.size()), p0(u0.size()), p1(u0.size());
        sm_fields_fill_gauge(seedU, sigma, LV::Nt, x_begin(), mpi::width_x, t_begin(), mpi::width_t,
                             u0.data(), u1.data());
        sm_fields_fill_spinor(seedP, LV::Nt, x_begin(), mpi::width_x, t_begin(), mpi::width_t,
                              p0.data(), p1.data());
        for (int n = 0; n < mpi::maxSize; n++) {
            U.mu0[n] = c_double(u0[2 * n], u0[2 * n + 1]);
            U.mu1[n] = c_double(u1[2 * n], u1[2 * n + 1]);
            psi.mu0[n] = c_double(p0[2 * n], p0[2 * n + 1]);
            psi.mu1[n] = c_double(p1[2 * n], p1[2 * n + 1]);
        }
    }
    MPI_Barrier(MPI_COMM_WORLD);
    double t0 = MPI_Wtime();
    for (int i = 0; i < napply; i++) D_phi(U, psi, out, m0);
    MPI_Barrier(MPI_COMM_WORLD);
    double t1 = MPI_Wtime();
    CG::tol = 0.0;
    CG::max_iter = ncg;
    long before = g_ddag_calls;
    MPI_Barrier(MPI_COMM_WORLD);
    double t2 = MPI_Wtime();
    conjugate_gradient(U, psi, x, m0);
    MPI_Barrier(MPI_COMM_WORLD);
    double t3 = MPI_Wtime();
    long it = g_ddag_calls - before - 1;
    if (mpi::rank == 0) {
        double sites = (double)LV::Ntot;
        double dt_apply = napply ? (t1 - t0) / napply : 0.0;
        printf("{\"Nx\": %d, \"Nt\": %d, \"ranks\": %d, \"ranks_x\": %d, \"ranks_t\": %d, "
               "\"apply_s\": %.6g, \"apply_GBps\": %.6g, \"cg_iters\": %ld, \"cg_s\": %.6g, "
               "\"cg_it_per_s\": %.6g}\n",
               LV::Nx, LV::Nt, mpi::size, mpi::ranks_x, mpi::ranks_t, dt_apply,
               napply ? 96.0 * sites / dt_apply / 1e9 : 0.0, it, t3 - t2,
               it > 0 ? it / (t3 - t2) : 0.0);
    }
    return 0;
}

static int run_gen(const std::string &dir, unsigned long long seedU, double sigma,
                   unsigned long long seedP, unsigned long long seedC) {
    const size_t S = (size_t)LV::Ntot;
    std::vector<double> a(4 * S);
    FILE *f;
    sm_fields_fill_gauge(seedU, sigma, LV::Nt, 0, LV::Nx, 0, LV::Nt, a.data(), a.data() + 2 * S);
    if (!(f = fopen((dir + "/U.bin").c_str(), "wb"))) return 1;
    fwrite(a.data(), sizeof(double), a.size(), f);
    fclose(f);
    sm_fields_fill_spinor(seedP, LV::Nt, 0, LV::Nx, 0, LV::Nt, a.data(), a.data() + 2 * S);
    if (!(f = fopen((dir + "/psi.bin").c_str(), "wb"))) return 1;
    fwrite(a.data(), sizeof(double), a.size(), f);
    fclose(f);
    sm_fields_fill_spinor(seedC, LV::Nt, 0, LV::Nx, 0, LV::Nt, a.data(), a.data() + 2 * S);
    if (!(f = fopen((dir + "/chi.bin").c_str(), "wb"))) return 1;
    fwrite(a.data(), sizeof(double), a.size(), f);
    fclose(f);
    return 0;
}

int main(int argc, char **argv) {
    MPI_Init(&argc, &argv);
    int rc = 2;
    if (argc >= 7 && !strcmp(argv[1], "gen")) {
        rc = run_gen(argv[2], strtoull(argv[3], 0, 10), atof(argv[4]), strtoull(argv[5], 0, 10),
                     strtoull(argv[6], 0, 10));
    } else if (argc >= 8 && !strcmp(argv[1], "fixture")) {
        setup(atoi(argv[3]), atoi(argv[4]));
        rc = run_fixture(argv[2], atof(argv[5]), atof(argv[6]), atoi(argv[7]));
    } else if (argc >= 3 && !strcmp(argv[1], "jk")) {
        // jk <bin> v1 v2 ...: the reference's Jackknife_error and mean
        std::vector<double> v;
        for (int i = 3; i < argc; i++) v.push_back(strtod(argv[i], nullptr));
        printf("%.17g %.17g\n", Jackknife_error(v, atoi(argv[2])), mean(v));
        rc = 0;
    } else if (argc >= 11 && !strcmp(argv[1], "md")) {
        setup(atoi(argv[3]), atoi(argv[4]));
        rc = run_md(argv[2], atof(argv[5]), atof(argv[6]), atof(argv[7]), atoi(argv[8]), atof(argv[9]),
                    atoi(argv[10]));
    } else if (argc >= 5 && !strcmp(argv[1], "conf")) {
        setup(atoi(argv[3]), atoi(argv[4]));
        rc = run_conf(argv[2]);
    } else if (argc >= 10 && !strcmp(argv[1], "bench")) {
        setup(atoi(argv[2]), atoi(argv[3]));
        rc = run_bench(strtoull(argv[4], 0, 10), atof(argv[5]), strtoull(argv[6], 0, 10),
                       atof(argv[7]), atoi(argv[8]), atoi(argv[9]));
    } else {
        fprintf(stderr, "usage: gen <dir> seedU sigma seedP seedC | fixture <dir> rx rt m0 tol max_iter | bench rx rt seedU sigma seedP m0 napply ncg | md <dir> rx rt m0 beta tau md_steps tol max_iter | conf <dir> rx rt\n");
    }
    MPI_Finalize();
    return rc;
}
