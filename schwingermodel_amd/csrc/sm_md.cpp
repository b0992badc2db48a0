// sm_md.cpp -- gauge field, molecular dynamics and HMC entry points of
// libsm_hip.so (include/sm_hip.h).
//
// The reference's MD step (src/hmc.cpp) with every field resident on the
// device: the gauge field lives in sm_ctx::U (and a second buffer U_alt for
// the leapfrog copy, so a Metropolis reject is a pointer swap, not a copy),
// momenta and forces in Pmd / Fmd. The force step is one CG solve
// (sm_cg_dev), one D^dag apply, the fermion bilinear (sm_force_dev) and the
// staple kernel; the leapfrog interleaves it with the fused link/momentum
// update kernel. Global sums use the same deterministic partial + all-reduce
// path as the CG. Kernels: sm_gauge.hip.
#include <cmath>
#include <utility>

#include "sm_ctx.h"
#include "sm_fields.h"
#include "sm_internal.h"

using namespace sm;
using namespace sm_host;

namespace {

int ensure_md(sm_ctx *c) {
    if (c->U_alt) return SM_OK;
    const size_t fb = sizeof(double2) * 2 * (size_t)c->g.V, rb = sizeof(double) * 2 * (size_t)c->g.V;
    HIP_TRY(hipMalloc(&c->U_alt, fb));
    HIP_TRY(hipMalloc(&c->Pmd, rb));
    HIP_TRY(hipMalloc(&c->Fmd, rb));
    return SM_OK;
}

const double2 *ufaces(sm_ctx *c) { return !c->sharded() ? nullptr : face2_recv(c, 2); }

int check_params(const sm_hmc_params *p) {
    if (!p) return fail(SM_ERR_ARG, "null params");
    if (p->even_odd != 0 && p->even_odd != 1) return fail(SM_ERR_ARG, "even_odd must be 0 or 1");
    if (p->md_steps < 1 || p->cg_max_iter < 1 || !(p->tau > 0.0))
        return fail(SM_ERR_ARG, "bad HMC params md_steps=%d tau=%g cg_max_iter=%d", p->md_steps, p->tau,
                    p->cg_max_iter);
    return SM_OK;
}

// Global sum of `nparts` gauge-kernel partials -> host.
int gauge_sum(sm_ctx *c, int nparts, double2 *out) {
    TRY(global_sum(c, nparts, c->partials, 0));
    HIP_TRY(hipMemcpyAsync(c->h_sums, c->sums, sizeof(double2), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    *out = c->h_sums[0];
    return SM_OK;
}

int plaquette_sums(sm_ctx *c, double beta, double *sp, double *action, double2 *field) {
    launch_plaquette(c->stream, c->g, c->kshards(), c->U, ufaces(c), beta, field, c->partials);
    HIP_TRY(hipGetLastError());
    double2 s;
    TRY(gauge_sum(c, gauge_reduce_blocks(c->g), &s));
    *sp = s.x;
    *action = s.y;
    return SM_OK;
}

int upload_real_pair(sm_ctx *c, double *dst, const double *p0, const double *p1) {
    const size_t b = sizeof(double) * c->g.V;
    HIP_TRY(hipMemcpyAsync(dst, p0, b, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(dst + c->g.V, p1, b, hipMemcpyHostToDevice, c->stream));
    return SM_OK;
}

int download_real_pair(sm_ctx *c, const double *src, double *p0, double *p1) {
    const size_t b = sizeof(double) * c->g.V;
    HIP_TRY(hipMemcpyAsync(p0, src, b, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipMemcpyAsync(p1, src + c->g.V, b, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return SM_OK;
}

// Leapfrog half/full step: [P += eps F;] U *= exp(i coef P); refresh the
// ghost links the next stencil reads.
int md_step(sm_ctx *c, double *P, double eps, int do_p, double coef) {
    launch_md_update(c->stream, c->g, c->U, P, c->Fmd, eps, do_p, coef);
    HIP_TRY(hipGetLastError());
    return exchange_ghost_U(c);
}

}  // namespace

extern "C" {

int sm_download_gauge(sm_ctx *c, double *U0, double *U1) {
    TRY(check_ready(c));
    if (!U0 || !U1) return fail(SM_ERR_ARG, "null argument");
    HIP_TRY(hipSetDevice(c->device));
    return download_plane_pair(c, c->U, U0, U1);
}

int sm_fill_gauge_dev(sm_ctx *c, uint64_t seed, double sigma) {
    if (!c) return fail(SM_ERR_ARG, "null context");
    HIP_TRY(hipSetDevice(c->device));
    launch_draw_gauge(c->stream, c->g, seed, sigma, c->U);
    HIP_TRY(hipGetLastError());
    TRY(exchange_ghost_U(c));
    c->have_gauge = true;
    return SM_OK;
}

int sm_plaquette(sm_ctx *c, double beta, double *sp, double *gauge_action, double *plaq) {
    TRY(check_ready(c));
    if (!sp || !gauge_action) return fail(SM_ERR_ARG, "null argument");
    HIP_TRY(hipSetDevice(c->device));
    double2 *field = plaq ? c->field(F_OUT) : nullptr;
    TRY(plaquette_sums(c, beta, sp, gauge_action, field));
    if (plaq) {
        HIP_TRY(hipMemcpyAsync(plaq, field, sizeof(double2) * c->g.V, hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(hipStreamSynchronize(c->stream));
    }
    return SM_OK;
}

int sm_staples(sm_ctx *c, double *S0, double *S1) {
    TRY(check_ready(c));
    if (!S0 || !S1) return fail(SM_ERR_ARG, "null argument");
    HIP_TRY(hipSetDevice(c->device));
    double2 *S = c->field(F_OUT);
    launch_staple_force(c->stream, c->g, c->kshards(), c->U, ufaces(c), 0.0, nullptr, S);
    HIP_TRY(hipGetLastError());
    return download_plane_pair(c, S, S0, S1);
}

int sm_gauge_force(sm_ctx *c, double beta, double *F0, double *F1) {
    TRY(check_ready(c));
    if (!F0 || !F1) return fail(SM_ERR_ARG, "null argument");
    HIP_TRY(hipSetDevice(c->device));
    TRY(ensure_md(c));
    TRY(upload_real_pair(c, c->Fmd, F0, F1));
    launch_staple_force(c->stream, c->g, c->kshards(), c->U, ufaces(c), beta, c->Fmd, nullptr);
    HIP_TRY(hipGetLastError());
    return download_real_pair(c, c->Fmd, F0, F1);
}

int sm_md_force_dev(sm_ctx *c, const sm_hmc_params *p, const double *phi, double *F, sm_cg_result *res) {
    TRY(check_ready(c));
    TRY(check_params(p));
    if (!phi || !F || !res) return fail(SM_ERR_ARG, "null argument");
    if (p->even_odd) {
        TRY(eo_md_force(c, p, (const double2 *)phi, F, res));  // sm_eo.cpp
    } else {
        // HMC::Force, src/hmc.cpp:44-60
        double2 *psi = c->field(F_X), *T = c->field(F_RR);
        TRY(sm_cg_dev(c, phi, (double *)psi, p->m0, p->cg_tol, p->cg_max_iter, res));  // x0 = phi
        TRY(apply(c, psi, T, p->m0 + 2, 1, nullptr, nullptr, nullptr));                 // TEMP = D^dag psi
        TRY(sm_force_dev(c, (const double *)psi, (const double *)T, F));                 // fermion bilinear
    }
    launch_staple_force(c->stream, c->g, c->kshards(), c->U, ufaces(c), p->beta, F, nullptr);  // Force_G
    HIP_TRY(hipGetLastError());
    return SM_OK;
}

int sm_md_force(sm_ctx *c, const sm_hmc_params *p, const double *phi0, const double *phi1, double *F0,
                double *F1, sm_cg_result *res) {
    TRY(check_ready(c));
    if (!phi0 || !phi1 || !F0 || !F1) return fail(SM_ERR_ARG, "null argument");
    HIP_TRY(hipSetDevice(c->device));
    TRY(ensure_md(c));
    double2 *phi = c->field(F_PHI);
    TRY(upload_plane_pair(c, phi, phi0, phi1));
    TRY(sm_md_force_dev(c, p, (const double *)phi, c->Fmd, res));
    return download_real_pair(c, c->Fmd, F0, F1);
}

int sm_leapfrog_dev(sm_ctx *c, const sm_hmc_params *p, const double *phi, double *P, long *cg_iters,
                    int *cg_failures) {
    TRY(check_ready(c));
    TRY(check_params(p));
    if (!phi || !P) return fail(SM_ERR_ARG, "null argument");
    TRY(ensure_md(c));
    // HMC::Leapfrog, src/hmc.cpp:63-101 (including its loop bound: the force
    // is evaluated md_steps - 1 times and the trajectory is (md_steps-1)*eps)
    const double eps = p->tau / (p->md_steps * 1.0);
    long iters = 0;
    int fails = 0;
    sm_cg_result r;
    auto force = [&]() -> int {
        TRY(sm_md_force_dev(c, p, phi, c->Fmd, &r));
        iters += r.iterations;
        fails += r.converged ? 0 : 1;
        return SM_OK;
    };
    TRY(md_step(c, P, eps, 0, 0.5 * eps));
    TRY(force());
    for (int step = 1; step < p->md_steps - 1; step++) {
        TRY(md_step(c, P, eps, 1, eps));
        TRY(force());
    }
    TRY(md_step(c, P, eps, 1, 0.5 * eps));
    if (cg_iters) *cg_iters = iters;
    if (cg_failures) *cg_failures = fails;
    return SM_OK;
}

int sm_leapfrog(sm_ctx *c, const sm_hmc_params *p, const double *phi0, const double *phi1, double *P0,
                double *P1, long *cg_iters, int *cg_failures) {
    TRY(check_ready(c));
    if (!phi0 || !phi1 || !P0 || !P1) return fail(SM_ERR_ARG, "null argument");
    HIP_TRY(hipSetDevice(c->device));
    TRY(ensure_md(c));
    double2 *phi = c->field(F_PHI);
    TRY(upload_plane_pair(c, phi, phi0, phi1));
    TRY(upload_real_pair(c, c->Pmd, P0, P1));
    TRY(sm_leapfrog_dev(c, p, (const double *)phi, c->Pmd, cg_iters, cg_failures));
    return download_real_pair(c, c->Pmd, P0, P1);
}

int sm_hamiltonian_dev(sm_ctx *c, const sm_hmc_params *p, const double *phi, const double *P,
                       sm_hamiltonian_terms *out) {
    TRY(check_ready(c));
    TRY(check_params(p));
    if (!phi || !P || !out) return fail(SM_ERR_ARG, "null argument");
    // HMC::Hamiltonian + HMC::Action, src/hmc.cpp:104-148
    launch_kinetic(c->stream, c->g, P, c->partials);
    HIP_TRY(hipGetLastError());
    double2 k;
    TRY(gauge_sum(c, gauge_reduce_blocks(c->g), &k));
    double sp, action;
    TRY(plaquette_sums(c, p->beta, &sp, &action, nullptr));
    sm_cg_result r;
    double z[2] = {0.0, 0.0};
    if (p->even_odd) {
        TRY(eo_fermion_action(c, p, (const double2 *)phi, &z[0], &r));
    } else {
        double2 *x = c->field(F_X);   // the reference's TEMP
        TRY(sm_cg_dev(c, phi, (double *)x, p->m0, p->cg_tol, p->cg_max_iter, &r));
        TRY(sm_dot_dev(c, (const double *)x, phi, z));
    }
    out->kinetic = k.x;
    out->gauge_action = action;
    out->fermion = z[0];
    out->sp = sp;
    out->H = k.x + (action + z[0]);
    out->cg_iterations = r.iterations;
    out->cg_converged = r.converged;
    return SM_OK;
}

int sm_hamiltonian(sm_ctx *c, const sm_hmc_params *p, const double *phi0, const double *phi1, const double *P0,
                   const double *P1, sm_hamiltonian_terms *out) {
    TRY(check_ready(c));
    if (!phi0 || !phi1 || !P0 || !P1) return fail(SM_ERR_ARG, "null argument");
    HIP_TRY(hipSetDevice(c->device));
    TRY(ensure_md(c));
    double2 *phi = c->field(F_PHI);
    TRY(upload_plane_pair(c, phi, phi0, phi1));
    TRY(upload_real_pair(c, c->Pmd, P0, P1));
    return sm_hamiltonian_dev(c, p, (const double *)phi, c->Pmd, out);
}

int sm_quenched_trajectory(sm_ctx *c, const sm_hmc_params *p, uint64_t traj) {
    TRY(check_ready(c));
    TRY(check_params(p));
    HIP_TRY(hipSetDevice(c->device));
    TRY(ensure_md(c));
    // HMC::Leapfrog (src/hmc.cpp:63-101, its loop bound included) with
    // HMC::Force_G alone (:31-40): the fermion force is dropped, so no CG runs
    launch_draw_momenta(c->stream, c->g, sm_traj_seed(p->seed, traj), c->Pmd);  // RandomPI
    const double eps = p->tau / (p->md_steps * 1.0);
    const size_t rb = sizeof(double) * 2 * (size_t)c->g.V;
    auto force = [&]() -> int {
        HIP_TRY(hipMemsetAsync(c->Fmd, 0, rb, c->stream));
        launch_staple_force(c->stream, c->g, c->kshards(), c->U, ufaces(c), p->beta, c->Fmd, nullptr);
        HIP_TRY(hipGetLastError());
        return SM_OK;
    };
    TRY(md_step(c, c->Pmd, eps, 0, 0.5 * eps));
    TRY(force());
    for (int step = 1; step < p->md_steps - 1; step++) {
        TRY(md_step(c, c->Pmd, eps, 1, eps));
        TRY(force());
    }
    TRY(md_step(c, c->Pmd, eps, 1, 0.5 * eps));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return SM_OK;
}

int sm_hmc_trajectory(sm_ctx *c, const sm_hmc_params *p, uint64_t traj, sm_hmc_result *out) {
    TRY(check_ready(c));
    TRY(check_params(p));
    if (!out) return fail(SM_ERR_ARG, "null argument");
    HIP_TRY(hipSetDevice(c->device));
    TRY(ensure_md(c));
    // HMC::HMC_Update, src/hmc.cpp:151-178
    const uint64_t ts = sm_traj_seed(p->seed, traj);
    double2 *chi = c->field(F_L), *phi = c->field(F_PHI);
    launch_draw_momenta(c->stream, c->g, ts, c->Pmd);   // RandomPI
    launch_draw_source(c->stream, c->g, ts, chi);       // RandomCHI
    HIP_TRY(hipGetLastError());
    if (p->even_odd) TRY(eo_pseudofermion(c, p, chi, phi));              // phi_e = Dhat chi_e
    else TRY(apply(c, chi, phi, p->m0 + 2, 0, nullptr, nullptr, nullptr));  // phi = D chi
    sm_hamiltonian_terms h0, h1;
    TRY(sm_hamiltonian_dev(c, p, (const double *)phi, c->Pmd, &h0));   // H[U][Pi] (P not yet evolved)
    // leapfrog on a copy of U: the kept configuration stays in U_alt
    HIP_TRY(hipMemcpyAsync(c->U_alt, c->U, sizeof(double2) * 2 * c->g.V, hipMemcpyDeviceToDevice, c->stream));
    std::swap(c->U, c->U_alt);   // ghost links are unchanged (identical copy)
    long lf_iters = 0;
    int lf_fails = 0;
    TRY(sm_leapfrog_dev(c, p, (const double *)phi, c->Pmd, &lf_iters, &lf_fails));
    TRY(sm_hamiltonian_dev(c, p, (const double *)phi, c->Pmd, &h1));   // H[U'][Pi']
    out->H_old = h0.H;
    out->H_new = h1.H;
    out->dH = h1.H - h0.H;
    out->r = sm_uniform(ts, SM_STREAM_ACCEPT, 0);
    out->accepted = out->r <= std::exp(-out->dH) ? 1 : 0;
    if (!out->accepted) {
        std::swap(c->U, c->U_alt);  // back to the previous configuration
        TRY(exchange_ghost_U(c));
    }
    const sm_hamiltonian_terms &kept = out->accepted ? h1 : h0;
    out->sp = kept.sp;
    out->gauge_action = kept.gauge_action;
    out->cg_iterations = (long)h0.cg_iterations + lf_iters + h1.cg_iterations;
    out->cg_failures = (h0.cg_converged ? 0 : 1) + lf_fails + (h1.cg_converged ? 0 : 1);
    return SM_OK;
}

}  // extern "C"
