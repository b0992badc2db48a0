// sm_eo.cpp -- even-odd (Schur) preconditioned pseudofermion action for the
// device HMC (opt-in via sm_hmc_params::even_odd).
//
// With D = [[m, D_eo], [D_oe, m]] (m = m0 + 2, D_eo/D_oe the hopping blocks),
// det D = m^{V/2} det Dhat, Dhat = m - (1/m) D_eo D_oe on the even sites, so
// det(D D^dag) is det(Dhat Dhat^dag) up to a constant and the action
//     S_f = phi_e^dag (Dhat Dhat^dag)^{-1} phi_e,   phi_e = Dhat chi_e
// samples the same gauge-field distribution as the reference's
// phi^dag (D D^dag)^{-1} phi (src/hmc.cpp:44-60, 114-126), with one CG on half
// the sites per force instead of one on all of them, and a better-conditioned
// operator (the prototype in DESIGN.md: 0.42x the iterations of the full solve).
//
// Force: with X = (Dhat Dhat^dag)^{-1} phi_e and Y = Dhat^dag X,
//     dS_f = -2 Re(X^dag dDhat Y) = -2 Re(l^dag dD r),
//     l = (X, -(1/m) (D^dag)_oe X),  r = (Y, -(1/m) D_oe Y),
// so the reference's own fermion-force bilinear phi_dag_partialD_phi(U, l, r)
// (src/dirac_operator.cpp:486-580; sm_force_dev) gives it, plus the gauge force.
// With H the hopping bracket (D = m - 0.5 H): D_oe v = -0.5 H_oe v and
//     Dhat v = m v + (0.5/m) H_eo (D_oe v),   l_o = (0.5/m) H'_oe X, r_o = (0.5/m) H_oe Y.
// Kernels: sm_eo.hip. t-sharded like the full operator: every hop exchanges
// the 2-column checkerboard faces of its input (and, once per gauge field,
// of both link parities) with the t +- 1 shards; dots are all-reduced.
#include <cmath>

#include <cstdio>

#include "sm_ctx.h"
#include "sm_fields.h"
#include "sm_internal.h"

using namespace sm;
using namespace sm_host;

namespace sm_host {

// eo work vectors (each one parity: 2 planes x V/2 = V complex)
enum { EO_X, EO_R, EO_D, EO_AD, EO_T, EO_W, EO_PHI, EO_Y, EO_CHI, EO_LO, EO_RO, EO_R2, EO_D2, EO_N };

static double2 *eo_vec(sm_ctx *c, int i) { return c->eo + (size_t)i * c->g.V; }
static double2 *ucb(sm_ctx *c, int parity) { return c->Ucb + (size_t)parity * c->g.V; }

// t-sharded: face slots of 8*Nx complex ([side][plane][col][x], sm_eo.hip):
// 0 send staging, 1 / 2 received faces of the even / odd links, 3 / 4 of the
// two vectors a hop sequence has in flight, 5 / 6 of r and Ad (folded CG).
enum { EOF_SEND, EOF_UE, EOF_UO, EOF_V, EOF_W, EOF_R, EOF_A, EOF_N };
static double2 *eo_face(sm_ctx *c, int slot) { return c->eo_faces + (size_t)slot * 8 * c->g.Nx; }

// 4-deep face slots of the one-pass eo CG (16*Nx complex each): 0 send
// staging, 1 / 2 even / odd links, 3 / 4 d_{j-1} by pass parity (pass j still
// holds d_{j-2}'s), 5 Ad_{j-1}.
enum { EOF4_SEND, EOF4_UE, EOF4_UO, EOF4_D0, EOF4_D1, EOF4_AD, EOF4_SEND2, EOF4_N };
static double2 *eo_face4(sm_ctx *c, int slot) { return c->eo_faces4 + (size_t)slot * 16 * c->g.Nx; }
static bool eo_td_sharded_ok(const sm_ctx *c) { return c->sharded() && c->g.Wt >= 8; }

static int eo_halo4(sm_ctx *c, const double2 *f, int slot) {
    double2 *snd = eo_face4(c, EOF4_SEND), *rcv = eo_face4(c, slot);
    const size_t half = (size_t)8 * c->g.Nx;  // complex per side
    launch_pack_cb_faces4(c->stream, c->g, f, snd);
    return exchange_faces_on(c, c->stream, snd, snd + half, rcv, rcv + half, 2 * half);
}

// The 4-deep faces of two vectors (d_{j-1} and Ad_{j-1}) in one transport round.
static int eo_halo4_pair(sm_ctx *c, const double2 *f1, int slot1, const double2 *f2, int slot2) {
    double2 *s1 = eo_face4(c, EOF4_SEND), *s2 = eo_face4(c, EOF4_SEND2);
    double2 *r1 = eo_face4(c, slot1), *r2 = eo_face4(c, slot2);
    const size_t half = (size_t)8 * c->g.Nx;  // complex per side
    launch_pack_cb_faces4(c->stream, c->g, f1, s1);
    launch_pack_cb_faces4(c->stream, c->g, f2, s2);
    double2 *slo[2] = {s1, s2}, *shi[2] = {s1 + half, s2 + half};
    double2 *rlo[2] = {r1, r2}, *rhi[2] = {r1 + half, r2 + half};
    return exchange_faces_multi(c, c->stream, 2, slo, shi, rlo, rhi, 2 * half);
}

// Exchange the checkerboard t-faces of f into face slot `slot`; returns the
// received faces (null on one shard: the kernels wrap periodically).
static int eo_halo(sm_ctx *c, const double2 *f, int slot, const double2 **out) {
    *out = nullptr;
    if (!c->sharded()) return SM_OK;
    double2 *snd = eo_face(c, EOF_SEND), *rcv = eo_face(c, slot);
    const size_t half = (size_t)4 * c->g.Nx;  // complex per side
    launch_pack_cb_faces(c->stream, c->g, f, snd);
    TRY(exchange_faces_on(c, c->stream, snd, snd + half, rcv, rcv + half, 2 * half));
    *out = rcv;
    return SM_OK;
}

static EoFaces u_faces(sm_ctx *c) {
    EoFaces f;
    if (c->sharded()) {
        f.ue = eo_face(c, EOF_UE);
        f.uo = eo_face(c, EOF_UO);
    }
    return f;
}

int eo_ready(sm_ctx *c) {
    // the periodic lattice is bipartite (a checkerboard) only for even Nx and
    // Nt; t-shards of even width keep every t0 even (local parity = global)
    if (c->g.Wt % 2 || c->g.Nx % 2)
        return fail(SM_ERR_ARG, "even-odd preconditioning needs even Nx and shard width (%d x %d)", c->g.Nx,
                    c->g.Wt);
    if (c->sharded() && c->g.Wt < 4)
        return fail(SM_ERR_ARG, "even-odd preconditioning needs t-shards at least 4 wide (Wt = %d)", c->g.Wt);
    if (!c->eo) {
        HIP_TRY(hipMalloc(&c->eo, sizeof(double2) * (size_t)EO_N * c->g.V));
        HIP_TRY(hipMalloc(&c->Ucb, sizeof(double2) * 2 * (size_t)c->g.V));
        if (c->sharded()) HIP_TRY(hipMalloc(&c->eo_faces, sizeof(double2) * (size_t)EOF_N * 8 * c->g.Nx));
        if (eo_td_sharded_ok(c))
            HIP_TRY(hipMalloc(&c->eo_faces4, sizeof(double2) * (size_t)EOF4_N * 16 * c->g.Nx));
    }
    // checkerboard copy of the current gauge field (U changes between calls)
    launch_to_cb(c->stream, c->g, c->U, ucb(c, 0), ucb(c, 1));
    HIP_TRY(hipGetLastError());
    const double2 *f;
    TRY(eo_halo(c, ucb(c, 0), EOF_UE, &f));
    TRY(eo_halo(c, ucb(c, 1), EOF_UO, &f));
    if (eo_td_sharded_ok(c)) {
        TRY(eo_halo4(c, ucb(c, 0), EOF4_UE));
        TRY(eo_halo4(c, ucb(c, 1), EOF4_UO));
    }
    return SM_OK;
}

// out_e = Dhat v_e (dagger = 0) or Dhat^dag v_e (dagger = 1). Fused: both
// hops in one marching pass (eo_dhat_fused_kernel), optionally with partials
// of sum aux * conj(out); unfused (c->eo_fused == 0): two eo_hop launches
// through EO_T, bitwise the same result. t-sharded: v's faces go to slot
// EOF_V first (and T's to EOF_W unfused). *nparts: the partial count.
int eo_dhat(sm_ctx *c, int dagger, const double2 *v, double2 *out, double mass, const double2 *aux = nullptr,
            double2 *partials = nullptr, int *nparts = nullptr) {
    EoFaces f = u_faces(c);
    TRY(eo_halo(c, v, EOF_V, &f.v));
    if (c->eo_fused) {
        const EoFusedCfg cfg = eo_fused_config(c->g);
        launch_eo_dhat_fused(c->stream, c->g, cfg, dagger, v, ucb(c, 0), ucb(c, 1), mass, out, aux, partials, f);
        if (nparts) *nparts = eo_fused_blocks(cfg);
        return SM_OK;
    }
    double2 *T = eo_vec(c, EO_T);
    launch_eo_hop(c->stream, c->g, dagger, 1, v, ucb(c, 1), ucb(c, 0), nullptr, 0.0, -0.5, T, f.v, f.ue);  // D_oe v
    const double2 *tf;
    TRY(eo_halo(c, T, EOF_W, &tf));
    launch_eo_hop(c->stream, c->g, dagger, 0, T, ucb(c, 0), ucb(c, 1), v, mass, 0.5 / mass, out, tf, f.uo);
    if (aux) launch_dot_partial(c->stream, c->g.V, aux, out, partials);
    if (nparts) *nparts = reduce_blocks(c->g.V);
    return SM_OK;
}

// out = Dhat Dhat^dag v (uses EO_W; EO_T unfused); dot partials of <v, out>
// into c->partials; returns their count.
static int eo_M(sm_ctx *c, const double2 *v, double2 *out, double mass, int *nparts) {
    double2 *W = eo_vec(c, EO_W);
    TRY(eo_dhat(c, 1, v, W, mass));
    return eo_dhat(c, 0, W, out, mass, v, c->partials, nparts);
}

// Folded CG on Dhat Dhat^dag (c->eo_cg_folded, needs the fused Dhat): the
// one-pass recurrence of the full CG (cg_onepass_kernel / cg1_scalars) on
// half-lattice vectors. Iteration j = pass A (r_j, d_j, x; W = Dhat^dag d_j)
// + pass B (Ad_j = Dhat W, <d_j,Ad_j>, <r_j,Ad_j>, |Ad_j|^2) + the scalar
// kernel (stop test on the direct |r_j|^2, alpha_j, beta_j by the expansion).
// 3 launches instead of 6, and r, Ad, d, x are not re-streamed by separate
// BLAS-1 kernels: ~512 instead of 576 B per even site. r and d ping-pong.
static int eo_cg_folded(sm_ctx *c, const double2 *b, double2 *x, double mass, double tol, int max_iter,
                        sm_cg_result *res) {
    const long n = c->g.V;
    const int nred = reduce_blocks(n);
    double2 *Ad = eo_vec(c, EO_AD), *W = eo_vec(c, EO_W);
    double2 *rb[2] = {eo_vec(c, EO_R), eo_vec(c, EO_R2)}, *db[2] = {eo_vec(c, EO_D), eo_vec(c, EO_D2)};
    if (x != b) launch_copy(c->stream, n, b, x);
    int np;
    TRY(eo_M(c, x, Ad, mass, &np));
    double2 *prr = c->partials, *ppp = c->partials + nred;
    launch_cg_init(c->stream, n, b, Ad, rb[0], db[0], prr, ppp);                // r_0 = b - M x_0; d_0 = r_0
    if (!c->sharded()) {
        launch_cg_finalize_init(c->stream, nred, prr, ppp, c->sc, tol);
    } else {
        launch_sum_partials(c->stream, nred, prr, c->sums);
        launch_sum_partials(c->stream, nred, ppp, c->sums + 1);
        TRY(allreduce_dev(c, (double *)c->sums, 4));
        launch_cg_init_from_sums(c->stream, c->sums, c->sc, tol);
    }
    HIP_TRY(hipMemsetD32Async((hipDeviceptr_t)&c->sc->max_iter, max_iter, 1, c->stream));
    const EoFusedCfg cfg = eo_fused_config(c->g);
    const int nparts = eo_fused_blocks(cfg);
    const EoFaces uf = u_faces(c);
    long j = 0;
    auto pass = [&]() -> int {
        const int o = j & 1;
        EoCgPass q;
        q.dold = db[o];
        q.rold = rb[o];
        q.dnew = db[1 - o];
        q.rnew = rb[1 - o];
        q.x = x;
        q.W = W;
        q.ad = Ad;
        q.first = j == 0;
        EoFaces f = uf;
        TRY(eo_halo(c, q.dold, EOF_V, &f.v));
        TRY(eo_halo(c, q.rold, EOF_R, &q.rf));
        TRY(eo_halo(c, Ad, EOF_A, &q.af));
        launch_eo_cg_pass(c->stream, c->g, cfg, 0, q, ucb(c, 0), ucb(c, 1), mass, f, c->sc, c->partials);
        TRY(eo_halo(c, W, EOF_W, &q.wf));
        launch_eo_cg_pass(c->stream, c->g, cfg, 1, q, ucb(c, 0), ucb(c, 1), mass, f, c->sc, c->partials);
        if (!c->sharded()) {
            launch_cg1_scalars(c->stream, nparts, c->partials, c->sc, q.first);
        } else {
            launch_cg1_local_sum(c->stream, nparts, c->partials, c->sc);
            TRY(allreduce_dev(c, (double *)c->sc->sum3, 6));
            launch_cg1_from_sums(c->stream, c->sc, q.first);
        }
        ++j;
        return SM_OK;
    };
    // pass 0 forms Ad_0; pass j >= 1 completes iteration j (the device stops
    // itself at convergence or k = max_iter); all ranks read the same status
    const long passes = (long)max_iter + 1;
    CgChunker plan;
    int chunk = plan.chunk;
    while (j < passes) {
        const long nb = (passes - j) < chunk ? (passes - j) : chunk;
        for (long i = 0; i < nb; ++i) TRY(pass());
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipMemcpyAsync(c->h_sc, c->sc, sizeof(CGScalars), hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(hipStreamSynchronize(c->stream));
        if (c->h_sc->done) break;
        chunk = plan.next(c->h_sc->k, c->h_sc->err, tol * c->h_sc->phi_norm);
    }
    res->converged = c->h_sc->converged;
    res->iterations = c->h_sc->k;
    res->residual = c->h_sc->err;
    res->phi_norm = c->h_sc->phi_norm;
    return SM_OK;
}

// One-pass two-direction CG on Dhat Dhat^dag (c->eo_cg_td; t-shards of width
// >= 8 exchange 4-deep checkerboard faces of d_{j-1} and Ad_{j-1}; sm_eotd.hip): pass j forms r_j, d_j, the even-pass x update and Ad_j =
// Dhat Dhat^dag d_j in one launch, then cg1_scalars. d_i rotates through three
// buffers (d_0 from cg_init in EO_D), Ad_j goes to abuf[j & 1]; after an odd
// final pass the pending alpha d is added (launch_cg_td_finish_x). ~256 B per
// even site and pass against ~575 for the six-launch iteration.
static int eo_cg_twodir(sm_ctx *c, const double2 *b, double2 *x, double mass, double tol, int max_iter,
                        sm_cg_result *res) {
    const long n = c->g.V;
    const int nred = reduce_blocks(n);
    double2 *dslot[3] = {eo_vec(c, EO_D2), eo_vec(c, EO_R), eo_vec(c, EO_D)};
    auto dbuf = [&](long i) { return dslot[((i % 3) + 3) % 3]; };
    double2 *abuf[2] = {eo_vec(c, EO_AD), eo_vec(c, EO_R2)};
    if (x != b) launch_copy(c->stream, n, b, x);
    int np;
    TRY(eo_M(c, x, eo_vec(c, EO_AD), mass, &np));
    double2 *prr = c->partials, *ppp = c->partials + nred;
    launch_cg_init(c->stream, n, b, eo_vec(c, EO_AD), eo_vec(c, EO_R), eo_vec(c, EO_D), prr, ppp);  // r_0, d_0
    if (!c->sharded()) {
        launch_cg_finalize_init(c->stream, nred, prr, ppp, c->sc, tol);
    } else {
        launch_sum_partials(c->stream, nred, prr, c->sums);
        launch_sum_partials(c->stream, nred, ppp, c->sums + 1);
        TRY(allreduce_dev(c, (double *)c->sums, 4));
        launch_cg_init_from_sums(c->stream, c->sums, c->sc, tol);
    }
    HIP_TRY(hipMemsetD32Async((hipDeviceptr_t)&c->sc->max_iter, max_iter, 1, c->stream));
    const EoTdCfg cfg = eo_td_config(c->g);
    const int nparts = eo_td_blocks(cfg);
    if (3 * nparts > 2 * kMaxPartials) return fail(SM_ERR_ARG, "even-odd CG grid too large");
    const bool tail = c->cg_tail && (nparts + 63) / 64 <= kMaxTickGroups;
    // t-shards: every block evaluates the previous pass's scalars from the
    // all-reduced sums (as the full CG's t-shard passes), flushed per chunk
    const bool red = c->sharded() && tail && c->cg_red_shards;
    long j = 0;
    auto pass = [&]() -> int {
        const bool first = j == 0;
        // pass 0 reads d_0 and takes zero multipliers: its d_{j-2} / Ad_{j-1}
        // operands only need to be finite, so they alias d_0 too
        const double2 *d1 = first ? eo_vec(c, EO_D) : dbuf(j - 1);
        const double2 *d2 = j >= 2 ? dbuf(j - 2) : d1;
        const double2 *aold = first ? d1 : abuf[(j - 1) & 1];
        EoTdFaces f;
        if (c->sharded()) {  // faces of d_{j-1} (d_{j-2}'s are the previous pass's) and Ad_{j-1}
            const int sd = (j & 1) ? EOF4_D1 : EOF4_D0, sp = (j & 1) ? EOF4_D0 : EOF4_D1;
            if (first) TRY(eo_halo4(c, d1, sd));
            else TRY(eo_halo4_pair(c, d1, sd, aold, EOF4_AD));  // one transport round for both
            f.d1 = eo_face4(c, sd);
            f.d2 = j >= 2 ? eo_face4(c, sp) : f.d1;
            f.ad = first ? f.d1 : eo_face4(c, EOF4_AD);
            f.ue = eo_face4(c, EOF4_UE);
            f.uo = eo_face4(c, EOF4_UO);
        }
        // ticketed tail: the pass's last block forms the scalars (or this
        // shard's sums) instead of a separate kernel
        double2 *sums = red ? &c->sc->sumr[j & 1][0] : c->sc->sum3;
        launch_eo_td(c->stream, c->g, cfg, d1, d2, aold, dbuf(j), abuf[j & 1], x, ucb(c, 0), ucb(c, 1), mass, j,
                     c->sc, c->partials, f, tail ? c->tick : nullptr, c->gsum, c->sharded() ? sums : nullptr, red);
        if (!c->sharded()) {
            if (!tail) launch_cg1_scalars(c->stream, nparts, c->partials, c->sc, first);
        } else {
            if (!tail) launch_cg1_local_sum(c->stream, nparts, c->partials, c->sc);
            TRY(allreduce_dev(c, (double *)sums, 6));
            if (!red) launch_cg1_from_sums(c->stream, c->sc, first);
        }
        ++j;
        return SM_OK;
    };
    const long passes = (long)max_iter + 1;
    CgChunker plan;
    int chunk = plan.chunk;
    while (j < passes) {
        const long nb = (passes - j) < chunk ? (passes - j) : chunk;
        for (long i = 0; i < nb; ++i) TRY(pass());
        if (red) launch_cg_ra_flush_sums(c->stream, c->sc, j - 1);  // the last pass's scalars for the host
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipMemcpyAsync(c->h_sc, c->sc, sizeof(CGScalars), hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(hipStreamSynchronize(c->stream));
        if (c->debug_cg)
            fprintf(stderr, "[sm eo_cg shard %d/%d] pass %ld k %d err %.3e target %.3e done %d\n", c->shard, c->nshard, j,
                    c->h_sc->k, c->h_sc->err, tol * c->h_sc->phi_norm, c->h_sc->done);
        if (c->h_sc->done) break;
        chunk = plan.next(c->h_sc->k, c->h_sc->err, tol * c->h_sc->phi_norm);
    }
    launch_cg_td_finish_x(c->stream, n, x, dbuf(0), dbuf(1), dbuf(2), c->sc);  // odd final pass: pending alpha d
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpyAsync(c->h_sc, c->sc, sizeof(CGScalars), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    res->converged = c->h_sc->converged;
    res->iterations = c->h_sc->k;
    res->residual = c->h_sc->err;
    res->phi_norm = c->h_sc->phi_norm;
    return SM_OK;
}

// CG on Dhat Dhat^dag x = b (x0 = b, the reference's convention), the
// reference's recurrence and stop test on half-lattice vectors.
int eo_cg(sm_ctx *c, const double2 *b, double2 *x, double mass, double tol, int max_iter, sm_cg_result *res) {
    if (c->eo_cg_td && (!c->sharded() || eo_td_sharded_ok(c))) return eo_cg_twodir(c, b, x, mass, tol, max_iter, res);
    if (c->eo_cg_folded && c->eo_fused) return eo_cg_folded(c, b, x, mass, tol, max_iter, res);
    const long n = c->g.V;  // complex entries of an even vector
    const int nparts = reduce_blocks(n);
    double2 *r = eo_vec(c, EO_R), *d = eo_vec(c, EO_D), *Ad = eo_vec(c, EO_AD);
    if (x != b) launch_copy(c->stream, n, b, x);
    int np;
    TRY(eo_M(c, x, Ad, mass, &np));                          // (its dot partials are not used)
    double2 *prr = c->partials, *ppp = c->partials + nparts;
    launch_cg_init(c->stream, n, b, Ad, r, d, prr, ppp);
    if (!c->sharded()) {
        launch_cg_finalize_init(c->stream, nparts, prr, ppp, c->sc, tol);
    } else {
        launch_sum_partials(c->stream, nparts, prr, c->sums);
        launch_sum_partials(c->stream, nparts, ppp, c->sums + 1);
        TRY(allreduce_dev(c, (double *)c->sums, 4));
        launch_cg_init_from_sums(c->stream, c->sums, c->sc, tol);
    }
    // every rank takes the same decisions: the status read back is global
    CgChunker plan;
    int issued = 0, chunk = plan.chunk;
    while (issued < max_iter) {
        const int nb = (max_iter - issued) < chunk ? (max_iter - issued) : chunk;
        for (int i = 0; i < nb; ++i) {
            TRY(eo_M(c, d, Ad, mass, &np));                          // Ad and partials of <d, Ad>
            TRY(cg_scalar(c, np, 0));                                // alpha
            launch_cg_update_xr(c->stream, n, x, r, d, Ad, c->sc, c->partials);
            TRY(cg_scalar(c, nparts, 1));                            // stop test, beta
            launch_cg_update_d(c->stream, n, d, r, c->sc);
        }
        HIP_TRY(hipGetLastError());
        issued += nb;
        HIP_TRY(hipMemcpyAsync(c->h_sc, c->sc, sizeof(CGScalars), hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(hipStreamSynchronize(c->stream));
        if (c->h_sc->done) break;
        chunk = plan.next(c->h_sc->k, c->h_sc->err, tol * c->h_sc->phi_norm);
    }
    res->converged = c->h_sc->converged;
    res->iterations = c->h_sc->k;
    res->residual = c->h_sc->err;
    res->phi_norm = c->h_sc->phi_norm;
    return SM_OK;
}

// phi (full layout) -> its even part in EO_PHI
static void eo_take_even(sm_ctx *c, const double2 *full, double2 *e) {
    launch_to_cb(c->stream, c->g, full, e, nullptr);
}

// Even-odd HMC force at the current U: F = bilinear(U, l, r) + gauge force.
int eo_md_force(sm_ctx *c, const sm_hmc_params *p, const double2 *phi_full, double *F, sm_cg_result *res) {
    TRY(eo_ready(c));
    const double m = p->m0 + 2;
    double2 *phie = eo_vec(c, EO_PHI), *X = eo_vec(c, EO_X), *Y = eo_vec(c, EO_Y);
    double2 *lo = eo_vec(c, EO_LO), *ro = eo_vec(c, EO_RO);
    eo_take_even(c, phi_full, phie);
    TRY(eo_cg(c, phie, X, m, p->cg_tol, p->cg_max_iter, res));
    TRY(eo_dhat(c, 1, X, Y, m));                                                        // Y = Dhat^dag X
    const EoFaces f = u_faces(c);
    const double2 *xf, *yf;
    TRY(eo_halo(c, X, EOF_V, &xf));
    launch_eo_hop(c->stream, c->g, 1, 1, X, ucb(c, 1), ucb(c, 0), nullptr, 0.0, 0.5 / m, lo, xf, f.ue);  // l_o
    TRY(eo_halo(c, Y, EOF_V, &yf));
    launch_eo_hop(c->stream, c->g, 0, 1, Y, ucb(c, 1), ucb(c, 0), nullptr, 0.0, 0.5 / m, ro, yf, f.ue);  // r_o
    double2 *L = c->field(F_L), *R = c->field(F_RR);
    launch_from_cb(c->stream, c->g, X, lo, L);
    launch_from_cb(c->stream, c->g, Y, ro, R);
    HIP_TRY(hipGetLastError());
    TRY(sm_force_dev(c, (const double *)L, (const double *)R, F));
    return SM_OK;
}

// Even-odd fermion action Re dot((Dhat Dhat^dag)^{-1} phi_e, phi_e).
int eo_fermion_action(sm_ctx *c, const sm_hmc_params *p, const double2 *phi_full, double *S, sm_cg_result *res) {
    TRY(eo_ready(c));
    const double m = p->m0 + 2;
    double2 *phie = eo_vec(c, EO_PHI), *X = eo_vec(c, EO_X);
    eo_take_even(c, phi_full, phie);
    TRY(eo_cg(c, phie, X, m, p->cg_tol, p->cg_max_iter, res));
    // dot over the V complex entries of an even vector (sm_dot_dev spans 2V)
    launch_dot_partial(c->stream, c->g.V, X, phie, c->partials);
    TRY(global_sum(c, reduce_blocks(c->g.V), c->partials, 0));
    HIP_TRY(hipMemcpyAsync(c->h_sums, c->sums, sizeof(double2), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    *S = c->h_sums[0].x;
    return SM_OK;
}

// phi_full = (Dhat chi_e, 0) for the pseudofermion heat bath.
int eo_pseudofermion(sm_ctx *c, const sm_hmc_params *p, const double2 *chi_full, double2 *phi_full) {
    TRY(eo_ready(c));
    double2 *chie = eo_vec(c, EO_CHI), *phie = eo_vec(c, EO_PHI);
    eo_take_even(c, chi_full, chie);
    TRY(eo_dhat(c, 0, chie, phie, p->m0 + 2));
    launch_from_cb(c->stream, c->g, phie, nullptr, phi_full);
    HIP_TRY(hipGetLastError());
    return SM_OK;
}

}  // namespace sm_host

extern "C" {

int sm_eo_dhat(sm_ctx *c, int dagger, const double *in0, const double *in1, double *out0, double *out1,
               double m0) {
    TRY(check_ready(c));
    if (!in0 || !in1 || !out0 || !out1) return fail(SM_ERR_ARG, "null argument");
    HIP_TRY(hipSetDevice(c->device));
    TRY(eo_ready(c));
    double2 *in = c->field(F_IN), *out = c->field(F_OUT);
    TRY(upload_plane_pair(c, in, in0, in1));
    double2 *ve = eo_vec(c, EO_CHI), *oe = eo_vec(c, EO_X);
    eo_take_even(c, in, ve);
    TRY(eo_dhat(c, dagger ? 1 : 0, ve, oe, m0 + 2));
    launch_from_cb(c->stream, c->g, oe, nullptr, out);
    HIP_TRY(hipGetLastError());
    return download_plane_pair(c, out, out0, out1);
}

int sm_eo_cg(sm_ctx *c, const double *phi0, const double *phi1, double *x0, double *x1, double m0, double tol,
             int max_iter, sm_cg_result *res) {
    TRY(check_ready(c));
    if (!phi0 || !phi1 || !x0 || !x1 || !res) return fail(SM_ERR_ARG, "null argument");
    HIP_TRY(hipSetDevice(c->device));
    TRY(eo_ready(c));
    double2 *in = c->field(F_IN), *out = c->field(F_OUT);
    TRY(upload_plane_pair(c, in, phi0, phi1));
    double2 *phie = eo_vec(c, EO_PHI), *X = eo_vec(c, EO_X);
    eo_take_even(c, in, phie);
    TRY(eo_cg(c, phie, X, m0 + 2, tol, max_iter, res));
    launch_from_cb(c->stream, c->g, X, nullptr, out);
    HIP_TRY(hipGetLastError());
    return download_plane_pair(c, out, x0, x1);
}

}  // extern "C"
