// sm_kernels.hip -- gfx950 (MI355X) kernels for the Wilson-Dirac / CG hot path.
//
// Drop-in target: src/dirac_operator.cpp + src/conjugate_gradient.cpp of
// Fabian2598/SchwingerModel. All arithmetic is IEEE fp64 with NO contraction
// (-ffp-contract=off + the pragma below) and the reference's evaluation order,
// so D, D^dagger and the force are bit-identical to the reference (checked in
// tests/test_gpu_parity.py against tests/golden/).
//
// The hot kernel is a marching 5-point stencil: a block owns `bt` consecutive
// t-columns and marches `xchunk` rows along x, keeping psi(x-1), psi(x),
// psi(x+1) and U_x(x-1) in registers, so each field row crosses HBM once
// (plus a 1-row halo per chunk). t-neighbours come from the wave's own
// coalesced row loads (L1/L2 hits). HBM-bound: 96 B/site algorithmic.
#include "sm_device.h"
#include "sm_internal.h"

#pragma clang fp contract(off)

namespace sm {

struct DArgs {
    const double2 *__restrict__ in;
    double2 *__restrict__ out;
    const double2 *__restrict__ U;
    const double2 *loU;
    TFaces f;
    const double2 *aux;
    double2 *partials;
    const CGScalars *sc;
    long V;
    int Nx, Wt, t0, Ntg, xchunk;
    int TB, XB, xcd_remap;   // tile grid (t-blocks x x-chunks), 1-D launch
    int tb0, tbn, part0;     // this launch covers t-blocks [tb0, tb0+tbn) mod TB; partials by tile
    double mass;
};

// Linear block id -> (t-block, x-chunk). With xcd_remap the ids that the
// dispatcher deals to one XCD (L, L+8, L+16, ...: round-robin, speed only,
// MI355X_MICROARCH.md) get a contiguous range of tiles, so the x-halo rows and
// t-edge lines shared by neighbouring tiles are L2 hits on that XCD.
// The t-block range wraps modulo TB, so the two edge block-columns of a
// t-shard (TB-1 and 0) are one launch.
__device__ __forceinline__ void block_tile(int L, int tb0, int tbn, int TB, int XB, int remap, int &tb, int &xc) {
    int w = L;
    if (remap) {
        const int n = tbn * XB, q = n >> 3, r = n & 7, xcd = L & 7;
        w = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (L >> 3);
    }
    tb = tb0 + w % tbn;
    if (tb >= TB) tb -= TB;
    xc = w / tbn;
}

// Row loads for column t of row x: centre psi, t-neighbours psi(t-1), psi(t+1),
// links U_t(x,t), U_x(x,t), U_t(x,t-1). Edge lanes read the faces (or the
// periodic wrap) through a per-lane POINTER select followed by one
// unconditional load: no branch, so the compiler can keep the next row's
// loads in flight across the loop back-edge (a divergent `c ? load : load`
// becomes a branch and a vmcnt(0) drain per row).
struct Row {
    double2 c0, c1, m0, m1, p0, p1, ut, ux, utm;
};

struct LaneSrc {             // per-lane neighbour addressing, fixed for the whole march
    const double2 *pm, *pp, *um;   // base of the t-1 / t+1 column and of U_t(t-1)
    long pms, pps;                 // plane stride for pm / pp
    long xs_m, xs_p;               // row stride for pm(+um) / pp
};

__device__ __forceinline__ LaneSrc lane_src(const DArgs &a, int t) {
    LaneSrc s;
    const bool lo = t == 0, hi = t + 1 == a.Wt;
    s.pm = lo ? a.f.lo : a.in + (t - 1);
    s.um = lo ? a.loU : a.U + (t - 1);
    s.pms = lo ? a.f.lo_ps : a.V;
    s.xs_m = lo ? a.f.lo_xs : (long)a.Wt;
    s.pp = hi ? a.f.hi : a.in + (t + 1);
    s.pps = hi ? a.f.hi_ps : a.V;
    s.xs_p = hi ? a.f.hi_xs : (long)a.Wt;
    return s;
}

// xn: row of the centre psi; xs: row of everything else (== xn except at the
// chunk's last step, where it re-reads the current row: cache hits, no HBM).
__device__ __forceinline__ void load_row(const DArgs &a, const LaneSrc &L, int xn, int xs, int t,
                                         Row &r) {
    const long n = (long)xn * a.Wt + t;
    r.c0 = a.in[n];
    r.c1 = a.in[n + a.V];
    const long ns = (long)xs * a.Wt + t;
    const double2 *pm = L.pm + (long)xs * L.xs_m;
    const double2 *pp = L.pp + (long)xs * L.xs_p;
    r.m0 = pm[0];
    r.m1 = pm[L.pms];
    r.p0 = pp[0];
    r.p1 = pp[L.pps];
    r.ut = a.U[ns];
    r.ux = a.U[ns + a.V];
    r.utm = L.um[(long)xs * L.xs_m];
}

// dirac_site with spin-projected t-faces (TFaces::proj, t-shards): on the
// edge lanes the t-hop operands arrive pre-combined. elo: pm0 holds
// conj(U_t(t-1)) * (backward combination), formed by the sending shard, and
// the hop is sl0 times it; ehi: pt0 holds the forward combination. The
// reference's second-spin terms (D: a(-pt0+pt1); D^dag: c(-pm0+pm1)) are the
// exact negations of the first's, so every value equals dirac_site's up to
// the sign of an exact zero; off the edges it IS dirac_site's arithmetic.
template <int DAG>
__device__ __forceinline__ void dirac_site_proj(double mass, double sr0, double sl0, bool elo, bool ehi, double2 p0,
                                                double2 p1, double2 pt0, double2 pt1, double2 px0, double2 px1,
                                                double2 pm0, double2 pm1, double2 pxm0, double2 pxm1, double2 Ut,
                                                double2 Ux, double2 Utm, double2 Uxm, double2 &s0, double2 &s1) {
    const double2 one = make_double2(1.0, 0.0);
    const double2 a = cmul(Ut, make_double2(sr0, 0.0));
    const double2 b = cmul(Ux, one);
    const double2 c = cmul(cconj(Utm), make_double2(sl0, 0.0));
    const double2 e = cmul(cconj(Uxm), one);
    const double2 Ce = make_double2(sl0 * pm0.x, sl0 * pm0.y);  // edge: sl0 * conj(U_t(t-1)) combo
    double2 h0, h1;
    if (!DAG) {
        double2 A = cmul(a, ehi ? pt0 : csub(pt0, pt1));
        double2 B = cmul(b, cadd(px0, cmul(I_NUM, px1)));
        const double2 C = elo ? Ce : cmul(c, cadd(pm0, pm1));
        double2 E = cmul(e, csub(pxm0, cmul(I_NUM, pxm1)));
        h0 = cadd(cadd(cadd(A, B), C), E);
        A = ehi ? cneg(A) : cmul(a, cadd(cneg(pt0), pt1));
        B = cmul(b, cadd(cmul(MI_NUM, px0), px1));
        E = cmul(e, cadd(cmul(I_NUM, pxm0), pxm1));
        h1 = cadd(cadd(cadd(A, B), C), E);
    } else {
        double2 C = elo ? Ce : cmul(c, csub(pm0, pm1));
        double2 E = cmul(e, cadd(pxm0, cmul(I_NUM, pxm1)));
        const double2 A = cmul(a, ehi ? pt0 : cadd(pt0, pt1));
        double2 B = cmul(b, csub(px0, cmul(I_NUM, px1)));
        h0 = cadd(cadd(cadd(C, E), A), B);
        C = elo ? cneg(C) : cmul(c, cadd(cneg(pm0), pm1));
        E = cmul(e, cadd(cmul(MI_NUM, pxm0), pxm1));
        B = cmul(b, cadd(cmul(I_NUM, px0), px1));
        h1 = cadd(cadd(cadd(C, E), A), B);
    }
    s0 = csub(rmul(mass, p0), rmul(0.5, h0));
    s1 = csub(rmul(mass, p1), rmul(0.5, h1));
}

template <int DAG, int PROJ>
__device__ __forceinline__ void dslash_site(const DArgs &a, double sr0, double sl0, bool elo, bool ehi, const Row &cur,
                                            const Row &nx1, double2 pxm0, double2 pxm1, double2 uxm, double2 &s0,
                                            double2 &s1) {
    if (PROJ)
        dirac_site_proj<DAG>(a.mass, sr0, sl0, elo, ehi, cur.c0, cur.c1, cur.p0, cur.p1, nx1.c0, nx1.c1, cur.m0,
                             cur.m1, pxm0, pxm1, cur.ut, cur.ux, cur.utm, uxm, s0, s1);
    else
        dirac_site<DAG>(a.mass, sr0, sl0, cur.c0, cur.c1, cur.p0, cur.p1, nx1.c0, nx1.c1, cur.m0, cur.m1, pxm0, pxm1,
                        cur.ut, cur.ux, cur.utm, uxm, s0, s1);
}

// Marching loop with a two-row prefetch: at step x the loads of row x+2 are
// issued while row x is computed from rows x-1 (centre), x and x+1, which
// were loaded one and two steps earlier. xn/xs clamp at the chunk end so no
// load is ever conditional (re-reads there are cache hits).
template <int DAG, int EPI, int PREF, int PROJ = 0>
__device__ __forceinline__ void dslash_body(const DArgs &a) {
    __shared__ double2 sh[4];
    if (a.sc && a.sc->done) return;  // grid-uniform early exit after CG convergence
    int tb, xc;
    block_tile(blockIdx.x, a.tb0, a.tbn, a.TB, a.XB, a.xcd_remap, tb, xc);
    const int t = tb * blockDim.x + threadIdx.x;
    const int xbeg = xc * a.xchunk;
    const int xend = min(a.Nx, xbeg + a.xchunk);
    double2 acc = make_double2(0.0, 0.0);
    if (t < a.Wt && xbeg < xend) {
        const int Nx = a.Nx, Wt = a.Wt;
        const long V = a.V;
        const double sr0 = (a.t0 + t == a.Ntg - 1) ? -1.0 : 1.0;
        const double sl0 = (a.t0 + t == 0) ? -1.0 : 1.0;
        const LaneSrc L = lane_src(a, t);
        const bool elo = PROJ && t == 0, ehi = PROJ && t + 1 == Wt;  // lanes reading projected faces
        auto wrap = [Nx](int x) { return x >= Nx ? x - Nx : x; };
        const int xm = (xbeg == 0) ? Nx - 1 : xbeg - 1;
        const long nm = (long)xm * Wt + t;
        double2 pxm0 = a.in[nm], pxm1 = a.in[nm + V], uxm = a.U[nm + V];
        if (PREF == 1) {
            // one-row lookahead (fewer registers, more waves per SIMD)
            Row cur;
            load_row(a, L, xbeg, xbeg, t, cur);
            for (int x = xbeg; x < xend; ++x) {
                const int xp = (x + 1 == Nx) ? 0 : x + 1;
                const int xs = (x + 1 < xend) ? xp : x;
                const long n = (long)x * Wt + t;
                Row nxt;
                load_row(a, L, xp, xs, t, nxt);
                double2 ax0, ax1;
                if (EPI == EPI_DOT) {
                    ax0 = a.aux[n];
                    ax1 = a.aux[n + V];
                }
                double2 s0, s1;
                dslash_site<DAG, PROJ>(a, sr0, sl0, elo, ehi, cur, nxt, pxm0, pxm1, uxm, s0, s1);
                st_nt(a.out + n, s0);
                st_nt(a.out + n + V, s1);
                if (EPI == EPI_DOT) {
                    acc = cadd(acc, cmul(ax0, cconj(s0)));
                    acc = cadd(acc, cmul(ax1, cconj(s1)));
                }
                pxm0 = cur.c0;
                pxm1 = cur.c1;
                uxm = cur.ux;
                cur = nxt;
            }
        } else {
        // Three row registers used round-robin (manual 3-way unroll): the
        // rotation is a renaming, so no register copy waits on an in-flight load.
        Row R0, R1, R2;
        load_row(a, L, xbeg, xbeg, t, R0);
        load_row(a, L, wrap(xbeg + 1), min(xbeg + 1, xend - 1), t, R1);
        int x = xbeg;
        auto step = [&](Row &cur, const Row &nx1, Row &nx2) {
            const long n = (long)x * Wt + t;
            load_row(a, L, wrap(min(x + 2, xend)), min(x + 2, xend - 1), t, nx2);
            double2 ax0, ax1;
            if (EPI == EPI_DOT) {
                ax0 = a.aux[n];
                ax1 = a.aux[n + V];
            }
            double2 s0, s1;
            dslash_site<DAG, PROJ>(a, sr0, sl0, elo, ehi, cur, nx1, pxm0, pxm1, uxm, s0, s1);
            st_nt(a.out + n, s0);
            st_nt(a.out + n + V, s1);
            if (EPI == EPI_DOT) {
                // dot(aux, out) = sum aux * conj(out), include/variables.h:185-188
                acc = cadd(acc, cmul(ax0, cconj(s0)));
                acc = cadd(acc, cmul(ax1, cconj(s1)));
            }
            pxm0 = cur.c0;
            pxm1 = cur.c1;
            uxm = cur.ux;
        };
        for (;;) {
            step(R0, R1, R2);
            if (++x >= xend) break;
            step(R1, R2, R0);
            if (++x >= xend) break;
            step(R2, R0, R1);
            if (++x >= xend) break;
        }
        }
    }
    if (EPI == EPI_DOT) {
        double2 bs = block_sum(acc, sh);
        if (threadIdx.x == 0) a.partials[(long)tb * a.XB + xc] = bs;  // one slot per tile
    }
}

// Variants (LaunchCfg::variant): 0 = one-row lookahead; 1 = two-row
// lookahead, registers unconstrained (2 waves/SIMD); 2 = two-row lookahead
// capped at 168 VGPRs (3 waves/SIMD).
template <int DAG, int EPI>
__global__ void __launch_bounds__(256) dslash_kernel_v0(DArgs a) { dslash_body<DAG, EPI, 1>(a); }
template <int DAG, int EPI>
__global__ void __launch_bounds__(256) dslash_kernel_v1(DArgs a) { dslash_body<DAG, EPI, 2>(a); }
template <int DAG, int EPI>
__global__ void __launch_bounds__(256, 3) dslash_kernel_v2(DArgs a) { dslash_body<DAG, EPI, 2>(a); }
// t-shards with spin-projected faces (the two-row lookahead body of v1)
template <int DAG, int EPI>
__global__ void __launch_bounds__(256) dslash_kernel_proj(DArgs a) { dslash_body<DAG, EPI, 2, 1>(a); }

LaunchCfg dslash_config(const Geometry &g) {
    LaunchCfg c;
    c.bt = g.Wt >= 256 ? 256 : (g.Wt >= 128 ? 128 : 64);
    const int tb = (g.Wt + c.bt - 1) / c.bt;
    // 32-row marches where they give 256..4096 blocks, 16 rows above that,
    // else ~2048 blocks (tools/shape_tune.hip, profiles/r02_shape_tune.jsonl,
    // GB/s against the old 2048-block rule: 4096x2048 5648 vs 5157, 4096x512
    // 6581 vs 6128, 8192x1024 5432 vs 5048, 8192x8192 5486 vs 5363; 4096^2
    // is 32 rows either way)
    const long b32 = (long)tb * ((g.Nx + 31) / 32);
    const int target = 2048;
    if (b32 >= 256 && b32 <= 4096) {
        c.xchunk = 32;
    } else if (b32 > 4096) {
        c.xchunk = 16;
    } else {
        int nchunks = (target + tb - 1) / tb;
        if (nchunks > g.Nx) nchunks = g.Nx;
        if (nchunks < 1) nchunks = 1;
        c.xchunk = (g.Nx + nchunks - 1) / nchunks;
    }
    c.xcd_remap = 1;
    c.variant = 1;  // two-row lookahead: 296 vs 315 us at 4096^2 (profiles/r01)
    return c;
}

int dslash_blocks(const Geometry &g, const LaunchCfg &c) {
    const int tb = (g.Wt + c.bt - 1) / c.bt;
    const int xb = (g.Nx + c.xchunk - 1) / c.xchunk;
    return tb * xb;
}

void launch_dslash(hipStream_t s, const Geometry &g, const LaunchCfg &c, int dagger,
                   const double2 *in, double2 *out, const double2 *U, const double2 *loU,
                   const TFaces &f, double mass, const double2 *aux, double2 *partials,
                   const CGScalars *skip_if_done, int tb0, int tbn) {
    DArgs a;
    a.in = in;
    a.out = out;
    a.U = U;
    a.loU = loU;
    a.f = f;
    a.aux = aux;
    a.partials = partials;
    a.sc = skip_if_done;
    a.V = g.V;
    a.Nx = g.Nx;
    a.Wt = g.Wt;
    a.t0 = g.t0;
    a.Ntg = g.Ntg;
    a.xchunk = c.xchunk;
    a.TB = (g.Wt + c.bt - 1) / c.bt;
    a.XB = (g.Nx + c.xchunk - 1) / c.xchunk;
    a.xcd_remap = c.xcd_remap;
    a.mass = mass;
    if (tbn < 0) {
        tb0 = 0;
        tbn = a.TB;
    }
    if (tbn == 0) return;
    a.tb0 = tb0;
    a.tbn = tbn;
    a.part0 = tb0 * a.XB;
    dim3 grid(tbn * a.XB);
    dim3 block(c.bt);
    const bool dot = aux != nullptr;
#define SM_LAUNCH(K)                                                                    \
    do {                                                                                \
        if (!dagger) {                                                                  \
            if (dot) hipLaunchKernelGGL((K<0, EPI_DOT>), grid, block, 0, s, a);         \
            else hipLaunchKernelGGL((K<0, EPI_NONE>), grid, block, 0, s, a);            \
        } else {                                                                        \
            if (dot) hipLaunchKernelGGL((K<1, EPI_DOT>), grid, block, 0, s, a);         \
            else hipLaunchKernelGGL((K<1, EPI_NONE>), grid, block, 0, s, a);            \
        }                                                                               \
    } while (0)
    if (f.proj) SM_LAUNCH(dslash_kernel_proj);
    else if (c.variant == 1) SM_LAUNCH(dslash_kernel_v1);
    else if (c.variant == 2) SM_LAUNCH(dslash_kernel_v2);
    else SM_LAUNCH(dslash_kernel_v0);
#undef SM_LAUNCH
}

// ---- fermion force bilinear (eqs. 37-38; src/dirac_operator.cpp:493-506) ----
struct FArgs {
    const double2 *U, *l, *r;
    TFaces fl, fr;   // only .hi is used: forward-only stencil
    double *F;
    long V;
    int Nx, Wt, t0, Ntg;
};

__global__ void __launch_bounds__(256) force_kernel(FArgs a) {
    const long V = a.V;
    for (long n = (long)blockIdx.x * blockDim.x + threadIdx.x; n < V; n += (long)gridDim.x * blockDim.x) {
        const int x = (int)(n / a.Wt), t = (int)(n - (long)x * a.Wt);
        const long nx = (long)((x + 1 == a.Nx) ? 0 : x + 1) * a.Wt + t;
        const double2 SR0 = make_double2((a.t0 + t == a.Ntg - 1) ? -1.0 : 1.0, 0.0);
        const double2 SR1 = make_double2(1.0, 0.0);
        const double2 U = a.U[n], W = a.U[n + V];
        const double2 L0 = a.l[n], L1 = a.l[n + V], R0 = a.r[n], R1 = a.r[n + V];
        double2 lsum, rdif;   // l0 + l1 and r0 - r1 at n + t^
        if (t + 1 < a.Wt) {
            lsum = cadd(a.l[n + 1], a.l[n + 1 + V]);
            rdif = csub(a.r[n + 1], a.r[n + 1 + V]);
        } else {
            const double2 *pl = a.fl.hi + (long)x * a.fl.hi_xs, *pr = a.fr.hi + (long)x * a.fr.hi_xs;
            // projected faces (t-shards) carry the combinations themselves
            lsum = a.fl.proj ? pl[0] : cadd(pl[0], pl[a.fl.hi_ps]);
            rdif = a.fr.proj ? pr[0] : csub(pr[0], pr[a.fr.hi_ps]);
        }
        // mu = 0
        double2 P = cmul(cmul(cmul(U, SR0), cconj(csub(L0, L1))), rdif);
        double2 Q = cmul(cmul(cmul(cconj(U), SR0), cconj(lsum)), cadd(R0, R1));
        a.F[n] = csub(P, Q).y;
        // mu = 1
        const double2 lx0 = a.l[nx], lx1 = a.l[nx + V], rx0 = a.r[nx], rx1 = a.r[nx + V];
        P = cmul(cmul(cmul(W, SR1), csub(cconj(L0), cmul(I_NUM, cconj(L1)))), cadd(rx0, cmul(I_NUM, rx1)));
        Q = cmul(cmul(cmul(cconj(W), SR1), cadd(cconj(lx0), cmul(I_NUM, cconj(lx1)))),
                 cadd(cneg(R0), cmul(I_NUM, R1)));
        a.F[n + V] = cadd(P, Q).y;
    }
}

void launch_force(hipStream_t s, const Geometry &g, const double2 *U, const double2 *l,
                  const double2 *r, const TFaces &fl, const TFaces &fr, double *F) {
    FArgs a;
    a.U = U; a.l = l; a.r = r; a.fl = fl; a.fr = fr; a.F = F;
    a.V = g.V; a.Nx = g.Nx; a.Wt = g.Wt; a.t0 = g.t0; a.Ntg = g.Ntg;
    long nb = (g.V + 255) / 256;
    if (nb > 4096) nb = 4096;
    hipLaunchKernelGGL(force_kernel, dim3((unsigned)nb), dim3(256), 0, s, a);
}

// ---- BLAS-1 / CG ------------------------------------------------------------
// All reductions: fixed grid, per-thread grid-stride partial (fixed order),
// deterministic block sum, then a single-block fixed-order sum of partials.
// Results are run-to-run reproducible (not the reference's sequential order:
// CG parity is on the converged solution).
constexpr int RB = 256;  // threads per reduction block

int reduce_blocks(long n) {
    long nb = (n + RB * 4 - 1) / (RB * 4);
    if (nb > 2048) nb = 2048;
    if (nb < 1) nb = 1;
    return (int)nb;
}

// Streaming loop over this block's chunk: f(i) for every i, 4 lane-tiles per
// step so 4 independent 16-B accesses per operand are in flight.
template <typename F>
__device__ __forceinline__ void chunk_loop(long n, F f) {
    const Chunk c = block_chunk(n);
    long i = c.beg + threadIdx.x;
    for (; i + 3 * RB < c.end; i += 4 * RB) {
        f(i);
        f(i + RB);
        f(i + 2 * RB);
        f(i + 3 * RB);
    }
    for (; i < c.end; i += RB) f(i);
}

__global__ void __launch_bounds__(RB) dot_partial_kernel(long n, const double2 *a, const double2 *b,
                                                         double2 *part) {
    __shared__ double2 sh[RB / 64];
    double2 acc = make_double2(0.0, 0.0);
    chunk_loop(n, [&](long i) { acc = cadd(acc, cmul(ld_nt(a + i), cconj(ld_nt(b + i)))); });
    double2 s = block_sum(acc, sh);
    if (threadIdx.x == 0) part[blockIdx.x] = s;
}

__global__ void __launch_bounds__(RB) sum_partials_kernel(int nparts, const double2 *part, double2 *out) {
    __shared__ double2 sh[RB / 64];
    double2 s = sum_partials_block(nparts, part, sh);
    if (threadIdx.x == 0) *out = s;
}

void launch_dot_partial(hipStream_t s, long n, const double2 *a, const double2 *b, double2 *partials) {
    hipLaunchKernelGGL(dot_partial_kernel, dim3(reduce_blocks(n)), dim3(RB), 0, s, n, a, b, partials);
}

void launch_sum_partials(hipStream_t s, int nparts, const double2 *partials, double2 *out) {
    hipLaunchKernelGGL(sum_partials_kernel, dim3(1), dim3(RB), 0, s, nparts, partials, out);
}

__global__ void __launch_bounds__(RB) copy_kernel(long n, const double2 *src, double2 *dst) {
    chunk_loop(n, [&](long i) { st_nt(dst + i, ld_nt(src + i)); });
}

void launch_copy(hipStream_t s, long n, const double2 *src, double2 *dst) {
    hipLaunchKernelGGL(copy_kernel, dim3(reduce_blocks(n)), dim3(RB), 0, s, n, src, dst);
}

// r = phi - Ax; d = r; partials of <r,r> and <phi,phi>  (src/conjugate_gradient.cpp:19-29)
__global__ void __launch_bounds__(RB) cg_init_kernel(long n, const double2 *phi, const double2 *Ax,
                                                     double2 *r, double2 *d, double2 *prr,
                                                     double2 *ppp) {
    __shared__ double2 sh[RB / 64];
    double2 arr = make_double2(0.0, 0.0), app = make_double2(0.0, 0.0);
    chunk_loop(n, [&](long i) {
        const double2 p = ld_nt(phi + i);
        const double2 ri = csub(p, ld_nt(Ax + i));
        st_nt(r + i, ri);
        st_nt(d + i, ri);
        arr = cadd(arr, cmul(ri, cconj(ri)));
        app = cadd(app, cmul(p, cconj(p)));
    });
    double2 s1 = block_sum(arr, sh);
    __syncthreads();
    double2 s2 = block_sum(app, sh);
    if (threadIdx.x == 0) {
        prr[blockIdx.x] = s1;
        ppp[blockIdx.x] = s2;
    }
}

void launch_cg_init(hipStream_t s, long n, const double2 *phi, const double2 *Ax, double2 *r,
                    double2 *d, double2 *part_rr, double2 *part_pp) {
    hipLaunchKernelGGL(cg_init_kernel, dim3(reduce_blocks(n)), dim3(RB), 0, s, n, phi, Ax, r, d,
                       part_rr, part_pp);
}

__device__ __forceinline__ void cg_init_scalars(CGScalars *sc, double2 rr, double2 pp, double tol) {
    sc->rn = rr;
    sc->phi_norm = sqrt(pp.x);
    sc->tol = tol;
    sc->err = 0.0;
    sc->k = 0;
    sc->done = 0;
    sc->converged = 0;
    sc->max_iter = 0x7fffffff;  // sm_cg_dev sets the caller's limit (one-pass path)
    sc->alpha = sc->beta = sc->alpha2 = sc->beta2 = make_double2(0.0, 0.0);
    CGRed s0;                   // S_-1 of the redundant-scalar path
    s0.rn = rr;
    s0.alpha = s0.beta = make_double2(0.0, 0.0);
    s0.alpha2 = s0.beta2 = make_double2(0.0, 0.0);
    s0.err = 0.0;
    s0.k = s0.done = s0.converged = s0.pad = 0;
    sc->red[0] = s0;
    sc->red[1] = s0;
}

__global__ void __launch_bounds__(RB) cg_finalize_init_kernel(int nparts, const double2 *prr,
                                                              const double2 *ppp, CGScalars *sc,
                                                              double tol) {
    __shared__ double2 sh[RB / 64];
    double2 rr = sum_partials_block(nparts, prr, sh);
    __syncthreads();
    double2 pp = sum_partials_block(nparts, ppp, sh);
    if (threadIdx.x == 0) cg_init_scalars(sc, rr, pp, tol);
}

void launch_cg_finalize_init(hipStream_t s, int nparts, const double2 *part_rr,
                             const double2 *part_pp, CGScalars *sc, double tol) {
    hipLaunchKernelGGL(cg_finalize_init_kernel, dim3(1), dim3(RB), 0, s, nparts, part_rr, part_pp, sc, tol);
}

__global__ void __launch_bounds__(RB) cg_alpha_kernel(int nparts, const double2 *part, CGScalars *sc) {
    __shared__ double2 sh[RB / 64];
    if (sc->done) return;
    double2 s = sum_partials_block(nparts, part, sh);
    if (threadIdx.x == 0) cg_alpha_scalar(sc, s);
}

void launch_cg_alpha(hipStream_t s, int nparts, const double2 *part, CGScalars *sc) {
    hipLaunchKernelGGL(cg_alpha_kernel, dim3(1), dim3(RB), 0, s, nparts, part, sc);
}

// x += alpha d; r -= alpha Ad; partial <r,r>   (src/conjugate_gradient.cpp:34-43)
__global__ void __launch_bounds__(RB) cg_update_xr_kernel(long n, double2 *x, double2 *r,
                                                          const double2 *d, const double2 *Ad,
                                                          const CGScalars *sc, double2 *part) {
    __shared__ double2 sh[RB / 64];
    if (sc->done) return;
    const double2 alpha = sc->alpha;
    double2 acc = make_double2(0.0, 0.0);
    chunk_loop(n, [&](long i) {
        st_nt(x + i, cadd(ld_nt(x + i), cmul(alpha, ld_nt(d + i))));
        const double2 ri = csub(ld_nt(r + i), cmul(alpha, ld_nt(Ad + i)));
        st_nt(r + i, ri);
        acc = cadd(acc, cmul(ri, cconj(ri)));
    });
    double2 s = block_sum(acc, sh);
    if (threadIdx.x == 0) part[blockIdx.x] = s;
}

void launch_cg_update_xr(hipStream_t s, long n, double2 *x, double2 *r, const double2 *d,
                         const double2 *Ad, CGScalars *sc, double2 *part) {
    hipLaunchKernelGGL(cg_update_xr_kernel, dim3(reduce_blocks(n)), dim3(RB), 0, s, n, x, r, d, Ad, sc, part);
}

__global__ void __launch_bounds__(RB) cg_beta_kernel(int nparts, const double2 *part, CGScalars *sc) {
    __shared__ double2 sh[RB / 64];
    if (sc->done) return;
    double2 s = sum_partials_block(nparts, part, sh);
    if (threadIdx.x == 0) cg_beta_scalar(sc, s);
}

void launch_cg_beta(hipStream_t s, int nparts, const double2 *part, CGScalars *sc) {
    hipLaunchKernelGGL(cg_beta_kernel, dim3(1), dim3(RB), 0, s, nparts, part, sc);
}

// d = d*beta + r   (src/conjugate_gradient.cpp:54-59)
__global__ void __launch_bounds__(RB) cg_update_d_kernel(long n, double2 *d, const double2 *r,
                                                         const CGScalars *sc) {
    if (sc->done) return;
    const double2 beta = sc->beta;
    chunk_loop(n, [&](long i) { st_nt(d + i, cadd(cmul(ld_nt(d + i), beta), ld_nt(r + i))); });
}

void launch_cg_update_d(hipStream_t s, long n, double2 *d, const double2 *r, const CGScalars *sc) {
    hipLaunchKernelGGL(cg_update_d_kernel, dim3(reduce_blocks(n)), dim3(RB), 0, s, n, d, r, sc);
}

// ---- multi-GPU variants: local partial sum -> (RCCL allreduce) -> scalar ----
__global__ void __launch_bounds__(RB) sum_to_scalar_kernel(int nparts, const double2 *part, CGScalars *sc) {
    __shared__ double2 sh[RB / 64];
    if (sc->done) return;
    double2 s = sum_partials_block(nparts, part, sh);
    if (threadIdx.x == 0) sc->sum = s;
}

void launch_sum_to_scalar(hipStream_t s, int nparts, const double2 *part, CGScalars *sc) {
    hipLaunchKernelGGL(sum_to_scalar_kernel, dim3(1), dim3(RB), 0, s, nparts, part, sc);
}

__global__ void cg_alpha_from_sum_kernel(CGScalars *sc) {
    if (sc->done) return;
    cg_alpha_scalar(sc, sc->sum);
}
__global__ void cg_beta_from_sum_kernel(CGScalars *sc) {
    if (sc->done) return;
    cg_beta_scalar(sc, sc->sum);
}
__global__ void cg_init_from_sums_kernel(const double2 *rr_pp, CGScalars *sc, double tol) {
    cg_init_scalars(sc, rr_pp[0], rr_pp[1], tol);
}

void launch_cg_alpha_from_sum(hipStream_t s, CGScalars *sc) {
    hipLaunchKernelGGL(cg_alpha_from_sum_kernel, dim3(1), dim3(1), 0, s, sc);
}
void launch_cg_beta_from_sum(hipStream_t s, CGScalars *sc) {
    hipLaunchKernelGGL(cg_beta_from_sum_kernel, dim3(1), dim3(1), 0, s, sc);
}
void launch_cg_init_from_sums(hipStream_t s, const double2 *rr_pp, CGScalars *sc, double tol) {
    hipLaunchKernelGGL(cg_init_from_sums_kernel, dim3(1), dim3(1), 0, s, rr_pp, sc, tol);
}

// ---- bandwidth ceilings (measured roofline reference) --------------------------
// out = a + b over n complex (2 reads + 1 write, the dslash byte mix) or
// out = a (1 read + 1 write); 4 independent 16-B loads per lane in flight.
template <int TWO>
__global__ void __launch_bounds__(256) stream_kernel(long n, const double2 *__restrict__ a,
                                                     const double2 *__restrict__ b,
                                                     double2 *__restrict__ out) {
    // the measured-best streaming form (tools/membench.hip): block-contiguous
    // chunks, 4 tiles in flight, non-temporal loads and stores
    chunk_loop(n, [&](long i) {
        double2 v = ld_nt(a + i);
        if (TWO) v = cadd(v, ld_nt(b + i));
        st_nt(out + i, v);
    });
}

void launch_stream(hipStream_t s, int two, long n, const double2 *a, const double2 *b, double2 *out,
                   int blocks) {
    if (blocks <= 0) blocks = 2048;
    if (two) hipLaunchKernelGGL(stream_kernel<1>, dim3(blocks), dim3(256), 0, s, n, a, b, out);
    else hipLaunchKernelGGL(stream_kernel<0>, dim3(blocks), dim3(256), 0, s, n, a, b, out);
}

// ---- halo faces ---------------------------------------------------------------
__global__ void pack_faces_kernel(int Nx, int Wt, long V, const double2 *f, double2 *lo, double2 *hi) {
    const int x = blockIdx.x * blockDim.x + threadIdx.x;
    if (x >= Nx) return;
    const long a = (long)x * Wt, b = (long)x * Wt + Wt - 1;
    lo[x] = f[a];
    lo[x + Nx] = f[a + V];
    hi[x] = f[b];
    hi[x + Nx] = f[b + V];
}

void launch_pack_faces(hipStream_t s, const Geometry &g, const double2 *field, double2 *lo_face,
                       double2 *hi_face) {
    hipLaunchKernelGGL(pack_faces_kernel, dim3((g.Nx + 63) / 64), dim3(64), 0, s, g.Nx, g.Wt, g.V,
                       field, lo_face, hi_face);
}

// Spin-projected faces (TFaces::proj): lo = my t = 0 column's forward-hop
// combination (it is the down-neighbour's t = Wt), hi = conj(U_t(t = Wt-1))
// times my t = Wt-1 column's backward-hop combination (the up-neighbour's
// t = -1 hop, without its antiperiodic sign). The sums and the product are the
// reference's own (src/dirac_operator.cpp:31-43, 255-267; force :493-506).
// Face packs: one thread per row x, strided loads (a row apart), so they are
// latency-bound; 64-thread blocks spread the Nx threads over 4x as many CUs.
// One thread per (x, side): side 0 forms the lo face from column 0, side 1 the
// hi face from column Wt-1 (with its link). The loads are one site per row,
// Wt sites apart, so the kernel is latency-bound: 2 Nx threads in 256-wide
// blocks put every load in flight at once (round 4's one thread per x, in
// 64-wide blocks: 6 us at Nx = 4096 on the RCCL loopback timeline).
__global__ void __launch_bounds__(256) pack_faces_proj_kernel(int Nx, int Wt, long V, const double2 *f,
                                                              const double2 *U, int kind, double2 *lo,
                                                              double2 *hi) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= 2 * Nx) return;
    const int x = i >> 1, side = i & 1;
    const long n = (long)x * Wt + (side ? Wt - 1 : 0);
    const double2 p0 = f[n], p1 = f[n + V];
    const double2 v = proj_face_value(kind, side, p0, p1, U + n);
    if (!side) lo[x] = v;
    else hi[x] = v;
}

void launch_pack_faces_proj(hipStream_t s, const Geometry &g, const double2 *field, const double2 *U, int kind,
                            double2 *lo_face, double2 *hi_face) {
    hipLaunchKernelGGL(pack_faces_proj_kernel, dim3((2 * g.Nx + 255) / 256), dim3(256), 0, s, g.Nx, g.Wt, g.V, field,
                       U, kind, lo_face, hi_face);
}

}  // namespace sm
