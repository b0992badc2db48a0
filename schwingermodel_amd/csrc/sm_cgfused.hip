// sm_cgfused.hip -- the two-direction one-pass CG iteration with a stored Ad
// (gfx950), the default below 256^2 sites per shard (mode 4 of sm_tune_cg),
// plus the CG scalar kernels shared with the recompute-Ad pass (sm_cgra.hip).
//
// Reference loop body (src/conjugate_gradient.cpp:31-63), iteration k:
//     Ad = D D^dag d_k ; alpha_k = rn / <d_k, Ad> ; x += alpha_k d_k ;
//     r -= alpha_k Ad ; err = |r| ; stop? ; beta_k = err^2 / rn ; d_{k+1} = d_k beta_k + r
// Pass j (j >= 1), every per-element operation the reference's:
//     r_{j-1} = d_{j-1} - d_{j-2} beta_{j-2}         (the reference's d *= beta; d += r, :55-58)
//     r_j     = r_{j-1} - alpha_{j-1} Ad_{j-1}       (:38-39)
//     d_j     = d_{j-1} beta_{j-1} + r_j             (:55-58)
//     x      <- (x + alpha_{j-2} d_{j-2}) + alpha_{j-1} d_{j-1}   on even j (:36-37)
//     Ad_j    = D D^dag d_j ; partials of <d_j,Ad_j>, <r_j,Ad_j>, |r_j|^2, |Ad_j|^2
// Then (cg1_scalar_kernel): err = sqrt|r_j|^2 (direct, as the reference) and its
// stop test; alpha_j = |r_j|^2 / <d_j,Ad_j>; and beta_j from the expansion
//     |r_{j+1}|^2 = |r_j|^2 - 2 Re(conj(alpha_j) <r_j,Ad_j>) + |alpha_j|^2 |Ad_j|^2
// of the pass's own direct dots (no conjugacy assumed), so r_{j+1} never has
// to be written before d_{j+1} is formed. Pass 0 only forms Ad_0 (d_0 = r_0).
// No r vector is stored: d rotates through three buffers, Ad ping-pongs (halo
// lanes / rows of neighbouring tiles read the j-1 fields while owners write
// the j fields). HBM bytes per site: read d_{j-1}, d_{j-2}, Ad_{j-1}, U (128),
// write d_j, Ad_j (64), plus read and write x on even passes: 224 mean,
// against 576 for the reference's sequence.
//
// Geometry: a wave owns 60 consecutive t-columns; its 64 lanes cover columns
// T0-2 .. T0+61 (2 halo lanes per side) and march along x. The t-neighbours of
// the intermediates (d_j, T, U_t) come from adjacent lanes through DPP
// wave-shifts; the x-neighbours are register rows. Halo lanes compute and are
// discarded, so waves are independent (no LDS, no barrier in the loop).
#include "sm_device.h"
#include "sm_internal.h"

#pragma clang fp contract(off)

namespace sm {

constexpr int FW = kFusedWaveCols;  // output t-columns per wave

struct CSrc {
    const double2 *p;
    long xs, ps;
};

struct CG1Args {
    const double2 *dold, *rold, *aold;  // d_{j-1}, d_{j-2}, Ad_{j-1}
    double2 *dnew, *anew;               // d_j, Ad_j
    double2 *x;
    const double2 *U;
    const double2 *fd, *fr, *fa, *fU;  // t-shards: 2-deep faces [-2,-1,Wt,Wt+1][plane][x]
    CGScalars *sc;
    double2 *partials;                 // 3 per block: <d,Ad>, <r,Ad>, (|r|^2, |Ad|^2)
    const double2 *prev;               // != null: redundant scalars from pass j-1's partials
    long pass;                         // j
    long V;
    int Nx, Wt, t0, Ntg, nshard;
    int xchunk, NWT, TBk, XB, remap, first;
    int tb0, tbn;
    double mass;
};

struct Raw3 {
    double2 d0, d1, r0, r1, a0, a1, ut, ux, x0, x1;
};

// Where column c of a field lives: in-domain, periodic wrap (one shard), or
// the received face (t-shard). Clamped so every lane's address is valid.
__device__ __forceinline__ CSrc csrc1(const double2 *base, const double2 *face, int c, const CG1Args &a) {
    CSrc s;
    if (c >= 0 && c < a.Wt) {
        s.p = base + c;
        s.xs = a.Wt;
        s.ps = a.V;
    } else if (a.nshard == 1) {
        int cw = c % a.Wt;
        if (cw < 0) cw += a.Wt;
        s.p = base + cw;
        s.xs = a.Wt;
        s.ps = a.V;
    } else {
        int fc = c < 0 ? c + 2 : c - a.Wt + 2;
        fc = fc < 0 ? 0 : (fc > 3 ? 3 : fc);
        s.p = face + (long)fc * 2 * a.Nx;
        s.xs = 1;
        s.ps = a.Nx;
    }
    return s;
}

// RED: redundant scalars (a.prev != null): every block evaluates pass j-1's
// scalars itself; its own instance keeps that code out of the large-grid kernel.
// XP: x takes the updates of passes j-1 and j together (even passes).
template <int RED, int XP>
__global__ void __launch_bounds__(256) cg_onepass_kernel(CG1Args a) {
    __shared__ double2 sh[4];
    CGScalars *sc = a.sc;
    double2 alpha, beta;                               // alpha_{j-1}, beta_{j-1}
    double2 alpha2, beta2;                             // alpha_{j-2}, beta_{j-2}
    if (RED) {
        __shared__ double2 s_ab[4];
        __shared__ int s_stop;
        if (!a.first) {
            const CGRed s = cg1_redundant(sc, a.prev, (int)gridDim.x, a.pass, sh);
            if (threadIdx.x == 0) {
                s_ab[0] = s.alpha;
                s_ab[1] = s.beta;
                s_ab[2] = s.alpha2;
                s_ab[3] = s.beta2;
                s_stop = s.done;
            }
        } else if (threadIdx.x == 0) {
            s_stop = 0;
        }
        __syncthreads();
        if (s_stop) return;                            // block-uniform
        alpha = s_ab[0];
        beta = s_ab[1];
        alpha2 = s_ab[2];
        beta2 = s_ab[3];
    } else {
        if (sc->done) return;  // grid-uniform: converged (or max_iter) in an earlier pass
        alpha = sc->alpha;
        beta = sc->beta;
        alpha2 = sc->alpha2;
        beta2 = sc->beta2;
    }
    int tb, xc;
    {
        int w = blockIdx.x;
        if (a.remap) {
            const int n = a.tbn * a.XB, q = n >> 3, rr = n & 7, xcd = w & 7;
            w = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (w >> 3);
        }
        tb = a.tb0 + w % a.tbn;
        if (tb >= a.TBk) tb -= a.TBk;  // edge block-columns TBk-1 and 0 in one launch
        xc = w / a.tbn;
    }
    const int lane = threadIdx.x & 63;
    const int g = tb * 4 + (threadIdx.x >> 6);
    const int x0 = xc * a.xchunk;
    const int xe = min(a.Nx, x0 + a.xchunk);
    double2 acc_dA = make_double2(0.0, 0.0), acc_rA = make_double2(0.0, 0.0);
    double2 acc_n = make_double2(0.0, 0.0);  // (|r|^2, |Ad|^2)
    if (g < a.NWT && x0 < xe) {
        const int Nx = a.Nx, Wt = a.Wt;
        const int c = g * FW - 2 + lane;
        const bool own = lane >= 2 && lane < FW + 2 && c < Wt;
        int tg = (a.t0 + c) % a.Ntg;
        if (tg < 0) tg += a.Ntg;
        const double sr0 = tg == a.Ntg - 1 ? -1.0 : 1.0;  // SignR[2n], include/dirac_operator.h:53-55
        const double sl0 = tg == 0 ? -1.0 : 1.0;          // SignL[2n], :56-58
        const CSrc Sd = csrc1(a.dold, a.fd, c, a), Sr = csrc1(a.rold, a.fr, c, a);
        const CSrc Sa = csrc1(a.aold, a.fa, c, a), Su = csrc1(a.U, a.fU, c, a);
        const int cx = c < 0 ? 0 : (c >= Wt ? Wt - 1 : c);
        const bool first = a.first != 0;
        auto wrap = [Nx](int x) { int w = x % Nx; return w < 0 ? w + Nx : w; };
        auto load = [&](int xr, Raw3 &R) {
            const long pr = (long)wrap(xr);
            const double2 *pd = Sd.p + pr * Sd.xs, *pq = Sr.p + pr * Sr.xs, *pa = Sa.p + pr * Sa.xs;
            R.d0 = pd[0];
            R.d1 = pd[Sd.ps];
            R.r0 = pq[0];
            R.r1 = pq[Sr.ps];
            R.a0 = pa[0];
            R.a1 = pa[Sa.ps];
            const double2 *pu = Su.p + (long)wrap(min(xr, xe)) * Su.xs;
            R.ut = pu[0];
            R.ux = pu[Su.ps];
            if (XP) {
                const long nx = (long)wrap(min(max(xr, x0), xe - 1)) * Wt + cx;
                R.x0 = a.x[nx];
                R.x1 = a.x[nx + a.V];
            }
        };
        const bool rebuild = a.pass >= 2;  // pass 1 has r_0 = d_0 (no d_{-1})
        // r_j and d_j of row xr; on owned rows store d_j, x_j, add |r_j|^2
        auto form = [&](int xr, const Raw3 &R, Sp &rj) {
            Sp rp;  // r_{j-1}: d_{j-1} = d_{j-2} beta_{j-2} + r_{j-1}
            rp.a = rebuild ? csub(R.d0, cmul(R.r0, beta2)) : R.d0;
            rp.b = rebuild ? csub(R.d1, cmul(R.r1, beta2)) : R.d1;
            rj.a = first ? rp.a : csub(rp.a, cmul(alpha, R.a0));
            rj.b = first ? rp.b : csub(rp.b, cmul(alpha, R.a1));
            Sp d;
            d.a = first ? R.d0 : cadd(cmul(R.d0, beta), rj.a);
            d.b = first ? R.d1 : cadd(cmul(R.d1, beta), rj.b);
            if (xr >= x0 && xr < xe && own) {
                const long n = (long)xr * Wt + c;
                st_nt(a.dnew + n, d.a);
                st_nt(a.dnew + n + a.V, d.b);
                if (XP) {  // x_j = (x_{j-2} + alpha_{j-2} d_{j-2}) + alpha_{j-1} d_{j-1}
                    st_nt(a.x + n, cadd(cadd(R.x0, cmul(alpha2, R.r0)), cmul(alpha, R.d0)));
                    st_nt(a.x + n + a.V, cadd(cadd(R.x1, cmul(alpha2, R.r1)), cmul(alpha, R.d1)));
                }
                acc_n.x += cmul(rj.a, cconj(rj.a)).x;  // Re dot(r, r), include/variables.h:185-188
                acc_n.x += cmul(rj.b, cconj(rj.b)).x;
            }
            return d;
        };
        auto ddag = [&](const Sp &p, const Sp &pxm, const Sp &pxp, double2 ut, double2 ux, double2 uxm,
                        double2 &utm_out) {
            const Sp pm = shr(p), pp = shl(p);
            utm_out = dpp_shr1(ut);
            Sp o;
            dirac_site<1>(a.mass, sr0, sl0, p.a, p.b, pp.a, pp.b, pxp.a, pxp.b, pm.a, pm.b, pxm.a, pxm.b, ut, ux,
                          utm_out, uxm, o.a, o.b);
            return o;
        };
        Raw3 R;
        Sp rj;
        load(x0 - 2, R);
        Sp dm2 = form(x0 - 2, R, rj);
        double2 uxm2 = R.ux;
        load(x0 - 1, R);
        Sp dm1 = form(x0 - 1, R, rj);
        double2 utm1 = R.ut, uxm1 = R.ux;
        load(x0, R);
        Sp rc;
        Sp dc = form(x0, R, rc);
        double2 utc = R.ut, uxc = R.ux;
        load(x0 + 1, R);
        Sp rn;
        Sp dn = form(x0 + 1, R, rn);
        double2 utn = R.ut, uxn = R.ux;
        load(x0 + 2, R);
        double2 dummy;
        Sp Tp = ddag(dm1, dm2, dc, utm1, uxm1, uxm2, dummy);
        double2 utmc;
        Sp Tc = ddag(dc, dm1, dn, utc, uxc, uxm1, utmc);
        double2 uxp = uxm1;
        for (int x = x0; x < xe; ++x) {
            Sp r2;
            const Sp d2 = form(x + 2, R, r2);
            const double2 ut2 = R.ut, ux2 = R.ux;
            load(min(x + 3, xe + 1), R);
            __builtin_amdgcn_sched_barrier(0);
            double2 utmn;
            const Sp Tn = ddag(dn, dc, d2, utn, uxn, uxc, utmn);
            const Sp Tm = shr(Tc), Tq = shl(Tc);
            Sp o;
            dirac_site<0>(a.mass, sr0, sl0, Tc.a, Tc.b, Tq.a, Tq.b, Tn.a, Tn.b, Tm.a, Tm.b, Tp.a, Tp.b, utc, uxc,
                          utmc, uxp, o.a, o.b);
            if (own) {
                const long n = (long)x * Wt + c;
                st_nt(a.anew + n, o.a);
                st_nt(a.anew + n + a.V, o.b);
                acc_dA = cadd(acc_dA, cmul(dc.a, cconj(o.a)));  // dot(d, Ad)
                acc_dA = cadd(acc_dA, cmul(dc.b, cconj(o.b)));
                acc_rA = cadd(acc_rA, cmul(rc.a, cconj(o.a)));  // dot(r, Ad)
                acc_rA = cadd(acc_rA, cmul(rc.b, cconj(o.b)));
                acc_n.y += cmul(o.a, cconj(o.a)).x;            // |Ad|^2
                acc_n.y += cmul(o.b, cconj(o.b)).x;
            }
            Tp = Tc;
            Tc = Tn;
            dc = dn;
            dn = d2;
            rc = rn;
            rn = r2;
            uxp = uxc;
            utc = utn;
            uxc = uxn;
            utmc = utmn;
            utn = ut2;
            uxn = ux2;
        }
    }
    const double2 s0 = block_sum(acc_dA, sh);
    __syncthreads();
    const double2 s1 = block_sum(acc_rA, sh);
    __syncthreads();
    const double2 s2 = block_sum(acc_n, sh);
    if (threadIdx.x == 0) {  // one slot per tile (also the redundant path: read by the next launch)
        double2 *p = a.partials + 3 * ((long)tb * a.XB + xc);
        p[0] = s0;
        p[1] = s1;
        p[2] = s2;
    }
}

// Scalars after pass j: a single block sums the 3*nparts partials in a fixed
// order (1024 threads, four independent loads in flight per thread).
constexpr int SB = 1024;
__device__ void sum3_partials(int nparts, const double2 *part, double2 out[3]) {
    __shared__ double2 sh[3][SB / 64];
    double2 acc[3] = {make_double2(0.0, 0.0), make_double2(0.0, 0.0), make_double2(0.0, 0.0)};
    // a thread's partials i = tid, tid + SB, ... summed in that order; up to
    // four of them loaded together (one memory latency instead of four)
    constexpr int K = 4;
    for (int base = threadIdx.x; base < nparts; base += K * SB) {
        double2 v[K][3];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const int i = base + k * SB;
            if (i < nparts) {
                const double2 *p = part + 3 * (long)i;
                v[k][0] = p[0];
                v[k][1] = p[1];
                v[k][2] = p[2];
            }
        }
#pragma unroll
        for (int k = 0; k < K; ++k)
            if (base + k * SB < nparts) {
                acc[0] = cadd(acc[0], v[k][0]);
                acc[1] = cadd(acc[1], v[k][1]);
                acc[2] = cadd(acc[2], v[k][2]);
            }
    }
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
    for (int q = 0; q < 3; ++q) {
        double2 v = acc[q];
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            v.x += __shfl_xor(v.x, off);
            v.y += __shfl_xor(v.y, off);
        }
        if (lane == 0) sh[q][wid] = v;
    }
    __syncthreads();
    if (threadIdx.x == 0)
#pragma unroll
        for (int q = 0; q < 3; ++q) {
            double2 r = make_double2(0.0, 0.0);
            for (int w = 0; w < SB / 64; ++w) r = cadd(r, sh[q][w]);
            out[q] = r;
        }
}

__device__ __attribute__((noinline)) void cg1_scalars(CGScalars *sc, int first, double2 dA, double2 rA, double2 nn) {
    cg1_update(sc, first, dA, rA, nn);
}

// Redundant-scalar path: S_J of the last issued pass J into red[J & 1] and the
// host-visible fields (the next pass recomputes exactly the same S_J).
__global__ void __launch_bounds__(256) cg1_flush_kernel(int nparts, const double2 *part, CGScalars *sc, long J) {
    __shared__ double2 sh[4];
    const CGRed s = cg1_redundant(sc, part, nparts, J + 1, sh);  // S_J from S_{J-1} and pass J's partials
    if (threadIdx.x == 0) store_state(sc, s);
}

void launch_cg1_flush(hipStream_t s, int nparts, const double2 *partials, CGScalars *sc, long pass) {
    hipLaunchKernelGGL(cg1_flush_kernel, dim3(1), dim3(256), 0, s, nparts, partials, sc, pass);
}

__global__ void __launch_bounds__(SB) cg1_scalar_kernel(int nparts, const double2 *part, CGScalars *sc, int first) {
    // the partial loads do not wait for the `done` flag's load: a finished
    // solve only skips the scalar update
    double2 t[3];
    sum3_partials(nparts, part, t);
    if (threadIdx.x == 0 && !sc->done) cg1_scalars(sc, first, t[0], t[1], t[2]);
}

// Multi-shard: local sums into sc->sum3 (all-reduced by the host), then the scalars.
__global__ void __launch_bounds__(SB) cg1_local_sum_kernel(int nparts, const double2 *part, CGScalars *sc) {
    double2 t[3];
    sum3_partials(nparts, part, t);
    if (threadIdx.x == 0 && !sc->done) {
        sc->sum3[0] = t[0];
        sc->sum3[1] = t[1];
        sc->sum3[2] = t[2];
    }
}

__global__ void cg1_from_sums_kernel(CGScalars *sc, int first) {
    if (sc->done) return;
    cg1_scalars(sc, first, sc->sum3[0], sc->sum3[1], sc->sum3[2]);
}

void launch_cg_onepass(hipStream_t s, const Geometry &g, const CGFusedCfg &c, int nshard,
                       const double2 *dold, const double2 *rold, const double2 *aold, double2 *dnew,
                       double2 *anew, double2 *x, const double2 *U, const double2 *fd, const double2 *fr,
                       const double2 *fa, const double2 *fU, double mass, int first, CGScalars *sc,
                       double2 *partials, int tb0, int tbn, const double2 *prev_partials, long pass) {
    if (tbn <= 0) return;
    CG1Args a;
    a.dold = dold; a.rold = rold; a.aold = aold;
    a.dnew = dnew; a.anew = anew;
    a.x = x; a.U = U;
    a.fd = fd; a.fr = fr; a.fa = fa; a.fU = fU;
    a.sc = sc; a.partials = partials;
    a.V = g.V; a.Nx = g.Nx; a.Wt = g.Wt; a.t0 = g.t0; a.Ntg = g.Ntg; a.nshard = nshard;
    a.xchunk = c.xchunk; a.NWT = c.NWT; a.TBk = c.TBk; a.XB = c.XB; a.remap = c.remap;
    a.first = first;
    a.mass = mass;
    a.tb0 = tb0;
    a.tbn = tbn;
    a.prev = prev_partials;
    a.pass = pass;
    const dim3 grid(tbn * c.XB), block(256);
    const bool xp = pass >= 2 && (pass & 1) == 0;  // x takes passes j-1 and j together
    if (prev_partials) {
        if (xp) hipLaunchKernelGGL((cg_onepass_kernel<1, 1>), grid, block, 0, s, a);
        else hipLaunchKernelGGL((cg_onepass_kernel<1, 0>), grid, block, 0, s, a);
    } else {
        if (xp) hipLaunchKernelGGL((cg_onepass_kernel<0, 1>), grid, block, 0, s, a);
        else hipLaunchKernelGGL((cg_onepass_kernel<0, 0>), grid, block, 0, s, a);
    }
}

void launch_cg1_scalars(hipStream_t s, int nparts, const double2 *partials, CGScalars *sc, int first) {
    hipLaunchKernelGGL(cg1_scalar_kernel, dim3(1), dim3(SB), 0, s, nparts, partials, sc, first);
}

void launch_cg1_local_sum(hipStream_t s, int nparts, const double2 *partials, CGScalars *sc) {
    hipLaunchKernelGGL(cg1_local_sum_kernel, dim3(1), dim3(SB), 0, s, nparts, partials, sc);
}

void launch_cg1_from_sums(hipStream_t s, CGScalars *sc, int first) {
    hipLaunchKernelGGL(cg1_from_sums_kernel, dim3(1), dim3(1), 0, s, sc, first);
}

CGFusedCfg cg_fused_config(const Geometry &g) {
    CGFusedCfg c;
    c.NWT = (g.Wt + FW - 1) / FW;
    c.TBk = (c.NWT + 3) / 4;
    const int target = 4096;  // 4096^2: xchunk 18 (tools/tune_cg.py: 16-32 best, 128 -12 %)
    int nchunks = (target + c.TBk - 1) / c.TBk;
    if (nchunks > g.Nx) nchunks = g.Nx;
    if (nchunks < 1) nchunks = 1;
    c.xchunk = (g.Nx + nchunks - 1) / nchunks;
    // mid-size lattices: at least min(12, Nx/64) rows per chunk, so the 4
    // halo rows a chunk re-reads stay a small fraction (tools/tune_cg.py,
    // one-pass ms per iteration: 512^2 8 rows 0.030 vs 1 row 0.039; 1024^2
    // 12 rows 0.076 vs 2 rows 0.087; 2048^2 8-12 rows 0.27 vs 0.28). Small
    // lattices keep one row per block (latency-bound: parallelism first).
    if (g.Nx >= 512) {
        const int xmin = g.Nx / 64 < 12 ? g.Nx / 64 : 12;
        if (c.xchunk < xmin) c.xchunk = xmin;
    }
    c.XB = (g.Nx + c.xchunk - 1) / c.xchunk;
    c.remap = 1;
    return c;
}

int cg_fused_blocks(const CGFusedCfg &c) { return c.TBk * c.XB; }

constexpr int RB2 = 256;

// Two-direction form: after the last pass J = k (pass J evaluated into sc), an
// odd J left alpha_{J-1} d_{J-1} out of x. A stopping evaluation keeps alpha =
// alpha_{J-1}; a non-final one has already moved it to alpha2.
__global__ void __launch_bounds__(RB2) cg_td_finish_x_kernel(long n, double2 *x, const double2 *d0,
                                                             const double2 *d1, const double2 *d2,
                                                             const CGScalars *sc) {
    const int k = sc->k;
    if (k < 1 || !(k & 1)) return;
    const double2 alpha = sc->done ? sc->alpha : sc->alpha2;
    const int i3 = (k - 1) % 3;
    const double2 *d = i3 == 0 ? d0 : (i3 == 1 ? d1 : d2);
    const Chunk ch = block_chunk(n);
    for (long i = ch.beg + threadIdx.x; i < ch.end; i += RB2) x[i] = cadd(x[i], cmul(alpha, d[i]));
}

void launch_cg_td_finish_x(hipStream_t s, long n, double2 *x, const double2 *d0, const double2 *d1,
                           const double2 *d2, const CGScalars *sc) {
    hipLaunchKernelGGL(cg_td_finish_x_kernel, dim3(reduce_blocks(n)), dim3(RB2), 0, s, n, x, d0, d1, d2, sc);
}

// ---- 2-deep t-faces: columns {Wt-2, Wt-1} go up (arrive as -2, -1), {0, 1} go
// down (arrive as Wt, Wt+1). Buffers [col][plane][x], 4*Nx complex each.
__global__ void pack_faces2_kernel(int Nx, int Wt, long V, const double2 *f, double2 *lo, double2 *hi) {
    const int x = blockIdx.x * blockDim.x + threadIdx.x;
    if (x >= Nx) return;
    const long row = (long)x * Wt;
    for (int col = 0; col < 2; ++col)
        for (int p = 0; p < 2; ++p) {
            const int c_lo = col < Wt ? col : Wt - 1;           // t = 0, 1
            const int c_hi = Wt - 2 + col >= 0 ? Wt - 2 + col : 0;  // t = Wt-2, Wt-1
            lo[(long)(col * 2 + p) * Nx + x] = f[row + c_lo + p * V];
            hi[(long)(col * 2 + p) * Nx + x] = f[row + c_hi + p * V];
        }
}

void launch_pack_faces2(hipStream_t s, const Geometry &g, const double2 *field, double2 *lo,
                        double2 *hi) {
    hipLaunchKernelGGL(pack_faces2_kernel, dim3((g.Nx + 63) / 64), dim3(64), 0, s, g.Nx, g.Wt, g.V,
                       field, lo, hi);
}

}  // namespace sm
