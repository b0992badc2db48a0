// sm_eotd.hip -- one-pass even-odd CG iteration on Dhat Dhat^dag (gfx950),
// the two-direction recurrence of sm_cgfused.hip on half-lattice vectors.
//
// Pass j (even sites; r is never stored, Ad is):
//     r_{j-1} = d_{j-1} - d_{j-2} beta_{j-2};  r_j = r_{j-1} - alpha_{j-1} Ad_{j-1}
//     d_j = d_{j-1} beta_{j-1} + r_j;  on even j x <- (x + alpha_{j-2} d_{j-2}) + alpha_{j-1} d_{j-1}
//     W = Dhat^dag d_j,  Ad_j = Dhat W  (four checkerboard hops, in registers)
//     partials |W|^2 (= <d_j, Ad_j>), <r_j, Ad_j>, |r_j|^2, |Ad_j|^2
// then cg1_scalars as for the full operator (sm_cgfused.hip). A pass reads
// d_{j-1}, d_{j-2}, Ad_{j-1} and both link parities (160 B per even site) and
// writes d_j, Ad_j (64) plus x on even passes: ~256 B per even site against
// ~575 for the six-launch iteration (sm_eo.cpp eo_cg).
//
// Layout (sm_eo.hip): a parity-p field holds Vh = Nx*Wh sites, h = x*Wh + k,
// t = 2k + ((p + x) & 1). Hops between parities use entries k-1+s, k+s of the
// same row (s row-dependent) and entry k of rows x +- 1. A wave owns 56
// k-columns (4 halo lanes per side: one per hop), rows march along x:
//     F   row y+4: r_j, d_j                       (d_{j-1}, d_{j-2}, Ad_{j-1} loaded)
//     H1  row y+3: T1 = D_oe^dag-hop of d_j        (odd)
//     H2  row y+2: W  = Dhat^dag d_j               (even; |W|^2)
//     H3  row y+1: T2 = D_oe-hop of W              (odd)
//     H4  row y  : Ad_j = Dhat W                   (even; dots with r_j(y))
// The hops use the folded bracket (dirac_bracket_folded): the same values as
// the reference arithmetic up to the sign of an exact zero. t-shards (SH = 1):
// halo lanes outside the shard read 4-deep checkerboard faces
// ([side][plane][col][x]: side 0 = my k = col-4, side 1 = my k = Wh+col).
// Registers: 256 VGPRs + ~105 AGPRs, so one wave per SIMD; measured 0.54 ms
// per iteration at 4096^2 against 0.94 ms for the six launches.
#include <type_traits>

#include "sm_device.h"
#include "sm_internal.h"

#pragma clang fp contract(off)

namespace sm {

constexpr int EW4 = kEoTdWaveCols;
constexpr int EH4 = 4;  // halo lanes per side

struct EoTDArgs {
    const double2 *d1, *d2, *aold;  // d_{j-1}, d_{j-2}, Ad_{j-1}
    double2 *dn, *anew, *x;
    const double2 *Ue, *Uo;         // checkerboard links: plane 0 U_t, plane 1 U_x
    const double2 *f1, *f2, *fa, *fue, *fuo;  // SH: 4-deep faces of d1, d2, aold, Ue, Uo
    CGScalars *sc;
    double2 *partials;              // 3 per block: (|W|^2, 0), <r,Ad>, (|r|^2, |Ad|^2)
    unsigned *tick;                 // != null: ticketed tail (sm_device.h cg_ticketed_tail)
    double2 *gsum, *out3;           // its group sums; out3 != null: the shard's sums instead of the scalars
    int red;                        // t-shards: every block evaluates pass j-1's scalars from sc->sumr
    long pass;
    long Vh;
    int Nx, Wh, t0, Ntg;
    int xchunk, NWT, TBk, XB, first, rebuild;
    double mass;
};

// One checkerboard hop's bracket (dirac_bracket_folded's terms) at a lane whose
// forward t-neighbour is lane+1 and backward one this lane (FWD = true), or
// forward this lane and backward lane-1 (FWD = false). The shifted hop crosses
// lanes as ONE complex: the forward spin combination, or the whole backward
// product conj(U_t) * combination formed by the sending lane with its own link
// (Ub) and signed after the shift. Negation commutes exactly with the rounded
// products and sums, so every value equals dirac_bracket_folded's up to the
// sign of an exact zero. v: centre (t-neighbour source), vxp / vxm: x+-1.
template <int DG, bool FWD>
__device__ __forceinline__ void eo_bracket(double sr0, double sl0, const Sp &v, const Sp &vxp, const Sp &vxm,
                                           double2 Ut, double2 Ux, double2 Ub, double2 Uxm, double2 &h0,
                                           double2 &h1) {
    const double2 qf = DG ? cadd(v.a, v.b) : csub(v.a, v.b);  // forward-hop combination
    const double2 qb = DG ? csub(v.a, v.b) : cadd(v.a, v.b);  // backward-hop combination
    const double2 a = make_double2(Ut.x * sr0, Ut.y * sr0);
    double2 A, C;
    if (FWD) {
        A = cmul(a, dpp_shl1(qf));
        C = cmul(make_double2(Ub.x * sl0, -(Ub.y * sl0)), qb);
    } else {
        A = cmul(a, qf);
        const double2 Cs = dpp_shr1(cmul(make_double2(Ub.x, -Ub.y), qb));
        C = make_double2(Cs.x * sl0, Cs.y * sl0);
    }
    const double2 e = make_double2(Uxm.x, -Uxm.y);
    if (!DG) {
        const double2 B = cmul(Ux, make_double2(vxp.a.x - vxp.b.y, vxp.a.y + vxp.b.x));  // px0 + i px1
        const double2 E = cmul(e, make_double2(vxm.a.x + vxm.b.y, vxm.a.y - vxm.b.x));   // pxm0 - i pxm1
        h0 = cadd(cadd(cadd(A, B), C), E);
        h1 = cadd(cadd(cadd(cneg(A), mul_mi(B)), C), mul_i(E));
    } else {
        const double2 E = cmul(e, make_double2(vxm.a.x - vxm.b.y, vxm.a.y + vxm.b.x));   // pxm0 + i pxm1
        const double2 B = cmul(Ux, make_double2(vxp.a.x + vxp.b.y, vxp.a.y - vxp.b.x));  // px0 - i px1
        h0 = cadd(cadd(cadd(C, E), A), B);
        h1 = cadd(cadd(cadd(cneg(C), mul_mi(E)), A), mul_i(B));
    }
}

template <int XP, int SH, int RED = 0>
__global__ void __launch_bounds__(256) eo_td_kernel(EoTDArgs a) {
    __shared__ double2 sh[4];
    __shared__ double2 rlds[5][2][256];  // r_j of rows y .. y+4
    CGScalars *sc = a.sc;
    const double2 z2 = make_double2(0.0, 0.0);
    const bool first = a.first != 0, rebuild = a.rebuild != 0;
    double2 alpha, beta, alpha2, beta2;
    if (RED) {  // t-shards: pass j-1's scalars from its all-reduced sums (same step in every block)
        __shared__ double2 s_ab[4];
        __shared__ int s_stop;
        if (threadIdx.x == 0) {
            if (first) {
                s_ab[0] = s_ab[1] = s_ab[2] = s_ab[3] = z2;
                s_stop = 0;
            } else {
                ra_scalars_from_sums(sc, a.pass, s_ab, &s_stop);
            }
        }
        __syncthreads();
        if (s_stop) return;  // block-uniform
        alpha = first ? z2 : uniform_d2(s_ab[0]);
        beta = first ? z2 : uniform_d2(s_ab[1]);
        alpha2 = uniform_d2(s_ab[2]);
        beta2 = rebuild ? uniform_d2(s_ab[3]) : z2;
    } else {
        if (sc->done) return;  // grid-uniform
        alpha = first ? z2 : sc->alpha;
        beta = first ? z2 : sc->beta;
        alpha2 = sc->alpha2;
        beta2 = rebuild ? sc->beta2 : z2;
    }
    const int tb = blockIdx.x % a.TBk, xc = blockIdx.x / a.TBk;
    const int lane = threadIdx.x & 63;
    const int gw = tb * 4 + (threadIdx.x >> 6);
    const int x0 = xc * a.xchunk, xe = min(a.Nx, x0 + a.xchunk);
    double aW = 0.0, aR = 0.0, aA = 0.0;  // |W|^2, |r|^2, |Ad|^2
    double2 aRA = z2;                      // <r, Ad>
    if (gw < a.NWT && x0 < xe) {
        const int Wh = a.Wh, Nx = a.Nx;
        const long Vh = a.Vh;
        const int k = gw * EW4 - EH4 + lane;
        int kw = k % Wh;
        if (kw < 0) kw += Wh;
        const bool own = lane >= EH4 && lane < EW4 + EH4 && k < Wh;
        const bool inside = k >= 0 && k < Wh;
        const int side = k < 0 ? 0 : 1;
        const int fcol = min(max(k < 0 ? k + EH4 : k - Wh, 0), EH4 - 1);
        const double m = a.mass, hm = 0.5 / a.mass;
        auto wrapx = [Nx](int x) { int w = x % Nx; return w < 0 ? w + Nx : w; };
        auto hidx = [&](int y) { return (long)wrapx(y) * Wh + kw; };
        // face entry (plane 0) of row y for this lane; plane 1 is 4*Nx further
        auto fidx = [&](int y) { return (long)((side * 2) * EH4 + fcol) * Nx + wrapx(y); };
        auto signs = [&](int t, double &sr0, double &sl0) {
            int tg = (a.t0 + t) % a.Ntg;
            if (tg < 0) tg += a.Ntg;
            sr0 = tg == a.Ntg - 1 ? -1.0 : 1.0;
            sl0 = tg == 0 ? -1.0 : 1.0;
        };
        struct Lk {
            double2 et, ex, ot, ox;  // even / odd links at (y, k)
        };
        auto ldl = [&](int y, Lk &L) {
            const int yc = min(max(y, x0 - 4), xe + 2);
            if (!SH || inside) {
                const long h = hidx(yc);
                L.et = a.Ue[h];
                L.ex = a.Ue[h + Vh];
                L.ot = a.Uo[h];
                L.ox = a.Uo[h + Vh];
            } else {
                const long f = fidx(yc), p1 = (long)EH4 * Nx;
                L.et = a.fue[f];
                L.ex = a.fue[f + p1];
                L.ot = a.fuo[f];
                L.ox = a.fuo[f + p1];
            }
        };
        struct Fr {
            Sp d1, d2, ad, xv;
        };
        auto ldf = [&](int y, Fr &F) {
            const int yc = min(max(y, x0 - 4), xe + 3);
            if (!SH || inside) {
                const long h = hidx(yc);
                F.d1 = Sp{a.d1[h], a.d1[h + Vh]};
                F.d2 = Sp{a.d2[h], a.d2[h + Vh]};
                F.ad = Sp{a.aold[h], a.aold[h + Vh]};
            } else {
                const long f = fidx(yc), p1 = (long)EH4 * Nx;
                F.d1 = Sp{a.f1[f], a.f1[f + p1]};
                F.d2 = Sp{a.f2[f], a.f2[f + p1]};
                F.ad = Sp{a.fa[f], a.fa[f + p1]};
            }
            if (XP) {
                const long hx = hidx(min(max(y, x0), xe - 1));
                F.xv = Sp{a.x[hx], a.x[hx + Vh]};
            }
        };
        // odd hop at odd site (y, k) from an even field: T = -0.5 H_oe v. YE: row
        // y even (the backward t-neighbour is this lane, the forward one lane+1).
        auto todd = [&](auto dag, auto ye, const Sp &vc, const Sp &vxm, const Sp &vxp, const Lk &L, double2 ex_m) {
            constexpr int DG = decltype(dag)::value;
            constexpr bool YE = decltype(ye)::value;
            double sr0, sl0;
            signs(2 * k + (YE ? 1 : 0), sr0, sl0);
            double2 h0, h1;
            eo_bracket<DG, YE>(sr0, sl0, vc, vxp, vxm, L.ot, L.ox, L.et, ex_m, h0, h1);
            return Sp{rmul(-0.5, h0), rmul(-0.5, h1)};
        };
        // even hop at even site (x, k) from an odd field: m v + (0.5/m) H_eo T.
        // XEV: row x even (the backward t-neighbour is lane-1, the forward one this lane).
        auto eout = [&](auto dag, auto xev, const Sp &Tc, const Sp &Txm, const Sp &Txp, const Lk &L, double2 ox_m,
                        const Sp &vc) {
            constexpr int DG = decltype(dag)::value;
            constexpr bool XEV = decltype(xev)::value;
            double sr0, sl0;
            signs(2 * k + (XEV ? 0 : 1), sr0, sl0);
            double2 h0, h1;
            eo_bracket<DG, !XEV>(sr0, sl0, Tc, Txp, Txm, L.et, L.ex, L.ot, ox_m, h0, h1);
            return Sp{cadd(rmul(m, vc.a), rmul(hm, h0)), cadd(rmul(m, vc.b), rmul(hm, h1))};
        };
        using DAG1 = std::integral_constant<int, 1>;
        using DAG0 = std::integral_constant<int, 0>;
        const double2 z = z2;
        const Sp zs = Sp{z, z};
        const Lk zl = Lk{z, z, z, z};
        // state at the top of iteration y (links Lk at rows y-1 .. y+2 held, y+3 in flight)
        Fr Fin;                            // in flight: row y+4
        Lk Lin;                            // in flight: row y+3
        Lk Lm = zl, L0 = zl, L1 = zl, L2 = zl;  // rows y-1, y, y+1, y+2
        Sp J2 = zs, J3 = zs;               // d_j rows y+2, y+3
        Sp A1 = zs, A2 = zs;               // T1 rows y+1, y+2
        Sp W0 = zs, W1 = zs;               // W rows y, y+1
        Sp B0 = zs, Bm = zs;               // T2 rows y, y-1
        Fin.xv = zs;
        const int y0 = x0 - 8;
        ldf(y0 + 4, Fin);
        ldl(y0 + 3, Lin);
        int s_w = 4, s_r = 0;              // r_j ring slots of rows y+4 (written) and y (read)
        // stage mask M: bit 0 H1, bit 1 H2, bit 2 H3, bit 3 H4 (F always)
        // P: parity of row y (x0 is even: Nx and xchunk are)
        auto step = [&](int y, auto mtag, auto ptag) {
            constexpr int M = decltype(mtag)::value;
            constexpr bool E0 = decltype(ptag)::value == 0;  // rows y, y+2, y+4 even
            using PE = std::integral_constant<bool, E0>;
            using PO = std::integral_constant<bool, !E0>;
            const Fr F = Fin;
            const Lk L3 = Lin;
            ldf(y + 5, Fin);
            ldl(y + 4, Lin);
            __builtin_amdgcn_sched_barrier(0);
            // F: r_j, d_j at row y+4
            const int xr = y + 4;
            Sp rp, R4, J4;
            rp.a = csub(F.d1.a, cmul(F.d2.a, beta2));
            rp.b = csub(F.d1.b, cmul(F.d2.b, beta2));
            R4.a = csub(rp.a, cmul(alpha, F.ad.a));
            R4.b = csub(rp.b, cmul(alpha, F.ad.b));
            J4.a = cadd(cmul(F.d1.a, beta), R4.a);
            J4.b = cadd(cmul(F.d1.b, beta), R4.b);
            if (xr >= x0 && xr < xe && own) {
                const long h = (long)xr * Wh + kw;
                st_nt(a.dn + h, J4.a);
                st_nt(a.dn + h + Vh, J4.b);
                if (XP) {
                    st_nt(a.x + h, cadd(cadd(F.xv.a, cmul(alpha2, F.d2.a)), cmul(alpha, F.d1.a)));
                    st_nt(a.x + h + Vh, cadd(cadd(F.xv.b, cmul(alpha2, F.d2.b)), cmul(alpha, F.d1.b)));
                }
                aR += cmul(R4.a, cconj(R4.a)).x;
                aR += cmul(R4.b, cconj(R4.b)).x;
            }
            rlds[s_w][0][threadIdx.x] = R4.a;
            rlds[s_w][1][threadIdx.x] = R4.b;
            Sp A3 = zs, W2 = zs, B1 = zs;
            if constexpr ((M & 1) != 0) A3 = todd(DAG1(), PO(), J3, J2, J4, L3, L2.ex);  // H1: T1(y+3)
            if constexpr ((M & 2) != 0) {                                                  // H2: W(y+2)
                W2 = eout(DAG1(), PE(), A2, A1, A3, L2, L1.ox, J2);
                if (y + 2 >= x0 && y + 2 < xe && own) {
                    aW += cmul(W2.a, cconj(W2.a)).x;  // |W|^2 = <d_j, Dhat Dhat^dag d_j>
                    aW += cmul(W2.b, cconj(W2.b)).x;
                }
            }
            if constexpr ((M & 4) != 0) B1 = todd(DAG0(), PO(), W1, W0, W2, L1, L0.ex);   // H3: T2(y+1)
            if constexpr ((M & 8) != 0) {                                                  // H4: Ad_j(y)
                const Sp o = eout(DAG0(), PE(), B0, Bm, B1, L0, Lm.ox, W0);
                if (own) {
                    const long h = (long)y * Wh + kw;
                    st_nt(a.anew + h, o.a);
                    st_nt(a.anew + h + Vh, o.b);
                    const Sp R0 = Sp{rlds[s_r][0][threadIdx.x], rlds[s_r][1][threadIdx.x]};
                    aRA = cadd(aRA, cmul(R0.a, cconj(o.a)));  // dot(r, Ad)
                    aRA = cadd(aRA, cmul(R0.b, cconj(o.b)));
                    aA += cmul(o.a, cconj(o.a)).x;
                    aA += cmul(o.b, cconj(o.b)).x;
                }
            }
            Lm = L0;
            L0 = L1;
            L1 = L2;
            L2 = L3;
            J2 = J3;
            J3 = J4;
            A1 = A2;
            A2 = A3;
            W0 = W1;
            W1 = W2;
            Bm = B0;
            B0 = B1;
            s_w = s_w == 4 ? 0 : s_w + 1;
            s_r = s_r == 4 ? 0 : s_r + 1;
        };
        using Ev = std::integral_constant<int, 0>;
        using Od = std::integral_constant<int, 1>;
        int y = y0;  // even; every chunk has an even number of rows
        step(y, std::integral_constant<int, 0>(), Ev());
        step(y + 1, std::integral_constant<int, 0>(), Od());
        step(y + 2, std::integral_constant<int, 1>(), Ev());
        step(y + 3, std::integral_constant<int, 1>(), Od());
        step(y + 4, std::integral_constant<int, 3>(), Ev());
        step(y + 5, std::integral_constant<int, 3>(), Od());
        step(y + 6, std::integral_constant<int, 7>(), Ev());
        step(y + 7, std::integral_constant<int, 7>(), Od());
        for (y += 8; y < xe; y += 2) {
            step(y, std::integral_constant<int, 15>(), Ev());
            step(y + 1, std::integral_constant<int, 15>(), Od());
        }
    }
    const double2 s0 = block_sum(make_double2(aW, 0.0), sh);
    __syncthreads();
    const double2 s1 = block_sum(aRA, sh);
    __syncthreads();
    const double2 s2 = block_sum(make_double2(aR, aA), sh);
    if (a.tick) {  // block-uniform
        cg_ticketed_tail(a.partials, blockIdx.x, (int)gridDim.x, a.tick, a.gsum, a.out3, sc, a.first, s0, s1, s2);
        return;
    }
    if (threadIdx.x == 0) {
        double2 *p = a.partials + 3 * (long)blockIdx.x;
        p[0] = s0;
        p[1] = s1;
        p[2] = s2;
    }
}

EoTdCfg eo_td_config(const Geometry &g) {
    EoTdCfg c;
    const int Wh = g.Wt / 2;
    c.NWT = (Wh + EW4 - 1) / EW4;
    c.TBk = (c.NWT + 3) / 4;
    // rows per block: 16 from 1024 rows up (tools/tune_eo.py, ms per iteration
    // incl. host transfers: 4096^2 16 rows 0.90 vs 24 1.01 vs 32 1.03; 1024^2
    // 16 rows 0.058 vs 8 0.066 vs 12 0.065). The kernel runs one block per CU
    // (360 registers per lane), so 1024^2 at 16 rows is 192 blocks, one round.
    if (g.Nx >= 1024) {
        c.xchunk = 16;
    } else {
        int nchunks = (2048 + c.TBk - 1) / c.TBk;
        if (nchunks > g.Nx) nchunks = g.Nx;
        if (nchunks < 1) nchunks = 1;
        c.xchunk = (g.Nx + nchunks - 1) / nchunks;
        if (c.xchunk < 2) c.xchunk = 2;
    }
    if (c.xchunk < 2) c.xchunk = 2;
    c.xchunk += c.xchunk & 1;  // even: the kernel's row parities are static
    c.XB = (g.Nx + c.xchunk - 1) / c.xchunk;
    return c;
}

int eo_td_blocks(const EoTdCfg &c) { return c.TBk * c.XB; }

void launch_eo_td(hipStream_t s, const Geometry &g, const EoTdCfg &c, const double2 *d1, const double2 *d2,
                  const double2 *aold, double2 *dn, double2 *anew, double2 *x, const double2 *Ue, const double2 *Uo,
                  double mass, long pass, CGScalars *sc, double2 *partials, const EoTdFaces &f, unsigned *tick,
                  double2 *gsum, double2 *out3, int red) {
    EoTDArgs a;
    a.red = red;
    a.pass = pass;
    a.d1 = d1; a.d2 = d2; a.aold = aold; a.dn = dn; a.anew = anew; a.x = x;
    a.Ue = Ue; a.Uo = Uo; a.sc = sc; a.partials = partials;
    a.tick = tick; a.gsum = gsum; a.out3 = out3;
    a.f1 = f.d1; a.f2 = f.d2; a.fa = f.ad; a.fue = f.ue; a.fuo = f.uo;
    a.Vh = g.V / 2; a.Nx = g.Nx; a.Wh = g.Wt / 2; a.t0 = g.t0; a.Ntg = g.Ntg;
    a.xchunk = c.xchunk; a.NWT = c.NWT; a.TBk = c.TBk; a.XB = c.XB;
    a.first = pass == 0;
    a.rebuild = pass >= 2;
    a.mass = mass;
    const dim3 grid(c.TBk * c.XB), block(256);
    const bool xp = pass >= 2 && (pass & 1) == 0;
    if (f.d1 && red) {
        if (xp) hipLaunchKernelGGL((eo_td_kernel<1, 1, 1>), grid, block, 0, s, a);
        else hipLaunchKernelGGL((eo_td_kernel<0, 1, 1>), grid, block, 0, s, a);
    } else if (f.d1) {
        if (xp) hipLaunchKernelGGL((eo_td_kernel<1, 1>), grid, block, 0, s, a);
        else hipLaunchKernelGGL((eo_td_kernel<0, 1>), grid, block, 0, s, a);
    } else {
        if (xp) hipLaunchKernelGGL((eo_td_kernel<1, 0>), grid, block, 0, s, a);
        else hipLaunchKernelGGL((eo_td_kernel<0, 0>), grid, block, 0, s, a);
    }
}

// 4-deep checkerboard t-faces [side][plane][col][x]: side 0 = columns k = 0..3
// (sent down), side 1 = k = Wh-4..Wh-1 (sent up); 16*Nx complex.
__global__ void __launch_bounds__(256) pack_cb_faces4_kernel(int Nx, int Wh, long Vh, const double2 *f, double2 *out) {
    const int n = 16 * Nx;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const int x = i % Nx, r = i / Nx;
        const int col = r & 3, plane = (r >> 2) & 1, side = r >> 3;
        const int k = side ? Wh - 4 + col : col;
        out[i] = f[plane * Vh + (long)x * Wh + k];
    }
}

void launch_pack_cb_faces4(hipStream_t s, const Geometry &g, const double2 *f, double2 *out) {
    hipLaunchKernelGGL(pack_cb_faces4_kernel, dim3((16 * g.Nx + 255) / 256), dim3(256), 0, s, g.Nx, g.Wt / 2,
                       g.V / 2, f, out);
}

}  // namespace sm
