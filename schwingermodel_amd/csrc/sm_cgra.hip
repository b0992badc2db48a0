// sm_cgra.hip -- two-direction CG pass that recomputes Ad_{j-1} instead of
// storing it (gfx950). Mode 5 of sm_tune_cg.
//
// Pass j of the two-direction CG (sm_cgfused.hip, cg_onepass_kernel<.,1,.>):
//     r_{j-1} = d_{j-1} - d_{j-2} beta_{j-2}      (the reference's d *= beta; d += r,
//                                                  src/conjugate_gradient.cpp:55-58)
//     r_j     = r_{j-1} - alpha_{j-1} Ad_{j-1}    (:38-39)
//     d_j     = d_{j-1} beta_{j-1} + r_j          (:55-58)
//     x      <- (x + alpha_{j-2} d_{j-2}) + alpha_{j-1} d_{j-1}   on the x rows of parity j & 1 (:36-37)
//     Ad_j    = D D^dag d_j ; partials <d_j,Ad_j>, <r_j,Ad_j>, |r_j|^2, |Ad_j|^2
// Mode 4 stores Ad_j and reads it back in pass j+1. Here Ad_{j-1} = D D^dag
// d_{j-1} is recomputed from the d_{j-1} rows the pass reads anyway, with the
// same stencil code on the same operands, so it is bitwise the value pass j-1
// used for its dots. A pass reads d_{j-1}, d_{j-2}, U (96 B/site) and writes
// d_j (32), plus x on half the rows (32 on average): 160 B/site against 224
// for mode 4 and 576 for the reference's sequence; 148 with
// the links read as exact codes (UC: one double and a 16-bit flag word per
// link, sm_linkcode.h). Each x row takes its two updates together
// every other pass, the even rows on even passes and the odd rows on odd
// ones, so every pass moves the same bytes (with all of x on even passes the
// odd pass was VALU-bound and the even one HBM-bound). The price of the
// recomputation is a second D^dag + D per site: fp64 VALU work that runs
// under the HBM time.
//
// Geometry: a wave owns RW = 56 consecutive t-columns; its 64 lanes cover
// columns T0-4 .. T0+59. The four stencil stages (D^dag, D on d_{j-1}; D^dag,
// D on d_j) each take their t-neighbours from adjacent lanes through DPP wave
// shifts, so each stage loses one lane per side: 4 halo lanes. Rows march
// along x with every intermediate held in registers:
//     S1  T'(y+3) = D^dag d_{j-1}     rows y+2 .. y+4 of d_{j-1}
//     S2  A (y+2) = D T' = Ad_{j-1}   rows y+1 .. y+3 of T'
//     S3  r_j, d_j at row y+2         (store d_j; x update)
//     S4  T (y+1) = D^dag d_j         rows y .. y+2 of d_j
//     S5  Ad_j(y) = D T               rows y-1 .. y+1 of T; dots
// A block of chunk [x0, xe) runs y = x0-6 .. xe-1; the first iterations run
// only the stages whose rows are needed (S1 from x0-6, S2/S3 from x0-4, S4
// from x0-2, S5 from x0). r_j waits two rows for its dot with Ad_j in a
// 3-slot LDS ring (each thread its own slots, no barrier).
//
// FOLD = 1 evaluates the hopping bracket with its products by 0, +-1 and +-i
// folded into sign flips and swaps (dirac_bracket_folded): the same values up
// to the sign of an exact zero, at 84 instead of ~126 fp64 operations a site.
// FOLD = 2 (the default) also forms the complex products, the CG updates and
// the dots with fused multiply-adds: one rounding where GCC's expansion has
// two or three, so the iterates differ from FOLD = 1 at rounding level (the
// parity bar for CG is the converged solution, 1e-12).
//
// TK = 1 (the default with FOLD = 2 on grids that do not take the redundant
// scalars) ends the pass with a ticketed tail instead of a separate scalar
// kernel: the last block of each group of 64 tiles sums the group's partials,
// the last group's block sums the group sums in order and forms the scalars
// (one shard) or writes the shard's three sums for the all-reduce (t-shards).
// The order is fixed, so results stay run-to-run reproducible.
#include <type_traits>

#include <hip/hip_ext.h>

#include "sm_device.h"
#include "sm_internal.h"
#include "sm_linkcode.h"

#pragma clang fp contract(off)

namespace sm {

constexpr int RW = kRAWaveCols;
constexpr int RH = 4;  // halo lanes per side

struct RAArgs {
    const double2 *d1, *d2;       // d_{j-1}, d_{j-2}
    double2 *dn;                  // d_j
    double2 *x;
    const double2 *U;
    const double2 *f1, *f2, *fU;  // t-shard 4-deep faces [col -4..-1, Wt..Wt+3][plane][x]
    CGScalars *sc;
    double2 *partials;            // 3 per tile: <d,Ad>, <r,Ad>, (|r|^2, |Ad|^2)
    long V;
    int Nx, Wt, t0, Ntg;
    int xchunk, NWT, TBk, XB, remap, first, rebuild, wpb;
    int tb0, tbn;
    double mass;
    const double2 *prev;  // RED: pass j-1's partials
    long pass;
    const double *Ua, *fUa;  // UC: link codes v of U_t, U_x (plane stride V, sm_linkcode.h) and their 4-deep faces
    const uint16_t *Uf, *fUf;  // UC 1: the codes' flag words (same layout; stored right after the codes)
    const uint8_t *Ub, *fUb;   // UC 2: one byte per site, the U_t (low) and U_x (high) flag nibbles
                               // (after the flag words; faces [col][x])
    int xpar;                // XP: this pass updates x on the rows of parity xpar (= pass & 1)
    int pbase;               // partial slots: tile pbase + (t-block - tb0) * XB + x-chunk
    double2 *fsend;          // SH: != null -> the edge blocks also write d_j's 4-deep send faces
    double2 *fsendh;         //   (lo part at fsend, hi part at fsendh)
    const PeerView *peer;    // peer transport: faces as 16-B write-through stores into the neighbours'
    unsigned long long pseq; //   rings, the tail all-reduces the sums (collective pseq)
    int pstore;              //   face store form: 0 16-B buffer stores sc0 sc1, 1 8-B atomic, 2 plain (A/B)
    // TK (ticketed tail): counters tick[0] (groups) and tick[1 + g] (64 tiles
    // each), ntiles tiles over every launch of the pass, group sums gsum; the
    // last block forms the scalars (out3 == null) or writes the 3 sums to out3
    unsigned *tick;
    int ntiles;
    double2 *gsum, *out3;
    // one-shard tail passes (REV kernels): flip = this pass reverses the
    // dispatch order of its tiles and the march direction; alt = x-adjacent
    // chunks march in opposite directions
    int flip, alt;
    int xbal;  // chunk xc covers rows [xc Nx / XB, (xc + 1) Nx / XB) (balanced) instead of xchunk-row chunks
};

// A link as the UC pass loads it: the code v and its flag word (UC 1), or the
// site's flag byte of two nibbles (UC 2), as loaded (converted only when the
// link is decoded, so the load stays a prefetch).
struct LinkCode {
    double v;
    uint32_t f;
};

// U(1) link from its code (UC; sm_linkcode.h: the smaller component as
// stored, the other one by a square root corrected by the flag word's ulp
// offset -- bitwise the stored link) in place of a 16-B load. UC 2: the
// nibble at bit `shift` of the flag byte.
template <int UC>
__device__ __forceinline__ double2 u_of(LinkCode code, int shift) {
    double c, s;
    const uint16_t f = UC == 2 ? sm_lc_flags_of_nibble(code.f >> shift) : (uint16_t)code.f;
    sm_link_decode(code.v, f, &c, &s);
    return make_double2(c, s);
}

template <typename T>
struct RSrc {
    const T *p;
    long xs, ps;
};

// Column c of a field: periodic wrap (one shard), in-domain, or the received
// 4-deep face (t-shard). Clamped so every lane's address is valid; lanes
// beyond the face depth only feed halo lanes.
template <int SH, typename T>
__device__ __forceinline__ RSrc<T> rsrc(const T *base, const T *face, int c, const RAArgs &a) {
    RSrc<T> s;
    if (!SH) {
        int cw = c % a.Wt;
        if (cw < 0) cw += a.Wt;
        s.p = base + cw;
        s.xs = a.Wt;
        s.ps = a.V;
    } else if (c >= 0 && c < a.Wt) {
        s.p = base + c;
        s.xs = a.Wt;
        s.ps = a.V;
    } else {
        int fc = c < 0 ? c + RH : c - a.Wt + RH;
        fc = fc < 0 ? 0 : (fc > 2 * RH - 1 ? 2 * RH - 1 : fc);
        s.p = face + (long)fc * 2 * a.Nx;
        s.xs = 1;
        s.ps = a.Nx;
    }
    return s;
}

// D (DAG = 0) / D^dag (DAG = 1) at this lane's column: centre p, x-neighbours
// pxm / pxp, t-neighbours from the adjacent lanes.
//
// FOLD: dirac_bracket_folded's terms with the t-hops moved to the sending
// lane, so each hop crosses lanes as ONE complex (4 DPP moves instead of 10):
// the forward hop needs only the spin combination at t+1 (D: pt0 - pt1,
// D^dag: pt0 + pt1), formed by its owner and shifted; the backward hop's whole
// product conj(U_t(t-1)) * combo(t-1) is formed by lane t-1 with its own link
// and shifted, and the antiperiodic sign applied after the shift. Negation
// commutes exactly with the rounded products and sums, so C = sl0 * that
// product equals the folded form's (U*sl0)^* combo up to the sign of an exact
// zero: the values are dirac_site_folded's.
//
// FOLD = 2 also takes its links pre-scaled (ra_march): U_t by -sr0/2 and U_x
// by -1/2, so A, B, C, E come out as -h/2's terms exactly (a power-of-two and
// sign scale commutes with every rounding) and the output is ONE fma,
// mass p + (-h/2), instead of a product and an fma. The backward hop's sign
// needs no product either: the receiving lane's SignL is -1 exactly when the
// sending lane t - 1 is at global t = Nt - 1, i.e. when the sender's SignR is,
// so the sender's scaled U_t already carries it. 8 fp64 operations less per
// stage.
// ST (t-strip blocks, round 6): the block's wpb waves form ONE strip of
// 64 wpb consecutive lanes (columns), owning 64 wpb - 2 RH of them, instead of
// wpb independent 64-lane windows of RW = 56 owned columns each. A stage's
// t-hops between the waves of a strip cross through LDS: lane 0 of each wave
// publishes its forward-hop combination qf, lane 63 its backward product bp,
// one barrier, and the neighbour waves' values enter the DPP shifts as the
// `old` operand (bound_ctrl off: the lane with no source lane in the wave
// keeps it), so no select is needed. Only the strip's own ends are halo
// lanes: 8 of 256 lanes instead of 8 of 64 (VALU work per owned site -8 % at
// 4096 columns: 17 strips x 4 waves against 74 waves a row), and the waves
// that share a row's lines run on one CU. xs: this stage's slots for this
// row's parity (the next row of the same parity is behind one more barrier,
// so one barrier per stage suffices).
__device__ __forceinline__ double dpp_shr1_keep(double v, double old) {  // lane l <- lane l-1; lane 0 keeps old
    const int lo = __builtin_amdgcn_update_dpp(__double2loint(old), __double2loint(v), 0x138, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp(__double2hiint(old), __double2hiint(v), 0x138, 0xf, 0xf, false);
    return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double dpp_shl1_keep(double v, double old) {  // lane l <- lane l+1; lane 63 keeps old
    const int lo = __builtin_amdgcn_update_dpp(__double2loint(old), __double2loint(v), 0x130, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp(__double2hiint(old), __double2hiint(v), 0x130, 0xf, 0xf, false);
    return __hiloint2double(hi, lo);
}

__device__ __forceinline__ void strip_hop(double2 *xs, double2 qf, double2 bp, double2 &qt, double2 &C) {
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, nw = blockDim.x >> 6;
    if (lane == 0) xs[2 * w] = qf;
    if (lane == 63) xs[2 * w + 1] = bp;
    __syncthreads();
    // the strip's first and last lanes are halo lanes: any finite value
    const double2 fl = xs[2 * (w > 0 ? w - 1 : 0) + 1];
    const double2 fr = xs[2 * (w + 1 < nw ? w + 1 : w)];
    C = make_double2(dpp_shr1_keep(bp.x, fl.x), dpp_shr1_keep(bp.y, fl.y));
    qt = make_double2(dpp_shl1_keep(qf.x, fr.x), dpp_shl1_keep(qf.y, fr.y));
}

template <int FOLD, int DAG, int ST = 0>
__device__ __forceinline__ Sp ra_site(double mass, double sr0, double sl0, const Sp &p, const Sp &pxm, const Sp &pxp,
                                      double2 ut, double2 ux, double2 uxm, double2 *xs = nullptr) {
    Sp o;
    static_assert(!ST || FOLD == 2, "t-strip blocks take the FOLD 2 arithmetic");
    if (FOLD == 2) {  // pre-scaled links: ut = -sr0 U_t / 2, ux = -U_x / 2, uxm = -U_x(x-1) / 2
        const double2 qf = DAG ? cadd(p.a, p.b) : csub(p.a, p.b);
        const double2 qb = DAG ? csub(p.a, p.b) : cadd(p.a, p.b);
        const double2 bp = cm<FOLD>(make_double2(ut.x, -ut.y), qb);
        double2 C, qt;  // C: lane t-1's -sl0 conj(U_t) qb / 2; qt: lane t+1's qf
        if constexpr (ST != 0) {
            strip_hop(xs, qf, bp, qt, C);
        } else {
            C = dpp_shr1(bp);
            qt = dpp_shl1(qf);
        }
        const double2 A = cm<FOLD>(ut, qt);
        const double2 e = make_double2(uxm.x, -uxm.y);
        double2 h0, h1;  // -h / 2
        if (!DAG) {
            const double2 B = cm<FOLD>(ux, make_double2(pxp.a.x - pxp.b.y, pxp.a.y + pxp.b.x));
            const double2 E = cm<FOLD>(e, make_double2(pxm.a.x + pxm.b.y, pxm.a.y - pxm.b.x));
            h0 = cadd(cadd(cadd(A, B), C), E);
            h1 = cadd(cadd(cadd(cneg(A), mul_mi(B)), C), mul_i(E));
        } else {
            const double2 E = cm<FOLD>(e, make_double2(pxm.a.x - pxm.b.y, pxm.a.y + pxm.b.x));
            const double2 B = cm<FOLD>(ux, make_double2(pxp.a.x + pxp.b.y, pxp.a.y - pxp.b.x));
            h0 = cadd(cadd(cadd(C, E), A), B);
            h1 = cadd(cadd(cadd(cneg(C), mul_mi(E)), A), mul_i(B));
        }
        o.a = make_double2(__builtin_fma(mass, p.a.x, h0.x), __builtin_fma(mass, p.a.y, h0.y));
        o.b = make_double2(__builtin_fma(mass, p.b.x, h1.x), __builtin_fma(mass, p.b.y, h1.y));
    } else if (FOLD) {
        const double2 qf = DAG ? cadd(p.a, p.b) : csub(p.a, p.b);  // forward-hop combination at this site
        const double2 qb = DAG ? csub(p.a, p.b) : cadd(p.a, p.b);  // backward-hop combination at this site
        const double2 Cb = cm<FOLD>(make_double2(ut.x, -ut.y), qb);  // conj(U_t) * qb, for lane t+1
        const double2 qt = dpp_shl1(qf);
        const double2 Cs = dpp_shr1(Cb);
        const double2 A = cm<FOLD>(make_double2(ut.x * sr0, ut.y * sr0), qt);
        const double2 C = make_double2(Cs.x * sl0, Cs.y * sl0);
        const double2 e = make_double2(uxm.x, -uxm.y);
        double2 h0, h1;
        if (!DAG) {
            const double2 B = cm<FOLD>(ux, make_double2(pxp.a.x - pxp.b.y, pxp.a.y + pxp.b.x));  // px0 + i px1
            const double2 E = cm<FOLD>(e, make_double2(pxm.a.x + pxm.b.y, pxm.a.y - pxm.b.x));   // pxm0 - i pxm1
            h0 = cadd(cadd(cadd(A, B), C), E);
            h1 = cadd(cadd(cadd(cneg(A), mul_mi(B)), C), mul_i(E));
        } else {
            const double2 E = cm<FOLD>(e, make_double2(pxm.a.x - pxm.b.y, pxm.a.y + pxm.b.x));   // pxm0 + i pxm1
            const double2 B = cm<FOLD>(ux, make_double2(pxp.a.x + pxp.b.y, pxp.a.y - pxp.b.x));  // px0 - i px1
            h0 = cadd(cadd(cadd(C, E), A), B);
            h1 = cadd(cadd(cadd(cneg(C), mul_mi(E)), A), mul_i(B));
        }
        // mass p - 0.5 h as fma(-0.5, h, mass p): 0.5 h is exact, so both are
        // the one rounding of (mass p) - 0.5 h
        o.a = make_double2(__builtin_fma(-0.5, h0.x, mass * p.a.x), __builtin_fma(-0.5, h0.y, mass * p.a.y));
        o.b = make_double2(__builtin_fma(-0.5, h1.x, mass * p.b.x), __builtin_fma(-0.5, h1.y, mass * p.b.y));
    } else {
        const Sp pm = shr(p), pp = shl(p);
        const double2 utm = dpp_shr1(ut);
        dirac_site<DAG>(mass, sr0, sl0, p.a, p.b, pp.a, pp.b, pxp.a, pxp.b, pm.a, pm.b, pxm.a, pxm.b, ut, ux, utm,
                        uxm, o.a, o.b);
    }
    return o;
}

__global__ void cg_ra_flush_sums_kernel(CGScalars *sc, long J) {
    double2 ab[4];
    int stop;
    ra_scalars_from_sums(sc, J + 1, ab, &stop);  // S_J into red[J & 1]
    store_state(sc, sc->red[J & 1]);
}

void launch_cg_ra_flush_sums(hipStream_t s, CGScalars *sc, long pass) {
    hipLaunchKernelGGL(cg_ra_flush_sums_kernel, dim3(1), dim3(1), 0, s, sc, pass);
}

// The row march of one tile (the kernel's body; see the header). REV = 1
// marches the chunk from its last row to its first (phys below).
// The lane group owns columns [cbase, cbase + span): a wave (cbase = g RW,
// span = RW, li = lane) or, ST, the block's t-strip (span = 64 wpb - 2 RH,
// li = threadIdx.x); its lanes cover cbase - RH + li.
template <int SH, int XP, int FOLD, int UC, int REV, int ST = 0>
__device__ __forceinline__ void ra_march(const RAArgs &a, int cbase, int span, int li, int x0, int xe, double2 alpha,
                                         double2 beta, double2 alpha2, double2 beta2, double2 *rlds, double2 *xl,
                                         double2 &acc_dA, double2 &acc_rA, double2 &acc_n) {
    const int Nx = a.Nx, Wt = a.Wt;
    // The wave owns columns [g RW, g RW + RW): its stores (lanes RH .. RW+RH-1)
    // start on a 128-B line (RW double2 = 7 lines), its 64-lane loads 64 B
    // before one (9 lines per row and plane). Shifting the window by RH so
    // the loads cover 8 lines misaligns the stores instead: 154.5 against
    // 153.3 B/site of counter bytes and 2092 against 2205 it/s (round 4,
    // interleaved bench.py, profiles/r04_a_window_shift_ab.jsonl). Partial
    // line writes cost more than a ninth line read through L2.
    const int c = cbase - RH + li;
    const bool own = li >= RH && li < span + RH && c < Wt;
    int tg = (a.t0 + c) % a.Ntg;
    if (tg < 0) tg += a.Ntg;
    const double sr0 = tg == a.Ntg - 1 ? -1.0 : 1.0;  // SignR[2n], include/dirac_operator.h:53-55
    const double sl0 = tg == 0 ? -1.0 : 1.0;          // SignL[2n], :56-58
    const double mass = a.mass;
    const RSrc<double2> S1 = rsrc<SH>(a.d1, a.f1, c, a);
    const RSrc<double2> S2 = rsrc<SH>(a.d2, a.f2, c, a);
    using LU = std::conditional_t<UC != 0, LinkCode, double2>;  // a link as loaded: code or complex
    using LV = std::conditional_t<UC != 0, double, double2>;    // its first (or only) stream
    const RSrc<LV> SU = [&] {
        if constexpr (UC != 0) return rsrc<SH>(a.Ua, a.fUa, c, a);
        else return rsrc<SH>(a.U, a.fU, c, a);
    }();
    // UC 1: the flag words, same strides as the codes (rsrc of the same column)
    const uint16_t *SF = UC == 1 ? rsrc<SH>(a.Uf, a.fUf, c, a).p : nullptr;
    // UC 2: the flag bytes of this column, one per site (in-domain rows Wt
    // apart; a received face's [col][x] rows 1 apart)
    long bxs = a.Wt;
    const uint8_t *SB = nullptr;
    if constexpr (UC == 2) {
        if (!SH) {
            int cw = c % a.Wt;
            if (cw < 0) cw += a.Wt;
            SB = a.Ub + cw;
        } else if (c >= 0 && c < a.Wt) {
            SB = a.Ub + c;
        } else {
            int fc = c < 0 ? c + RH : c - a.Wt + RH;
            fc = fc < 0 ? 0 : (fc > 2 * RH - 1 ? 2 * RH - 1 : fc);
            SB = a.fUb + (long)fc * a.Nx;
            bxs = 1;
        }
    }
    // x is read and written by the owned lanes only: the halo lanes load their
    // wave's nearest owned column (no partial line outside the owned ones;
    // 106.6 against 108.0 read B/site, profiles/r05_x_halo_variants_counters.jsonl)
    const int co = min(max(c, cbase), cbase + span - 1);
    const int cx = co < 0 ? 0 : (co >= Wt ? Wt - 1 : co);
    auto wrap = [Nx](int x) { int w = x % Nx; return w < 0 ? w + Nx : w; };
    // REV marches the chunk from its last row to its first: virtual row v
    // (the march order, x0 - 6 .. xe - 1 as forward) is physical row
    // x0 + xe - 1 - v. The x-hops then swap roles (the physical x + 1
    // neighbour is the row BEHIND in the march), and U_x is loaded one
    // physical row up (U_x(X - 1) for virtual row v), so each stage's two
    // x-links are again the current and the previous register row.
    auto phys = [x0, xe](int v) { return REV ? x0 + xe - 1 - v : v; };
    // d_{j-1}: rows x0-4 .. xe+3; U: x0-4 .. xe+2; d_{j-2}: x0-2 .. xe+1; x: owned rows
    auto ld1 = [&](int xr, Sp &d) {
        const double2 *p = S1.p + (long)wrap(phys(min(xr, xe + 3))) * S1.xs;
        d.a = p[0];
        d.b = p[S1.ps];
    };
    auto ldu = [&](int xr, LU &ut, LU &ux) {
        const int X = phys(min(xr, xe + 2));
        const long ot = (long)wrap(X) * SU.xs, ox = (REV ? (long)wrap(X - 1) * SU.xs : ot) + SU.ps;
        if constexpr (UC == 2) {
            const uint8_t bt = SB[(long)wrap(X) * bxs];
            ut = LinkCode{SU.p[ot], bt};
            ux = LinkCode{SU.p[ox], REV ? SB[(long)wrap(X - 1) * bxs] : bt};
        } else if constexpr (UC == 1) {
            ut = LinkCode{SU.p[ot], SF[ot]};
            ux = LinkCode{SU.p[ox], SF[ox]};
        } else {
            ut = SU.p[ot];
            ux = SU.p[ox];
        }
    };
    auto cvu = [](LU v, int shift) -> double2 {  // shift: the U_t (0) or U_x (4) nibble of UC 2
        if constexpr (UC != 0) return u_of<UC>(v, shift);
        else return v;
    };
    // FOLD 2 takes pre-scaled links (ra_site): U_t by -sr0/2, U_x by -1/2
    const double kt = FOLD == 2 ? -0.5 * sr0 : 1.0, kx = FOLD == 2 ? -0.5 : 1.0;
    auto cvt = [&](LU v) -> double2 {
        const double2 u = cvu(v, 0);
        return FOLD == 2 ? make_double2(u.x * kt, u.y * kt) : u;
    };
    auto cvx = [&](LU v) -> double2 {
        const double2 u = cvu(v, 4);
        return FOLD == 2 ? make_double2(u.x * kx, u.y * kx) : u;
    };
    auto ld2 = [&](int xr, Sp &q, Sp &xv) {
        const double2 *p = S2.p + (long)wrap(phys(min(max(xr, x0 - 2), xe + 1))) * S2.xs;
        q.a = p[0];
        q.b = p[S2.ps];
        if (XP && (phys(xr) & 1) == a.xpar) {  // wave-uniform: only the rows this pass updates
            const long n = (long)wrap(phys(min(max(xr, x0), xe - 1))) * Wt + cx;
            xv.a = a.x[n];
            xv.b = a.x[n + a.V];
        }
    };
    const double2 z = make_double2(0.0, 0.0);
    const Sp zs = Sp{z, z};
    // state at the top of iteration y (see the header)
    Sp D2, D3, Ld;                                   // d_{j-1}(y+2), (y+3); in flight (y+4)
    LU Lut, Lux;                                     // in flight U(y+3)
    Sp Mq, Mx = zs;                                  // in flight d_{j-2}(y+2), x(y+2)
    double2 Ut0 = z, Ut1 = z, Ut2, Ux0 = z, Ux1 = z, Ux2, Uxm = z;  // U_t(y..y+2), U_x(y-1..y+2)
    Sp P1 = zs, P2 = zs;                             // T'(y+1), T'(y+2)
    Sp J0 = zs, J1 = zs;                             // d_j at rows y, y+1
    Sp Q0 = zs, Q1 = zs;                             // T(y-1), T(y)
    const int y0 = x0 - 6;
    ld1(y0 + 2, D2);
    ld1(y0 + 3, D3);
    {
        LU t2, x2;
        ldu(y0 + 2, t2, x2);
        Ut2 = cvt(t2);
        Ux2 = cvx(x2);
    }
    ld1(y0 + 4, Ld);
    ldu(y0 + 3, Lut, Lux);
    ld2(y0 + 2, Mq, Mx);
    int s_w = 2, s_r = 0;  // LDS ring slots of r_j rows y+2 (written) and y (read)
    // stage mask M: bit 0 = S2 + S3, bit 1 = S4, bit 2 = S5 (S1 always)
    auto step = [&](int y, auto mtag) {
        constexpr int M = decltype(mtag)::value;
        const Sp D4 = Ld;
        const double2 Ut3 = cvt(Lut), Ux3 = cvx(Lux);
        double2 *const xr = ST ? xl + (y & 1) * 32 : nullptr;  // ST: this row's exchange slots, 8 per stage
        ld1(y + 5, Ld);
        ldu(y + 4, Lut, Lux);
        __builtin_amdgcn_sched_barrier(0);  // keep the next rows' loads issued here
        const Sp P3 = REV ? ra_site<FOLD, 1, ST>(mass, sr0, sl0, D3, D4, D2, Ut3, Ux2, Ux3, xr)
                          : ra_site<FOLD, 1, ST>(mass, sr0, sl0, D3, D2, D4, Ut3, Ux3, Ux2, xr);  // S1: T'(y+3)
        Sp J2 = zs, Q2 = zs;
        if constexpr ((M & 1) != 0) {
            const Sp A = REV ? ra_site<FOLD, 0, ST>(mass, sr0, sl0, P2, P3, P1, Ut2, Ux1, Ux2, xr + 8)
                             : ra_site<FOLD, 0, ST>(mass, sr0, sl0, P2, P1, P3, Ut2, Ux2, Ux1, xr + 8);  // S2: Ad_{j-1}(y+2)
            // S3: r_j, d_j at row y+2
            const int xr = y + 2;
            const Sp Q = Mq, X = Mx;
            Sp rp, R2;
            rp.a = cfms<FOLD>(D2.a, Q.a, beta2);
            rp.b = cfms<FOLD>(D2.b, Q.b, beta2);
            R2.a = cfms<FOLD>(rp.a, alpha, A.a);
            R2.b = cfms<FOLD>(rp.b, alpha, A.b);
            J2.a = cfma<FOLD>(R2.a, D2.a, beta);
            J2.b = cfma<FOLD>(R2.b, D2.b, beta);
            if (xr >= x0 && xr < xe && own) {
                const int Xr = phys(xr);
                const long n = (long)Xr * Wt + c;
                st_nt(a.dn + n, J2.a);
                st_nt(a.dn + n + a.V, J2.b);
                if (SH && a.fsend) {  // fused face pack ([col][plane][x], lo: columns 0..3, hi: Wt-4..Wt-1)
                    const int fcol = c < RH ? c : (c >= Wt - RH ? c - (Wt - RH) + RH : -1);
                    if (fcol >= 0) {
                        if (a.peer && a.pstore == 0) {  // into the neighbour's ring: 16-B write-through stores
                            // (sm_peer.h; one resource per side, both from kernel arguments: uniform)
                            const __amdgpu_buffer_rsrc_t rlo = sys_rsrc(a.fsend, 16u * 8u * Nx);
                            const __amdgpu_buffer_rsrc_t rhi = sys_rsrc(a.fsendh, 16u * 8u * Nx);
                            const int fo = 16 * ((fcol & (RH - 1)) * 2 * Nx + Xr);
                            if (fcol < RH) {
                                sys_st16(rlo, fo, J2.a);
                                sys_st16(rlo, fo + 16 * Nx, J2.b);
                            } else {
                                sys_st16(rhi, fo, J2.a);
                                sys_st16(rhi, fo + 16 * Nx, J2.b);
                            }
                        } else if (a.peer && a.pstore == 1) {  // 8-B write-through (atomic) stores (A/B)
                            double2 *fb = fcol < RH ? a.fsend + (long)(2 * fcol) * Nx : a.fsendh + (long)(2 * (fcol - RH)) * Nx;
                            sys_st(&fb[Xr].x, J2.a.x);
                            sys_st(&fb[Xr].y, J2.a.y);
                            sys_st(&fb[Nx + Xr].x, J2.b.x);
                            sys_st(&fb[Nx + Xr].y, J2.b.y);
                        } else {
                            double2 *fb = fcol < RH ? a.fsend + (long)(2 * fcol) * Nx : a.fsendh + (long)(2 * (fcol - RH)) * Nx;
                            fb[Xr] = J2.a;
                            fb[Nx + Xr] = J2.b;
                        }
                    }
                }
                if (XP && (Xr & 1) == a.xpar) {  // x_j = (x_{j-2} + alpha_{j-2} d_{j-2}) + alpha_{j-1} d_{j-1}
                    st_nt(a.x + n, cfma<FOLD>(cfma<FOLD>(X.a, alpha2, Q.a), alpha, D2.a));
                    st_nt(a.x + n + a.V, cfma<FOLD>(cfma<FOLD>(X.b, alpha2, Q.b), alpha, D2.b));
                }
                acc_n.x = nacc<FOLD>(acc_n.x, R2.a);  // Re dot(r, r), include/variables.h:185-188
                acc_n.x = nacc<FOLD>(acc_n.x, R2.b);
            }
            rlds[(2 * s_w) * blockDim.x + threadIdx.x] = R2.a;
            rlds[(2 * s_w + 1) * blockDim.x + threadIdx.x] = R2.b;
        }
        ld2(y + 3, Mq, Mx);  // consumed above: issued now, used next iteration
        if constexpr ((M & 2) != 0)  // S4: T(y+1)
            Q2 = REV ? ra_site<FOLD, 1, ST>(mass, sr0, sl0, J1, J2, J0, Ut1, Ux0, Ux1, xr + 16)
                     : ra_site<FOLD, 1, ST>(mass, sr0, sl0, J1, J0, J2, Ut1, Ux1, Ux0, xr + 16);
        if constexpr ((M & 4) != 0) {
            const Sp o = REV ? ra_site<FOLD, 0, ST>(mass, sr0, sl0, Q1, Q2, Q0, Ut0, Uxm, Ux0, xr + 24)
                             : ra_site<FOLD, 0, ST>(mass, sr0, sl0, Q1, Q0, Q2, Ut0, Ux0, Uxm, xr + 24);  // S5: Ad_j(y)
            if (own) {
                const Sp R0 = Sp{rlds[(2 * s_r) * blockDim.x + threadIdx.x], rlds[(2 * s_r + 1) * blockDim.x + threadIdx.x]};
                acc_dA = cfma<FOLD>(acc_dA, J0.a, cconj(o.a));  // dot(d, Ad)
                acc_dA = cfma<FOLD>(acc_dA, J0.b, cconj(o.b));
                acc_rA = cfma<FOLD>(acc_rA, R0.a, cconj(o.a));  // dot(r, Ad)
                acc_rA = cfma<FOLD>(acc_rA, R0.b, cconj(o.b));
                acc_n.y = nacc<FOLD>(acc_n.y, o.a);            // |Ad|^2
                acc_n.y = nacc<FOLD>(acc_n.y, o.b);
            }
        }
        D2 = D3;
        D3 = D4;
        Uxm = Ux0;
        Ut0 = Ut1;
        Ux0 = Ux1;
        Ut1 = Ut2;
        Ux1 = Ux2;
        Ut2 = Ut3;
        Ux2 = Ux3;
        P1 = P2;
        P2 = P3;
        J0 = J1;
        J1 = J2;
        Q0 = Q1;
        Q1 = Q2;
        s_w = s_w == 2 ? 0 : s_w + 1;
        s_r = s_r == 2 ? 0 : s_r + 1;
    };
    int y = y0;
    for (; y < x0 - 4; ++y) step(y, std::integral_constant<int, 0>());
    for (; y < x0 - 2; ++y) step(y, std::integral_constant<int, 1>());
    for (; y < x0; ++y) step(y, std::integral_constant<int, 3>());
    // three steps per trip: the period-3 rotations (d_{j-1}, T', d_j, T)
    // become register renaming instead of copies
    for (; y + 2 < xe; y += 3) {
        step(y, std::integral_constant<int, 7>());
        step(y + 1, std::integral_constant<int, 7>());
        step(y + 2, std::integral_constant<int, 7>());
    }
    for (; y < xe; ++y) step(y, std::integral_constant<int, 7>());
}

template <int SH, int XP, int FOLD, int RED = 0, int UC = 0, int TK = 0, int REV = 0, int ST = 0>
__global__ void __launch_bounds__(256) cg_ra_kernel(RAArgs a) {
    __shared__ double2 sh[4];
    __shared__ double2 xl[ST ? 64 : 1];  // ST: t-hop exchange, 2 row parities x 4 stages x 4 waves x (qf, bp)
    extern __shared__ double2 rlds[];  // r_j ring: 3 slots x 2 planes x blockDim (dynamic: sized by waves per block)
    CGScalars *sc = a.sc;
    // Passes 0 and 1 take zero multipliers instead of branches: pass 0 has
    // d_0 = r_0 (alpha = beta = 0), pass 1 has r_0 = d_0 (beta2 = 0). The
    // products by zero leave every value unchanged up to the sign of an exact zero.
    const double2 z2 = make_double2(0.0, 0.0);
    const bool first = a.first != 0, rebuild = a.rebuild != 0;
    double2 alpha, beta, alpha2, beta2;  // alpha_{j-1}, beta_{j-1}, alpha_{j-2}, beta_{j-2}
    if (RED) {  // every block evaluates pass j-1's scalars itself (same sums, same order)
        __shared__ double2 s_ab[4];
        __shared__ int s_stop;
        if (!first && RED == 2) {
            if (threadIdx.x == 0) ra_scalars_from_sums(sc, a.pass, s_ab, &s_stop);
        } else if (!first) {
            const CGRed s = cg1_redundant(sc, a.prev, a.TBk * a.XB, a.pass, sh);
            if (threadIdx.x == 0) {
                s_ab[0] = s.alpha;
                s_ab[1] = s.beta;
                s_ab[2] = s.alpha2;
                s_ab[3] = s.beta2;
                s_stop = s.done;
            }
        } else if (threadIdx.x == 0) {
            s_ab[0] = s_ab[1] = s_ab[2] = s_ab[3] = z2;
            s_stop = 0;
        }
        __syncthreads();
        if (s_stop) return;  // block-uniform
        // block-uniform values: into scalar registers, as the sc loads of the
        // non-redundant path are (not 16 VGPRs held across the march)
        alpha = first ? z2 : uniform_d2(s_ab[0]);
        beta = first ? z2 : uniform_d2(s_ab[1]);
        alpha2 = uniform_d2(s_ab[2]);
        beta2 = rebuild ? uniform_d2(s_ab[3]) : z2;
    } else {
        if (sc->done) return;  // grid-uniform: converged (or max_iter) in an earlier pass
        alpha = first ? z2 : sc->alpha;
        beta = first ? z2 : sc->beta;
        alpha2 = sc->alpha2;
        beta2 = rebuild ? sc->beta2 : z2;
    }
    int tb, tbr, xc;
    {
        int w = blockIdx.x;
        const int n = a.tbn * a.XB;
        if (a.remap) {  // each XCD takes a contiguous range of tiles: its own x-chunks (L2 reuse of halo rows)
            const int q = n >> 3, rr = n & 7, xcd = w & 7;
            const int len = xcd < rr ? q + 1 : q;
            // t-adjacent tiles consecutive. (Round 5: taking the range
            // t-block-major instead, so every x-adjacent pair of the XCD's
            // chunks starts together, changed the read bytes by 0.1 % and was
            // slower, profiles/r05_i_remap2.jsonl.)
            const int i = a.flip ? len - 1 - (w >> 3) : (w >> 3);  // flip: the XCD's tiles in reverse order
            w = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + i;
        } else if (a.flip) {
            w = n - 1 - w;
        }
        tbr = w % a.tbn;
        xc = w / a.tbn;
        tb = a.tb0 + tbr;
        if (tb >= a.TBk) tb -= a.TBk;  // edge block-columns TBk-1 and 0 in one launch
    }
    const int lane = threadIdx.x & 63;
    // ST: the block's waves share strip tb (every wave marches, in step: the
    // stages' barriers); else each wave owns its own window g
    const int g = tb * a.wpb + (threadIdx.x >> 6);
    const int span = ST ? 64 * a.wpb - 2 * RH : RW;
    const int cbase = ST ? tb * span : g * RW;
    const int x0 = a.xbal ? (int)((long)xc * a.Nx / a.XB) : xc * a.xchunk;
    const int xe = a.xbal ? (int)((long)(xc + 1) * a.Nx / a.XB) : min(a.Nx, x0 + a.xchunk);
    double2 acc_dA = make_double2(0.0, 0.0), acc_rA = make_double2(0.0, 0.0);
    double2 acc_n = make_double2(0.0, 0.0);  // (|r|^2, |Ad|^2)
    if ((ST || g < a.NWT) && x0 < xe) {  // ST: block-uniform
        // REV 0 / 1: every tile forward / backward; REV 2: per tile, backward
        // iff (x-chunk parity & alt) ^ flip, so x-adjacent chunks march
        // towards their shared boundary rows at the same time (alt = 1)
        const bool back = REV == 1 || (REV == 2 && (((xc & a.alt) ^ a.flip) & 1));
        const int li = ST ? (int)threadIdx.x : lane;
        if (REV != 0 && back)
            ra_march<SH, XP, FOLD, UC, 1, ST>(a, cbase, span, li, x0, xe, alpha, beta, alpha2, beta2, rlds, xl, acc_dA,
                                              acc_rA, acc_n);
        else if (REV != 1)
            ra_march<SH, XP, FOLD, UC, 0, ST>(a, cbase, span, li, x0, xe, alpha, beta, alpha2, beta2, rlds, xl, acc_dA,
                                              acc_rA, acc_n);
    }
    const double2 s0 = block_sum(acc_dA, sh);
    __syncthreads();
    const double2 s1 = block_sum(acc_rA, sh);
    __syncthreads();
    const double2 s2 = block_sum(acc_n, sh);
    const long tile = a.pbase + (long)tbr * a.XB + xc;
    double2 *p = a.partials + 3 * tile;  // one slot per tile
    if (!TK) {
        if (threadIdx.x == 0) {
            p[0] = s0;
            p[1] = s1;
            p[2] = s2;
        }
        return;
    }
    cg_ticketed_tail(a.partials, tile, a.ntiles, a.tick, a.gsum, a.out3, sc, a.first, s0, s1, s2, SH ? a.peer : nullptr, a.pseq);
}

CGFusedCfg cg_ra_config(const Geometry &g) {
    CGFusedCfg c;
    c.NWT = (g.Wt + RW - 1) / RW;
    c.wpb = 4;
    c.TBk = (c.NWT + c.wpb - 1) / c.wpb;
    // rows per block: a chunk re-reads 8 halo rows of d_{j-1} (4 per side) and
    // runs 6 prologue steps, so chunks stay long where the grid is big enough
    // (tools/tune_cg.py, ms per iteration: 4096^2 32 rows 0.588 vs 16 0.604
    // vs 64 0.596; 2048^2 16 rows 0.174 vs 12 0.183; 1024^2 12 rows 0.054 vs
    // 16 0.063). Smaller lattices fill the chip first (>= 2 rows).
    if (g.Nx >= 1024) {
        c.xchunk = g.Nx >= 4096 ? 32 : (g.Nx >= 2048 ? 16 : 12);
    } else {
        int nchunks = (2048 + c.TBk - 1) / c.TBk;
        if (nchunks > g.Nx) nchunks = g.Nx;
        if (nchunks < 1) nchunks = 1;
        c.xchunk = (g.Nx + nchunks - 1) / nchunks;
        if (c.xchunk < 2) c.xchunk = 2;
    }
    // Shard shapes of the BASELINE configs (4096^2 and its t-shards over 2/4/8
    // GPUs, 8192^2 and its 8-way shard, 2048^2): measured in the library's own
    // CG loop (tools/tune_shapes.py, profiles/r02_tune_shapes.jsonl; ms per
    // iteration against the rule above): 4096x4096 one-wave blocks of 64 rows
    // 0.477 vs 0.484; 4096x2048 1/32 0.257 vs 0.263; 4096x1024 1/40 0.141 vs
    // 0.169; 4096x512 1/48 0.068 vs 0.079; 8192x8192 4/48 1.798 vs 1.820;
    // 8192x1024 1/40 0.253 vs 0.260; 2048x2048 1/40 0.140 vs 0.151. Other
    // shapes of >= 2048 rows take one-wave blocks of 40 rows.
    // Re-checked after the ticketed tail and the x row parity
    // (profiles/r02_v9_reshape.log, same box per line): 8192^2 4/32 1.741 vs
    // 4/48 1.78-1.92; 8192x1024 1/32 0.2635 vs 1/40 0.2650; 2048^2 1/64 0.142
    // vs 1/40 0.146; the others unchanged. At 4096 columns chunk lengths that
    // are not powers of two are ~10 % slower (48 / 80 / 96 rows 0.538-0.541
    // against 0.488 for 32 and 64).
    // March schedule (one shard, ticketed tail; round 3, interleaved bench
    // runs on one box): 1 = odd passes reversed, 2 = alternating x-chunks as
    // well. 4096^2: 2090 / 2090 it/s for 2 against 2065 / 2061 for 1 and
    // 2049 / 2044 all forward; 8192^2 (config 5, 4-wave blocks): 7.92-7.95 s
    // for 1 against 8.24 s for 2 and 8.48 s all forward
    // (profiles/r03_ij_march_schedule_ab.jsonl, r03_n_c5_march_schedule.jsonl).
    // Round 6: 4096^2 takes 40 balanced chunks (102-103 rows; 74 x 40 = 2960
    // one-wave tiles) instead of 64 chunks of 64 rows: 2327-2336 against
    // 2277-2284 it/s in four interleaved bench pairs, each its own context
    // and placement probe (profiles/r06_ag_chunks40_bench_ab.jsonl). The
    // optimum is sharp -- 38 / 42 chunks are 2-8 % slower than 64 rows
    // (r06_af_chunk_count_scan.jsonl) -- so it is a measured point, not a rule.
    // 4096 x 512 (config 4's 8-GPU shard) takes 28 rows instead of 48: RCCL
    // loopback 0.0849 / 0.0856 against 0.0889 / 0.0885 ms per iteration, one
    // shard 0.0697 / 0.0700 against 0.0716 / 0.0718 (two interleaved scans,
    // r06_aj_tshard_rows_4096x512.jsonl).
    c.rev_odd = 1;
    static const int kShapes[][6] = {  // Nx, Wt, waves per block, rows per block, march schedule, balanced chunks
        {4096, 4096, 1, 103, 2, 1}, {4096, 2048, 1, 32, 1, 0}, {4096, 1024, 1, 40, 1, 0}, {4096, 512, 1, 28, 1, 0},
        {8192, 8192, 4, 32, 1, 0},  {8192, 1024, 1, 32, 1, 0}, {2048, 2048, 1, 64, 1, 0},
    };
    bool known = false;
    for (const auto &k : kShapes)
        if (k[0] == g.Nx && k[1] == g.Wt) {
            c.wpb = k[2];
            c.xchunk = k[3];
            c.rev_odd = k[4];
            c.xbal = k[5];
            known = true;
        }
    if (!known && g.Nx >= 2048 && g.Wt >= 256) {
        c.wpb = 1;
        c.xchunk = 40;
    }
    c.TBk = (c.NWT + c.wpb - 1) / c.wpb;
    c.XB = (g.Nx + c.xchunk - 1) / c.xchunk;
    c.remap = 1;
    // 1: folded bracket, 0.604 vs 0.625 ms per iteration at 4096^2 against the
    // exact bracket arithmetic; 2: plus fused multiply-adds, ~1 % faster again
    // (tools/ab_fold.sh, ABBA: 0.513-0.517 vs 0.519-0.520 ms burst, 0.548-0.554
    // vs 0.552-0.557 sustained)
    c.fold = 2;
    return c;
}

// stop != null: the launch itself records the event at the kernel's end
// (hipExtLaunchKernelGGL), so a stream that waits for this kernel needs no
// marker packet behind it on the launching stream (~3 us per cross-stream
// hand-off, tools/stream_gap_probe.hip)
template <typename K>
static void ra_launch(K kern, dim3 grid, dim3 block, size_t lds, hipStream_t s, const RAArgs &a, hipEvent_t stop) {
    if (stop) hipExtLaunchKernelGGL(kern, grid, block, (uint32_t)lds, s, nullptr, stop, 0u, a);
    else hipLaunchKernelGGL(kern, grid, block, lds, s, a);
}

template <int SH, int RED, int UC, int F>
static void ra_go(int xp, int tk, dim3 grid, dim3 block, size_t lds, hipStream_t s, const RAArgs &a, int rev = 0,
                  hipEvent_t stop = nullptr) {
    // march schedules: one-shard tail passes, and the peer transport's one-launch t-shard pass
    if constexpr (F == 2 && ((SH == 0 && RED == 0) || (SH == 1 && RED == 2))) {
        if (tk && rev == 1) {
            if (xp) ra_launch(cg_ra_kernel<SH, 1, F, RED, UC, 1, 1>, grid, block, lds, s, a, stop);
            else ra_launch(cg_ra_kernel<SH, 0, F, RED, UC, 1, 1>, grid, block, lds, s, a, stop);
            return;
        }
        if (tk && rev == 2) {
            if (xp) ra_launch(cg_ra_kernel<SH, 1, F, RED, UC, 1, 2>, grid, block, lds, s, a, stop);
            else ra_launch(cg_ra_kernel<SH, 0, F, RED, UC, 1, 2>, grid, block, lds, s, a, stop);
            return;
        }
    }
    if constexpr (F == 2) {
        if (tk) {
            if (xp) ra_launch(cg_ra_kernel<SH, 1, F, RED, UC, 1>, grid, block, lds, s, a, stop);
            else ra_launch(cg_ra_kernel<SH, 0, F, RED, UC, 1>, grid, block, lds, s, a, stop);
            return;
        }
    }
    if (xp) ra_launch(cg_ra_kernel<SH, 1, F, RED, UC, 0>, grid, block, lds, s, a, stop);
    else ra_launch(cg_ra_kernel<SH, 0, F, RED, UC, 0>, grid, block, lds, s, a, stop);
}

template <int UC>
static void ra_strip(int xp, int rev, dim3 grid, dim3 block, size_t lds, hipStream_t s, const RAArgs &a) {
    if (rev == 2) {
        if (xp) hipLaunchKernelGGL((cg_ra_kernel<0, 1, 2, 0, UC, 1, 2, 1>), grid, block, lds, s, a);
        else hipLaunchKernelGGL((cg_ra_kernel<0, 0, 2, 0, UC, 1, 2, 1>), grid, block, lds, s, a);
    } else if (rev == 1) {
        if (xp) hipLaunchKernelGGL((cg_ra_kernel<0, 1, 2, 0, UC, 1, 1, 1>), grid, block, lds, s, a);
        else hipLaunchKernelGGL((cg_ra_kernel<0, 0, 2, 0, UC, 1, 1, 1>), grid, block, lds, s, a);
    } else {
        if (xp) hipLaunchKernelGGL((cg_ra_kernel<0, 1, 2, 0, UC, 1, 0, 1>), grid, block, lds, s, a);
        else hipLaunchKernelGGL((cg_ra_kernel<0, 0, 2, 0, UC, 1, 0, 1>), grid, block, lds, s, a);
    }
}

int launch_cg_ra(hipStream_t s, const Geometry &g, const CGFusedCfg &c, int nshard, const double2 *d1,
                 const double2 *d2, double2 *dn, double2 *x, const double2 *U, const double2 *f1,
                  const double2 *f2, const double2 *fU, double mass, long pass, CGScalars *sc, double2 *partials,
                  int tb0, int tbn, const double2 *prev_partials, const double *Uang, const double *fUang,
                  double2 *fsend, int pbase, unsigned *tick, int ntiles, double2 *gsum, double2 *out3,
                  int red_sums, int link_fmt, double2 *fsendh, const PeerView *peer, unsigned long long pseq,
                  int pstore, int sched, hipEvent_t stop) {
    if (tbn <= 0) return 0;
    RAArgs a;
    a.d1 = d1; a.d2 = d2; a.dn = dn; a.x = x; a.U = U;
    a.f1 = f1; a.f2 = f2; a.fU = fU;
    a.sc = sc; a.partials = partials;
    a.V = g.V; a.Nx = g.Nx; a.Wt = g.Wt; a.t0 = g.t0; a.Ntg = g.Ntg;
    a.xchunk = c.xchunk; a.NWT = c.NWT; a.TBk = c.TBk; a.XB = c.XB; a.remap = c.remap; a.wpb = c.wpb;
    a.first = pass == 0;
    a.rebuild = pass >= 2;  // pass 1 has r_0 = d_0 (no d_{-1})
    a.tb0 = tb0;
    a.tbn = tbn;
    a.mass = mass;
    a.prev = prev_partials;
    a.pass = pass;
    a.Ua = Uang;
    a.fUa = fUang;
    // flag words right after the codes, flag bytes right after the flag words
    a.Uf = Uang ? reinterpret_cast<const uint16_t *>(Uang + 2 * g.V) : nullptr;
    a.fUf = fUang ? reinterpret_cast<const uint16_t *>(fUang + 16 * (long)g.Nx) : nullptr;
    a.Ub = Uang ? reinterpret_cast<const uint8_t *>(a.Uf + 2 * g.V) : nullptr;
    a.fUb = fUang ? reinterpret_cast<const uint8_t *>(a.fUf + 16 * (long)g.Nx) : nullptr;
    a.fsend = fsend;
    a.fsendh = fsendh ? fsendh : (fsend ? fsend + 8 * (long)g.Nx : nullptr);
    a.peer = peer;
    a.pseq = pseq;
    a.pstore = pstore;
    a.pbase = pbase;
    a.tick = tick;
    a.ntiles = ntiles;
    a.gsum = gsum;
    a.out3 = out3;
    a.flip = 0;
    a.alt = 0;
    a.xbal = c.xbal;
    const dim3 grid(tbn * c.XB), block(64 * c.wpb);
    const size_t lds = sizeof(double2) * 6 * 64 * c.wpb;  // the r_j ring
    // x takes passes j-1 and j together, on the rows of parity j & 1: every
    // pass from 1 on updates half the rows (pass 1: alpha_{-1} = 0)
    const int xp = pass >= 1;
    a.xpar = (int)(pass & 1);
    // one kernel per (shards, x pass, fold, scalar mode, link form, tail) combination
    const int f = c.fold >= 2 ? 2 : (c.fold ? 1 : 0);
    const int uc = Uang && f == 2 ? (link_fmt == 2 ? 2 : 1) : 0;  // link codes: with the fused multiply-add fold only
    const int link_bytes = uc == 2 ? 17 : (uc ? 20 : 32);
    const int tk = tick != nullptr && f == 2;
    if (prev_partials && nshard == 1 && f == 2 && tb0 == 0 && tbn == c.TBk && !c.strip) {
        if (uc == 2) ra_go<0, 1, 2, 2>(xp, 0, grid, block, lds, s, a);
        else if (uc) ra_go<0, 1, 1, 2>(xp, 0, grid, block, lds, s, a);
        else ra_go<0, 1, 0, 2>(xp, 0, grid, block, lds, s, a);
        return link_bytes;
    }
    const bool sh = nshard > 1;
    if (red_sums && sh && f == 2 && tk) {  // t-shards: scalars from pass j-1's all-reduced sums (sc->sumr)
        // the peer transport's pass is one launch over every t-block, so it can
        // take the shape's march schedule (sched: where a one-shard pass of the
        // same grid would, i.e. with the ticketed tail) as a one-shard pass does (odd passes
        // in reverse tile order, marching backwards; rev 2: x-adjacent chunks
        // in opposite directions); the split RCCL / host-staged launches cannot
        int prev = 0;
        if (sched && tb0 == 0 && tbn == c.TBk && c.rev_odd == 1 && (pass & 1)) {
            prev = 1;
            a.flip = 1;
        } else if (sched && tb0 == 0 && tbn == c.TBk && c.rev_odd == 2) {
            prev = 2;
            a.flip = (int)(pass & 1);
            a.alt = 1;
        }
        if (uc == 2) ra_go<1, 2, 2, 2>(xp, tk, grid, block, lds, s, a, prev, stop);
        else if (uc) ra_go<1, 2, 1, 2>(xp, tk, grid, block, lds, s, a, prev, stop);
        else ra_go<1, 2, 0, 2>(xp, tk, grid, block, lds, s, a, prev, stop);
        return link_bytes;
    }
    // one shard with the ticketed tail: odd passes take the tiles in reverse
    // order and flip the march direction, so a pass starts on the rows its
    // predecessor touched last (still in the XCD's L2 / the Infinity Cache)
    // instead of the ones it touched first. rev_odd 1: every tile of an odd
    // pass marches backwards (REV 1 kernel); rev_odd 2: x-adjacent chunks
    // also march in opposite directions, towards / away from their shared
    // halo rows together (REV 2 kernel, both marches)
    int rev = 0;
    a.flip = 0;
    a.alt = 0;
    if (!sh && tk && f == 2 && c.rev_odd == 1 && (pass & 1)) {
        rev = 1;
        a.flip = 1;
    } else if (!sh && tk && f == 2 && c.rev_odd == 2) {
        rev = 2;
        a.flip = (int)(pass & 1);
        a.alt = 1;
    }
    if (c.strip && !sh && tk && f == 2) {  // t-strip blocks (one shard, ticketed tail)
        if (uc == 2) ra_strip<2>(xp, rev, grid, block, lds, s, a);
        else if (uc) ra_strip<1>(xp, rev, grid, block, lds, s, a);
        else ra_strip<0>(xp, rev, grid, block, lds, s, a);
        return link_bytes;
    }
    if (f == 2) {
        if (uc == 2) {
            if (sh) ra_go<1, 0, 2, 2>(xp, tk, grid, block, lds, s, a);
            else ra_go<0, 0, 2, 2>(xp, tk, grid, block, lds, s, a, rev);
        } else if (uc) {
            if (sh) ra_go<1, 0, 1, 2>(xp, tk, grid, block, lds, s, a);
            else ra_go<0, 0, 1, 2>(xp, tk, grid, block, lds, s, a, rev);
        } else {
            if (sh) ra_go<1, 0, 0, 2>(xp, tk, grid, block, lds, s, a);
            else ra_go<0, 0, 0, 2>(xp, tk, grid, block, lds, s, a, rev);
        }
    } else if (f == 1) {
        if (sh) ra_go<1, 0, 0, 1>(xp, 0, grid, block, lds, s, a);
        else ra_go<0, 0, 0, 1>(xp, 0, grid, block, lds, s, a);
    } else {
        if (sh) ra_go<1, 0, 0, 0>(xp, 0, grid, block, lds, s, a);
        else ra_go<0, 0, 0, 0>(xp, 0, grid, block, lds, s, a);
    }
    return link_bytes;
}

// Resident blocks of the t-shard pass per CU (the edge-rows rule in
// sm_capi.cpp cg_ra_pass): what the runtime computes for the kernel the
// sharded pass launches (x-updating, ticketed tail, scalars from the
// all-reduced sums), at this geometry's block size and LDS ring, so a change
// of the kernel's register or LDS use moves the rule with it.
int cg_ra_set_strip(CGFusedCfg &c, const Geometry &g, int strip) {
    c.strip = strip ? 1 : 0;
    if (c.strip) {
        if (c.wpb != 2 && c.wpb != 4) c.wpb = 4;  // strips of 2 or 4 waves (128 / 256 lanes)
        c.TBk = (g.Wt + 64 * c.wpb - 2 * RH - 1) / (64 * c.wpb - 2 * RH);
    } else {
        c.TBk = (c.NWT + c.wpb - 1) / c.wpb;
    }
    return c.TBk;
}

int cg_ra_shard_blocks_per_cu(const CGFusedCfg &c, int link_fmt) {
    const int block = 64 * c.wpb;
    const size_t lds = sizeof(double2) * 6 * 64 * c.wpb;
    int n = 0;
    hipError_t e;
    if (link_fmt == 2) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, cg_ra_kernel<1, 1, 2, 2, 2, 1>, block, lds);
    else if (link_fmt == 1) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, cg_ra_kernel<1, 1, 2, 2, 1, 1>, block, lds);
    else e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, cg_ra_kernel<1, 1, 2, 2, 0, 1>, block, lds);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    return n;
}

// Link codes for the UC passes (sm_linkcode.h) for each of the n links (both
// planes): codes v into Ua[0, n), flag words into the n uint16 after them, and
// per block the count of links that are NOT encodable bitwise -- each code is
// decoded again with the pass's own decoder and compared with the stored bits
// (one such link and the field keeps the complex-link passes, sm_capi.cpp).
__global__ void __launch_bounds__(256) link_code_kernel(long n, const double2 *U, double *Ua, double2 *part) {
    __shared__ double2 sh[4];
    uint16_t *Uf = reinterpret_cast<uint16_t *>(Ua + n);
    double bad = 0.0, wide = 0.0;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
        const double2 u = U[i];
        double v, c2, s2;
        uint16_t f;
        const int ok = sm_link_encode(u.x, u.y, &v, &f);
        sm_link_decode(v, f, &c2, &s2);
        Ua[i] = v;
        Uf[i] = f;
        if (!ok || sm_lc_bits(c2) != sm_lc_bits(u.x) || sm_lc_bits(s2) != sm_lc_bits(u.y)) bad += 1.0;
        if (sm_lc_nibble(f) == 0xff) wide += 1.0;  // needs the 16-bit flag word
    }
    const double2 b = block_sum(make_double2(bad, wide), sh);
    if (threadIdx.x == 0) part[blockIdx.x] = b;
}

int launch_link_codes(hipStream_t s, long n, const double2 *U, double *Ua, double2 *partials) {
    const int nb = reduce_blocks(n);
    hipLaunchKernelGGL(link_code_kernel, dim3(nb), dim3(256), 0, s, n, U, Ua, partials);
    return nb;
}

// Diagnostic: encode and decode every link on the device; the rebuilt links
// (nullable out), per block (links not rebuilt bitwise, largest |difference|).
__global__ void __launch_bounds__(256) link_code_check_kernel(long n, const double2 *U, double2 *out,
                                                             double2 *part) {
    __shared__ double2 sh[4];
    __shared__ double shm[256];
    double bad = 0.0, mx = 0.0;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
        const double2 u = U[i];
        double v, c2, s2;
        uint16_t f;
        const int ok = sm_link_encode(u.x, u.y, &v, &f);
        sm_link_decode(v, f, &c2, &s2);
        if (out) out[i] = make_double2(c2, s2);
        const double err = fmax(fabs(c2 - u.x), fabs(s2 - u.y));
        if (!ok || sm_lc_bits(c2) != sm_lc_bits(u.x) || sm_lc_bits(s2) != sm_lc_bits(u.y)) bad += 1.0;
        mx = err > mx || err != err ? err : mx;
    }
    shm[threadIdx.x] = mx;
    const double2 b = block_sum(make_double2(bad, 0.0), sh);
    __syncthreads();
    if (threadIdx.x == 0) {
        double m = 0.0;
        for (int t = 0; t < (int)blockDim.x; ++t) m = shm[t] > m || shm[t] != shm[t] ? shm[t] : m;
        part[blockIdx.x] = make_double2(b.x, m);
    }
}

int launch_link_code_check(hipStream_t s, long n, const double2 *U, double2 *out, double2 *partials) {
    const int nb = reduce_blocks(n);
    hipLaunchKernelGGL(link_code_check_kernel, dim3(nb), dim3(256), 0, s, n, U, out, partials);
    return nb;
}

// Flag bytes of the packed form (sm_linkcode.h sm_lc_nibble): byte i of Ub =
// the nibbles of flag words i (low) and i + ps (high), for i < m. Main field:
// m = V, ps = V (U_t, U_x planes); faces [col][plane][x]: called per column.
__global__ void __launch_bounds__(256) link_nibbles_kernel(long m, long ps, long rows, long rs, const uint16_t *Uf,
                                                           uint8_t *Ub, long bs) {
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < m * rows; i += (long)gridDim.x * blockDim.x) {
        const long r = i / m, k = i - r * m;
        const uint16_t *f = Uf + r * rs;
        Ub[r * bs + k] = (uint8_t)(sm_lc_nibble(f[k]) | (sm_lc_nibble(f[k + ps]) << 4));
    }
}

void launch_link_nibbles(hipStream_t s, long V, const double *Ua) {
    const uint16_t *Uf = reinterpret_cast<const uint16_t *>(Ua + 2 * V);
    uint8_t *Ub = const_cast<uint8_t *>(reinterpret_cast<const uint8_t *>(Uf + 2 * V));
    hipLaunchKernelGGL(link_nibbles_kernel, dim3(reduce_blocks(V)), dim3(256), 0, s, V, V, 1L, 0L, Uf, Ub, 0L);
}

void launch_face_nibbles(hipStream_t s, int Nx, const double *fUa) {
    // 8 columns of [plane][x] flag words -> 8 columns of [x] bytes
    const long n = 16L * Nx;
    const uint16_t *Uf = reinterpret_cast<const uint16_t *>(fUa + n);
    uint8_t *Ub = const_cast<uint8_t *>(reinterpret_cast<const uint8_t *>(Uf + n));
    hipLaunchKernelGGL(link_nibbles_kernel, dim3((unsigned)((8L * Nx + 255) / 256)), dim3(256), 0, s, (long)Nx,
                       (long)Nx, 8L, 2L * Nx, Uf, Ub, (long)Nx);
}

// After the last pass J = k of the recompute-Ad CG, the rows of parity
// != (k & 1) still lack alpha_{k-1} d_{k-1} (their last update was pass k-1).
// A stopping evaluation keeps alpha = alpha_{k-1}; a non-final one has moved it
// to alpha2 (as cg_td_finish_x_kernel).
__global__ void __launch_bounds__(256) cg_ra_finish_x_kernel(long V, int Wt, double2 *x, const double2 *d0,
                                                             const double2 *d1, const double2 *d2,
                                                             const CGScalars *sc) {
    const int k = sc->k;
    if (k < 1) return;
    const double2 alpha = sc->done ? sc->alpha : sc->alpha2;
    const int i3 = (k - 1) % 3;
    const double2 *d = i3 == 0 ? d0 : (i3 == 1 ? d1 : d2);
    const int par = k & 1;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < 2 * V; i += (long)gridDim.x * blockDim.x) {
        const long site = i < V ? i : i - V;
        if ((int)((site / Wt) & 1) != par) x[i] = cfma<2>(x[i], alpha, d[i]);
    }
}

void launch_cg_ra_finish_x(hipStream_t s, const Geometry &g, double2 *x, const double2 *d0, const double2 *d1,
                           const double2 *d2, const CGScalars *sc) {
    hipLaunchKernelGGL(cg_ra_finish_x_kernel, dim3(reduce_blocks(2 * g.V)), dim3(256), 0, s, g.V, g.Wt, x, d0, d1, d2,
                       sc);
}

// k-deep t-faces: columns 0..k-1 go down (arrive as Wt..Wt+k-1), columns
// Wt-k..Wt-1 go up (arrive as -k..-1). Buffers [col][plane][x], 2k*Nx complex.
__global__ void pack_faces_k_kernel(int Nx, int Wt, long V, int k, const double2 *f, double2 *lo, double2 *hi) {
    const int x = blockIdx.x * blockDim.x + threadIdx.x;
    if (x >= Nx) return;
    const long row = (long)x * Wt;
    for (int col = 0; col < k; ++col)
        for (int p = 0; p < 2; ++p) {
            lo[(long)(col * 2 + p) * Nx + x] = f[row + col + p * V];
            hi[(long)(col * 2 + p) * Nx + x] = f[row + Wt - k + col + p * V];
        }
}

void launch_pack_faces_k(hipStream_t s, const Geometry &g, int k, const double2 *field, double2 *lo, double2 *hi) {
    hipLaunchKernelGGL(pack_faces_k_kernel, dim3((g.Nx + 63) / 64), dim3(64), 0, s, g.Nx, g.Wt, g.V, k, field,
                       lo, hi);
}

}  // namespace sm
