// sm_device.h -- device-side helpers shared by the gfx950 kernels:
// std::complex<double> arithmetic with GCC's exact semantics (no contraction),
// the Wilson-Dirac site stencil, deterministic block reduction, DPP lane shifts.
#pragma once
#include <hip/hip_runtime.h>

#include "sm_internal.h"
#include "sm_peer.h"

#pragma clang fp contract(off)

namespace sm {

// ---- complex<double> with std::complex / GCC semantics --------------------
__device__ __forceinline__ double2 cadd(double2 a, double2 b) { return make_double2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ double2 csub(double2 a, double2 b) { return make_double2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ double2 cneg(double2 a) { return make_double2(-a.x, -a.y); }
__device__ __forceinline__ double2 cconj(double2 a) { return make_double2(a.x, -a.y); }
// GCC expansion of complex multiply: (ac - bd, ad + bc), separately rounded.
__device__ __forceinline__ double2 cmul(double2 a, double2 b) {
    return make_double2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
__device__ __forceinline__ double2 rmul(double s, double2 a) { return make_double2(s * a.x, s * a.y); }

// libgcc __divdc3 as shipped with GCC 11 (std::complex<double> division).
__device__ __forceinline__ double2 cdiv(double a, double b, double c, double d) {
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
    return make_double2(x, y);
}

#define I_NUM make_double2(0.0, 1.0)      /* I_number, src/dirac_operator.cpp:3 */
#define MI_NUM make_double2(-0.0, -1.0)   /* -I_number                         */

// One site of D (eq. 34; src/dirac_operator.cpp:31-43) or D^dagger
// (eqs. 35-36; :255-267). Hop coefficients a,b (forward) c,e (backward)
// carry the gauge link times the boundary sign, exactly as (U*Sign)*combo.
// Hopping bracket of eq. (34) (DAG = 0) / eqs. (35)-(36) (DAG = 1) at one site:
// D psi = mass psi - 0.5 * bracket, the four terms summed in the reference's
// order. p*: t+1 neighbour (pt), x+1 (px), t-1 (pm), x-1 (pxm); Ut, Ux: links
// of this site, Utm = U_t(n - t^), Uxm = U_x(n - x^); sr0 / sl0: the
// antiperiodic signs of the forward / backward t hop.
template <int DAG>
__device__ __forceinline__ void dirac_bracket(double sr0, double sl0, double2 pt0, double2 pt1, double2 px0,
                                              double2 px1, double2 pm0, double2 pm1, double2 pxm0,
                                              double2 pxm1, double2 Ut, double2 Ux, double2 Utm, double2 Uxm,
                                              double2 &h0, double2 &h1) {
    const double2 one = make_double2(1.0, 0.0);
    const double2 a = cmul(Ut, make_double2(sr0, 0.0));
    const double2 b = cmul(Ux, one);
    const double2 c = cmul(cconj(Utm), make_double2(sl0, 0.0));
    const double2 e = cmul(cconj(Uxm), one);
    if (!DAG) {
        double2 A = cmul(a, csub(pt0, pt1));
        double2 B = cmul(b, cadd(px0, cmul(I_NUM, px1)));
        double2 C = cmul(c, cadd(pm0, pm1));
        double2 E = cmul(e, csub(pxm0, cmul(I_NUM, pxm1)));
        h0 = cadd(cadd(cadd(A, B), C), E);
        A = cmul(a, cadd(cneg(pt0), pt1));
        B = cmul(b, cadd(cmul(MI_NUM, px0), px1));
        E = cmul(e, cadd(cmul(I_NUM, pxm0), pxm1));
        h1 = cadd(cadd(cadd(A, B), C), E);
    } else {
        double2 C = cmul(c, csub(pm0, pm1));
        double2 E = cmul(e, cadd(pxm0, cmul(I_NUM, pxm1)));
        double2 A = cmul(a, cadd(pt0, pt1));
        double2 B = cmul(b, csub(px0, cmul(I_NUM, px1)));
        h0 = cadd(cadd(cadd(C, E), A), B);
        C = cmul(c, cadd(cneg(pm0), pm1));
        E = cmul(e, cadd(cmul(MI_NUM, pxm0), pxm1));
        B = cmul(b, cadd(cmul(I_NUM, px0), px1));
        h1 = cadd(cadd(cadd(C, E), A), B);
    }
}

// dirac_bracket with its products by 0, +-1 and +-i folded into sign flips and
// swaps: (U*Sign) = (Re U * s, Im U * s), U*1 = U, i*p = (-Im p, Re p). For
// finite operands every value equals dirac_bracket's up to the sign of an
// exact zero. The second spin component reuses the first one's four products:
// its terms are exact negations / i-rotations of them (D: -A, -iB, C, iE;
// D^dag: -C, -iE, A, iB), since IEEE negation commutes exactly with every
// product and sum here. 4 complex products instead of 7: ~56 instead of ~114
// fp64 operations (the CG pass of sm_cgra.hip, not the bitwise operator path).
__device__ __forceinline__ double2 mul_i(double2 z) { return make_double2(-z.y, z.x); }
__device__ __forceinline__ double2 mul_mi(double2 z) { return make_double2(z.y, -z.x); }

template <int DAG>
__device__ __forceinline__ void dirac_bracket_folded(double sr0, double sl0, double2 pt0, double2 pt1, double2 px0,
                                                     double2 px1, double2 pm0, double2 pm1, double2 pxm0,
                                                     double2 pxm1, double2 Ut, double2 Ux, double2 Utm, double2 Uxm,
                                                     double2 &h0, double2 &h1) {
    const double2 a = make_double2(Ut.x * sr0, Ut.y * sr0);
    const double2 b = Ux;
    const double2 c = make_double2(Utm.x * sl0, -(Utm.y * sl0));
    const double2 e = make_double2(Uxm.x, -Uxm.y);
    if (!DAG) {
        const double2 A = cmul(a, csub(pt0, pt1));
        const double2 B = cmul(b, make_double2(px0.x - px1.y, px0.y + px1.x));      // px0 + i px1
        const double2 C = cmul(c, cadd(pm0, pm1));
        const double2 E = cmul(e, make_double2(pxm0.x + pxm1.y, pxm0.y - pxm1.x));  // pxm0 - i pxm1
        h0 = cadd(cadd(cadd(A, B), C), E);
        h1 = cadd(cadd(cadd(cneg(A), mul_mi(B)), C), mul_i(E));  // a(-pt0+pt1), b(-i px0+px1), e(i pxm0+pxm1)
    } else {
        const double2 C = cmul(c, csub(pm0, pm1));
        const double2 E = cmul(e, make_double2(pxm0.x - pxm1.y, pxm0.y + pxm1.x));  // pxm0 + i pxm1
        const double2 A = cmul(a, cadd(pt0, pt1));
        const double2 B = cmul(b, make_double2(px0.x + px1.y, px0.y - px1.x));      // px0 - i px1
        h0 = cadd(cadd(cadd(C, E), A), B);
        h1 = cadd(cadd(cadd(cneg(C), mul_mi(E)), A), mul_i(B));  // c(-pm0+pm1), e(-i pxm0+pxm1), b(i px0+px1)
    }
}

template <int DAG>
__device__ __forceinline__ void dirac_site_folded(double mass, double sr0, double sl0, double2 p0, double2 p1,
                                                  double2 pt0, double2 pt1, double2 px0, double2 px1, double2 pm0,
                                                  double2 pm1, double2 pxm0, double2 pxm1, double2 Ut, double2 Ux,
                                                  double2 Utm, double2 Uxm, double2 &s0, double2 &s1) {
    double2 h0, h1;
    dirac_bracket_folded<DAG>(sr0, sl0, pt0, pt1, px0, px1, pm0, pm1, pxm0, pxm1, Ut, Ux, Utm, Uxm, h0, h1);
    s0 = csub(rmul(mass, p0), rmul(0.5, h0));
    s1 = csub(rmul(mass, p1), rmul(0.5, h1));
}

// One site of D (DAG = 0) / D^dagger (DAG = 1): mass*psi - 0.5*bracket.
template <int DAG>
__device__ __forceinline__ void dirac_site(double mass, double sr0, double sl0, double2 p0,
                                           double2 p1, double2 pt0, double2 pt1, double2 px0,
                                           double2 px1, double2 pm0, double2 pm1, double2 pxm0,
                                           double2 pxm1, double2 Ut, double2 Ux, double2 Utm,
                                           double2 Uxm, double2 &s0, double2 &s1) {
    double2 h0, h1;
    dirac_bracket<DAG>(sr0, sl0, pt0, pt1, px0, px1, pm0, pm1, pxm0, pxm1, Ut, Ux, Utm, Uxm, h0, h1);
    s0 = csub(rmul(mass, p0), rmul(0.5, h0));
    s1 = csub(rmul(mass, p1), rmul(0.5, h1));
}

// Complex products of the CG passes built with FOLD = 2 (sm_cgra.hip,
// sm_eotd.hip): fused multiply-adds, one rounding per component instead of
// two or three; FOLD <= 1 keeps GCC's separately rounded expansion.
// cm = a b, cfma = c + a b, cfms = c - a b, nacc = acc + |z|^2.
template <int FOLD>
__device__ __forceinline__ double2 cm(double2 a, double2 b) {
    if (FOLD < 2) return cmul(a, b);
    return make_double2(__builtin_fma(a.x, b.x, -(a.y * b.y)), __builtin_fma(a.x, b.y, a.y * b.x));
}
template <int FOLD>
__device__ __forceinline__ double2 cfma(double2 c, double2 a, double2 b) {
    if (FOLD < 2) return cadd(c, cmul(a, b));
    return make_double2(__builtin_fma(a.x, b.x, __builtin_fma(-a.y, b.y, c.x)),
                        __builtin_fma(a.x, b.y, __builtin_fma(a.y, b.x, c.y)));
}
template <int FOLD>
__device__ __forceinline__ double2 cfms(double2 c, double2 a, double2 b) {
    if (FOLD < 2) return csub(c, cmul(a, b));
    return make_double2(__builtin_fma(-a.x, b.x, __builtin_fma(a.y, b.y, c.x)),
                        __builtin_fma(-a.x, b.y, __builtin_fma(-a.y, b.x, c.y)));
}
// |z|^2 accumulated: acc + Re(z conj z)
template <int FOLD>
__device__ __forceinline__ double nacc(double acc, double2 z) {
    if (FOLD < 2) return acc + cmul(z, cconj(z)).x;
    return __builtin_fma(z.x, z.x, __builtin_fma(z.y, z.y, acc));
}

// Deterministic block sum: wave butterfly, then lane-0 sums waves in order.
__device__ __forceinline__ double2 block_sum(double2 v, double2 *sh) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        v.x += __shfl_xor(v.x, off);
        v.y += __shfl_xor(v.y, off);
    }
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    if (lane == 0) sh[wid] = v;
    __syncthreads();
    double2 r = make_double2(0.0, 0.0);
    if (threadIdx.x == 0) {
        const int nw = (blockDim.x + 63) >> 6;
        for (int w = 0; w < nw; ++w) r = cadd(r, sh[w]);
    }
    return r;
}

// ---- one-pass CG scalars (sm_cgfused.hip, sm_cgra.hip) ----------------------
// From the three global sums: stop test on the direct |r_j|^2 (j >= 1), then
// alpha_j and beta_j (src/conjugate_gradient.cpp:33, 43-61).
__device__ __forceinline__ CGRed cg1_eval(CGRed s, double tol, double phi_norm, int max_iter, int first, double2 dA,
                                          double2 rA, double2 nn) {
    const double rr = nn.x, AA = nn.y;
    if (!first) {
        s.err = sqrt(rr);
        s.k += 1;
        if (s.err < tol * phi_norm) {
            s.done = 1;
            s.converged = 1;
            return s;
        }
        if (s.k >= max_iter) {
            s.done = 1;
            return s;
        }
    }
    s.rn = make_double2(rr, 0.0);
    const double2 al = cdiv(rr, 0.0, dA.x, dA.y);   // r_norm2 / dot(d, Ad)
    s.alpha2 = s.alpha;                             // two-direction CG keeps one pass of history
    s.beta2 = s.beta;
    s.alpha = al;
    const double est = rr - 2.0 * (al.x * rA.x + al.y * rA.y) + (al.x * al.x + al.y * al.y) * AA;
    s.beta = cdiv(est, 0.0, rr, 0.0);               // err^2 / r_norm2
    return s;
}

__device__ __forceinline__ void store_state(CGScalars *sc, const CGRed &s) {
    sc->rn = s.rn;
    sc->alpha = s.alpha;
    sc->beta = s.beta;
    sc->alpha2 = s.alpha2;
    sc->beta2 = s.beta2;
    sc->err = s.err;
    sc->k = s.k;
    sc->done = s.done;
    sc->converged = s.converged;
}

// One scalar step on the state in sc (the scalar kernel's, or the ticketed
// tail's last block, sm_cgra.hip).
__device__ __forceinline__ void cg1_update(CGScalars *sc, int first, double2 dA, double2 rA, double2 nn) {
    CGRed s;
    s.rn = sc->rn;
    s.alpha = sc->alpha;
    s.beta = sc->beta;
    s.alpha2 = sc->alpha2;
    s.beta2 = sc->beta2;
    s.err = sc->err;
    s.k = sc->k;
    s.done = sc->done;
    s.converged = sc->converged;
    s.pad = 0;
    store_state(sc, cg1_eval(s, sc->tol, sc->phi_norm, sc->max_iter, first, dA, rA, nn));
}

// Redundant scalars: S_{j-1} from S_{j-2} (red[j & 1]) and pass j-1's partials,
// evaluated by every block (all threads: block sums in a fixed order); block 0
// stores it to red[(j-1) & 1]. Returns S_{j-1} (valid in thread 0).
__device__ __forceinline__ CGRed cg1_redundant(CGScalars *sc, const double2 *prev, int nparts, long j, double2 *sh) {
    CGRed s = sc->red[j & 1];
    if (!s.done) {
        double2 acc[3] = {make_double2(0.0, 0.0), make_double2(0.0, 0.0), make_double2(0.0, 0.0)};
        for (int i = threadIdx.x; i < nparts; i += blockDim.x) {
            acc[0] = cadd(acc[0], prev[3 * i]);
            acc[1] = cadd(acc[1], prev[3 * i + 1]);
            acc[2] = cadd(acc[2], prev[3 * i + 2]);
        }
        double2 t[3];
#pragma unroll
        for (int q = 0; q < 3; ++q) {
            t[q] = block_sum(acc[q], sh);
            __syncthreads();
        }
        s = cg1_eval(s, sc->tol, sc->phi_norm, sc->max_iter, j - 1 == 0, t[0], t[1], t[2]);
    }
    if (threadIdx.x == 0 && blockIdx.x == 0) sc->red[(j - 1) & 1] = s;
    return s;
}

// t-shards (sm_cgra.hip RED = 2, sm_eotd.hip red): pass j-1's scalars from its all-reduced sums
// (sumr[(j-1) & 1]) and the state two passes back (red[j & 1]); block 0 keeps
// the new state. One thread per block calls it; noinline keeps the division
// chain's registers out of the march's allocation (inlined, the x-updating
// t-shard kernels reached 256 VGPRs and one wave per SIMD).
//
// Invariant after the stop: the host keeps issuing passes (chunks overshoot)
// and each one all-reduces sumr[j & 1] in place, although no block wrote that
// slot, so the slot becomes nshard times a stale sum. That is harmless ONLY
// because it is never read: pass J+1 (the first after the stopping
// evaluation of pass J) finds red[(J+1) & 1] without done, evaluates the
// stop from sumr[J & 1] (still valid: written by pass J, reduced once) and
// block 0 stores the stopped state into red[J & 1]; pass J+2 then finds
// red[J & 1] done and returns, and from there both red slots carry done, so
// `if (!s.done)` skips every sumr read. Any change that lets a pass read sumr
// before both red slots are done must stop the overshoot all-reduces first.
static __device__ __attribute__((noinline)) void ra_scalars_from_sums(CGScalars *sc, long j, double2 *ab, int *stop) {
    CGRed s = sc->red[j & 1];
    const double2 *sums = sc->sumr[(j - 1) & 1];
    if (!s.done) s = cg1_eval(s, sc->tol, sc->phi_norm, sc->max_iter, j - 1 == 0, sums[0], sums[1], sums[2]);
    if (blockIdx.x == 0) sc->red[(j - 1) & 1] = s;
    ab[0] = s.alpha;
    ab[1] = s.beta;
    ab[2] = s.alpha2;
    ab[3] = s.beta2;
    *stop = s.done;
}

// A block-uniform double2 (e.g. read back from LDS) into scalar registers.
__device__ __forceinline__ double2 uniform_d2(double2 v) {
    return make_double2(__hiloint2double(__builtin_amdgcn_readfirstlane(__double2hiint(v.x)),
                                         __builtin_amdgcn_readfirstlane(__double2loint(v.x))),
                        __hiloint2double(__builtin_amdgcn_readfirstlane(__double2hiint(v.y)),
                                         __builtin_amdgcn_readfirstlane(__double2loint(v.y))));
}

// Wave-wide lane shifts by one (DPP wave_shr:1 / wave_shl:1, GFX9-family
// incl. gfx950): no LDS, no barrier. Lane 0 (shr) / lane 63 (shl) receive 0.
__device__ __forceinline__ double dpp_shr1(double v) {  // lane l <- lane l-1
    const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), 0x138, 0xf, 0xf, true);
    const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), 0x138, 0xf, 0xf, true);
    return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double dpp_shl1(double v) {  // lane l <- lane l+1
    const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), 0x130, 0xf, 0xf, true);
    const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), 0x130, 0xf, 0xf, true);
    return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double2 dpp_shr1(double2 v) { return make_double2(dpp_shr1(v.x), dpp_shr1(v.y)); }
__device__ __forceinline__ double2 dpp_shl1(double2 v) { return make_double2(dpp_shl1(v.x), dpp_shl1(v.y)); }

struct Sp {   // a 2-spinor at one site
    double2 a, b;
};
__device__ __forceinline__ Sp shr(Sp v) { return Sp{dpp_shr1(v.a), dpp_shr1(v.b)}; }
__device__ __forceinline__ Sp shl(Sp v) { return Sp{dpp_shl1(v.a), dpp_shl1(v.b)}; }

// Non-temporal (streaming) 16-B loads/stores: data touched once per pass.
// Measured on MI355X (tools/membench.hip): block-contiguous chunks with nt
// loads+stores reach 5.7 TB/s on the 2-read/1-write BLAS-1 pattern against
// 4.4-5.1 TB/s for plain grid-stride loops.
typedef double sm_v2d __attribute__((ext_vector_type(2)));
__device__ __forceinline__ double2 ld_nt(const double2 *p) {
    const sm_v2d v = __builtin_nontemporal_load(reinterpret_cast<const sm_v2d *>(p));
    return make_double2(v.x, v.y);
}
__device__ __forceinline__ void st_nt(double2 *p, double2 v) {
    const sm_v2d w = {v.x, v.y};
    __builtin_nontemporal_store(w, reinterpret_cast<sm_v2d *>(p));
}

// Block-contiguous chunk of [0, n) for streaming kernels: block b owns
// [b*per, min(n, (b+1)*per)), lanes stride 256 inside it, 4 tiles per step.
struct Chunk {
    long beg, end;
};
__device__ __forceinline__ Chunk block_chunk(long n) {
    const long per = (n + gridDim.x - 1) / gridDim.x;
    Chunk c;
    c.beg = (long)blockIdx.x * per;
    c.end = c.beg + per < n ? c.beg + per : n;
    return c;
}

// Fixed-order sum of per-block partials by one block (deterministic).
__device__ __forceinline__ double2 sum_partials_block(int nparts, const double2 *part, double2 *sh) {
    double2 acc = make_double2(0.0, 0.0);
    for (int i = threadIdx.x; i < nparts; i += blockDim.x) acc = cadd(acc, part[i]);
    return block_sum(acc, sh);
}

// alpha = r_norm2 / <d, Ad>   (complex division, src/conjugate_gradient.cpp:33)
__device__ __forceinline__ void cg_alpha_scalar(CGScalars *sc, double2 dAd) {
    sc->alpha = cdiv(sc->rn.x, sc->rn.y, dAd.x, dAd.y);
}

// err = sqrt(Re<r,r>); stop test; beta = err^2 / r_norm2   (src/conjugate_gradient.cpp:43-61)
__device__ __forceinline__ void cg_beta_scalar(CGScalars *sc, double2 rr) {
    const double err_sqr = rr.x;
    const double err = sqrt(err_sqr);
    sc->err = err;
    sc->k = sc->k + 1;
    if (err < sc->tol * sc->phi_norm) {
        sc->done = 1;
        sc->converged = 1;
        return;
    }
    sc->beta = cdiv(err_sqr, 0.0, sc->rn.x, sc->rn.y);
    sc->rn = make_double2(err_sqr, 0.0);
}

// Ticketed tail (sm_cgra.hip, TK): blocks publish their partials with
// write-through (agent-scope atomic) stores -- no release fence, which would
// write back the XCD's whole dirty L2 in every block -- wait for them, then
// take a relaxed agent-scope ticket; the block drawing the last ticket of a
// group issues an agent-scope acquire, reads the group's partials with
// agent-scope atomic loads and re-arms the counter (zeroed at context
// creation).
//
// Memory-model note (gfx9 / gfx950 assumption): the publishing side has no
// release operation. Its ordering comes from the hardware: agent-scope atomic
// stores are written through to the (coherent, memory-side) fabric, the
// vector memory counter counts stores, so `s_waitcnt vmcnt(0)` before the
// barrier means every publishing wave's stores have completed before its
// block's ticket is taken. The winning block's acquire fence (an L1
// invalidate, no L2 writeback) and its atomic loads then see them from any
// XCD. Under the portable HIP/C++ model this is a relaxed publication; a
// target without write-through atomic stores or with a different vmcnt
// meaning needs a release fetch_add instead.
__device__ __forceinline__ void publish_partial(double2 *slot, double2 v) {
    __hip_atomic_store(&slot->x, v.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&slot->y, v.y, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double2 load_published(const double2 *slot) {
    return make_double2(__hip_atomic_load(&slot->x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                        __hip_atomic_load(&slot->y, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
// Every thread of the block calls it; true in the block that arrived last.
__device__ __forceinline__ bool last_block_arrive(unsigned *counter, unsigned nblocks, int *sh_flag) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every wave: its write-through stores are done
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned t = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int last = t == nblocks - 1;
        if (last) __hip_atomic_store(counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        *sh_flag = last;
    }
    __syncthreads();
    const bool last = *sh_flag != 0;
    if (last) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // block-uniform: the winner only
    return last;
}
// One spin-projected face value (TFaces::proj; launch_pack_faces_proj and the
// peer transport's pack): side 0 = the t = 0 column's forward-hop combination
// (sent down), side 1 = conj(U_t(t = Wt-1)) times the backward combination
// (sent up). The reference's own sums and product (src/dirac_operator.cpp:31-43,
// 255-267; force :493-506).
__device__ __forceinline__ double2 proj_face_value(int kind, int side, double2 p0, double2 p1, const double2 *Ut) {
    if (!side) return (kind == FACE_DDAG || kind == FACE_FORCE_L) ? cadd(p0, p1) : csub(p0, p1);
    switch (kind) {
        case FACE_D: return cmul(cconj(*Ut), cadd(p0, p1));
        case FACE_DDAG: return cmul(cconj(*Ut), csub(p0, p1));
        default: return make_double2(0.0, 0.0);  // the force reads only t+1 neighbours: the lo face sent down
    }
}

// Fixed-order wave sum (butterfly; every lane gets the same bits).
__device__ __forceinline__ double2 wave_sum(double2 v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        v.x += __shfl_xor(v.x, off);
        v.y += __shfl_xor(v.y, off);
    }
    return v;
}

// The ticketed tail of a CG pass (sm_cgra.hip, sm_eotd.hip): this block's
// partials (s0, s1, s2 in thread 0) go to slot `tile` of ntiles; the last
// block of each group of 64 tiles sums the group (one wave, one tile per
// lane, fixed butterfly order), the last group's block sums the group sums in
// order and forms the scalars in sc (out3 == null) or writes the three sums
// to out3 (a t-shard's, for the all-reduce). Every thread of the block calls it.
// peer != null (t-shards over the peer transport, sm_peer.h): the last block
// all-reduces the three sums over every shard (collective number pseq) before
// writing them to out3.
__device__ __forceinline__ void cg_ticketed_tail(double2 *partials, long tile, int ntiles, unsigned *tick,
                                                 double2 *gsum, double2 *out3, CGScalars *sc, int first, double2 s0,
                                                 double2 s1, double2 s2, const PeerView *peer = nullptr,
                                                 unsigned long long pseq = 0) {
    double2 *p = partials + 3 * tile;
    if (threadIdx.x == 0) {
        publish_partial(p, s0);
        publish_partial(p + 1, s1);
        publish_partial(p + 2, s2);
    }
    __shared__ int s_last;
    const int lane = threadIdx.x & 63;
    const int grp = (int)(tile >> 6);
    const int gsz = min(64, ntiles - (grp << 6));
    if (!last_block_arrive(tick + 1 + grp, (unsigned)gsz, &s_last)) return;
    const double2 zz = make_double2(0.0, 0.0);
    if (threadIdx.x < 64) {
        double2 v0 = zz, v1 = zz, v2 = zz;
        if (lane < gsz) {
            const double2 *q = partials + 3 * (((long)grp << 6) + lane);
            v0 = load_published(q);
            v1 = load_published(q + 1);
            v2 = load_published(q + 2);
        }
        v0 = wave_sum(v0);
        v1 = wave_sum(v1);
        v2 = wave_sum(v2);
        if (lane == 0) {
            publish_partial(gsum + 3 * grp, v0);
            publish_partial(gsum + 3 * grp + 1, v1);
            publish_partial(gsum + 3 * grp + 2, v2);
        }
    }
    const int ngrp = (ntiles + 63) >> 6;
    if (!last_block_arrive(tick, (unsigned)ngrp, &s_last)) return;
    if (threadIdx.x < 64) {
        double2 v0 = zz, v1 = zz, v2 = zz;
        for (int i = lane; i < ngrp; i += 64) {
            v0 = cadd(v0, load_published(gsum + 3 * i));
            v1 = cadd(v1, load_published(gsum + 3 * i + 1));
            v2 = cadd(v2, load_published(gsum + 3 * i + 2));
        }
        v0 = wave_sum(v0);
        v1 = wave_sum(v1);
        v2 = wave_sum(v2);
        if (lane == 0) {
            if (out3) {
                if (peer) {
                    double val[6] = {v0.x, v0.y, v1.x, v1.y, v2.x, v2.y};
                    peer_allreduce_thread(*peer, pseq, val, 6);
                    v0 = make_double2(val[0], val[1]);
                    v1 = make_double2(val[2], val[3]);
                    v2 = make_double2(val[4], val[5]);
                }
                out3[0] = v0;
                out3[1] = v1;
                out3[2] = v2;
            } else {
                cg1_update(sc, first, v0, v1, v2);
            }
        }
    }
}

}  // namespace sm

