// sm_eo.hip -- checkerboard (even-odd) kernels for the even-odd preconditioned
// HMC action, gfx950.
//
// Sites split by parity p = (x + t) & 1 (t0 is even, so local and global
// parity agree). A checkerboard field of parity p stores its Vh = Nx*Wt/2
// sites as two planes of complex<double>, half-site index h = x*Wh + k with
// t = 2k + ((p + x) & 1), Wh = Wt/2. In that layout the t-neighbours of a
// parity-p site are the opposite-parity entries k + s and k + s - 1
// (s = (p + x) & 1) of the same row, and the x-neighbours are entry k of the
// rows x +- 1: every access of a hop is unit-stride in k.
//
// D = m - 0.5 H with H the hopping bracket (dirac_bracket): H connects only
// opposite parities, so D = [[m, D_eo], [D_oe, m]] and the Schur complement is
//     Dhat = m - (1/m) D_eo D_oe = m + (0.5/m) H_eo (D_oe)  ... see sm_eo.cpp.
// eo_hop computes  out_p = a * aux_p + b * H_{p,q} in_q  for one parity, with
// the reference's bracket arithmetic (a = 0, b = -0.5 reproduces D on an
// input that vanishes on parity p bit for bit).
//
// t-sharded (SH = 1): a checkerboard field's t-faces are its k = 0, 1 columns
// (sent down) and k = Wh-2, Wh-1 columns (sent up), both parities of the
// global checkerboard agreeing with the local one because t0 is even. The
// received faces of one field are laid out [side][plane][col][x] (side 0: the
// down-neighbour's k = Wh-2+col, i.e. my k = col-2; side 1: the
// up-neighbour's k = col, i.e. my k = Wh+col), 8*Nx complex.
#include "sm_device.h"
#include "sm_internal.h"

#pragma clang fp contract(off)

namespace sm {

struct EoGeom {
    int Nx, Wt, Wh, t0, Ntg;
    long V, Vh;
};

// full <-> checkerboard (both parities; either cb pointer may be null)
__global__ void __launch_bounds__(256) to_cb_kernel(EoGeom g, const double2 *full, double2 *e, double2 *o) {
    for (long n = (long)blockIdx.x * blockDim.x + threadIdx.x; n < g.V; n += (long)gridDim.x * blockDim.x) {
        const int x = (int)(n / g.Wt), t = (int)(n - (long)x * g.Wt);
        const long h = (long)x * g.Wh + (t >> 1);
        double2 *dst = ((x + t) & 1) ? o : e;
        if (!dst) continue;
        dst[h] = full[n];
        dst[h + g.Vh] = full[n + g.V];
    }
}

__device__ __forceinline__ long cb_face_at(int Nx, int side, int plane, int col, int x) {
    return (long)((side * 2 + plane) * 2 + col) * Nx + x;
}

// pack the t-faces of a checkerboard field into [side][plane][col][x]
__global__ void __launch_bounds__(256) pack_cb_faces_kernel(EoGeom g, const double2 *f, double2 *out) {
    const int n = 8 * g.Nx;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const int x = i % g.Nx, r = i / g.Nx;
        const int col = r & 1, plane = (r >> 1) & 1, side = r >> 2;
        const int k = side ? g.Wh - 2 + col : col;
        out[i] = f[plane * g.Vh + (long)x * g.Wh + k];
    }
}

__global__ void __launch_bounds__(256) from_cb_kernel(EoGeom g, const double2 *e, const double2 *o, double2 *full) {
    for (long n = (long)blockIdx.x * blockDim.x + threadIdx.x; n < g.V; n += (long)gridDim.x * blockDim.x) {
        const int x = (int)(n / g.Wt), t = (int)(n - (long)x * g.Wt);
        const long h = (long)x * g.Wh + (t >> 1);
        const double2 *src = ((x + t) & 1) ? o : e;
        full[n] = src ? src[h] : make_double2(0.0, 0.0);
        full[n + g.V] = src ? src[h + g.Vh] : make_double2(0.0, 0.0);
    }
}

// out_p = a*aux_p + b*H in_q for the sites of parity p (one shard: periodic
// x, periodic t with the antiperiodic sign on the global t boundary).
// Up: U of parity p (plane 0 U_t, plane 1 U_x); Uq: U of parity q = 1-p.
// SH = 1: t-neighbours beyond the shard come from the received faces of `in`
// (inf) and of Uq (uqf).
template <int DAG, int SH>
__global__ void __launch_bounds__(256) eo_hop_kernel(EoGeom g, int p, const double2 *in, const double2 *Up,
                                                     const double2 *Uq, const double2 *aux, double a, double b,
                                                     double2 *out, const double2 *inf, const double2 *uqf) {
    const long Vh = g.Vh;
    for (long h = (long)blockIdx.x * blockDim.x + threadIdx.x; h < Vh; h += (long)gridDim.x * blockDim.x) {
        const int x = (int)(h / g.Wh), k = (int)(h - (long)x * g.Wh);
        const int s = (p + x) & 1;
        const int t = 2 * k + s;
        int kp = k + s, km = k + s - 1;            // t+1, t-1 in the opposite parity's row
        const int xp = x + 1 == g.Nx ? 0 : x + 1, xm = x == 0 ? g.Nx - 1 : x - 1;
        const long row = (long)x * g.Wh;
        const long ixp = (long)xp * g.Wh + k, ixm = (long)xm * g.Wh + k;
        double2 pt0, pt1, pm0, pm1, um;
        if (SH && kp == g.Wh) {                    // up-neighbour's k = 0
            pt0 = inf[cb_face_at(g.Nx, 1, 0, 0, x)];
            pt1 = inf[cb_face_at(g.Nx, 1, 1, 0, x)];
        } else {
            if (kp == g.Wh) kp = 0;
            pt0 = in[row + kp];
            pt1 = in[row + kp + Vh];
        }
        if (SH && km < 0) {                        // down-neighbour's k = Wh-1
            pm0 = inf[cb_face_at(g.Nx, 0, 0, 1, x)];
            pm1 = inf[cb_face_at(g.Nx, 0, 1, 1, x)];
            um = uqf[cb_face_at(g.Nx, 0, 0, 1, x)];
        } else {
            if (km < 0) km = g.Wh - 1;
            pm0 = in[row + km];
            pm1 = in[row + km + Vh];
            um = Uq[row + km];
        }
        const int tg = g.t0 + t;
        const double sr0 = tg == g.Ntg - 1 ? -1.0 : 1.0;
        const double sl0 = tg == 0 ? -1.0 : 1.0;
        double2 h0, h1;
        dirac_bracket<DAG>(sr0, sl0, pt0, pt1, in[ixp], in[ixp + Vh], pm0, pm1, in[ixm], in[ixm + Vh], Up[h],
                           Up[h + Vh], um, Uq[ixm + Vh], h0, h1);
        double2 o0 = rmul(b, h0), o1 = rmul(b, h1);
        if (aux) {
            o0 = cadd(rmul(a, aux[h]), o0);
            o1 = cadd(rmul(a, aux[h + Vh]), o1);
        }
        out[h] = o0;
        out[h + Vh] = o1;
    }
}

// ---- fused Dhat: both hops in one marching pass ------------------------------
// out_e = m v + (0.5/m) H_eo T,  T = -0.5 H_oe v  (Dhat v; DAG = 1: Dhat^dag v
// with the D^dag bracket), the odd intermediate T kept in registers. Same
// structure as the fused CG pass: a wave owns 60 k-columns (lanes k-2 .. k+61,
// two halo lanes per side), marches x, t-neighbours by DPP. In the
// checkerboard the t-neighbours of a site are lanes (l-1, l) or (l, l+1)
// depending on the row's parity (row-uniform), the x-neighbours are lane l of
// the rows x +- 1. Per-element arithmetic = two eo_hop launches (bitwise).
// EPI_DOT: per-block partials of sum aux * conj(out) (the CG's <d, Ad>).
constexpr int EW = 60;

struct EoFArgs {
    const double2 *v, *Ue, *Uo;
    const double2 *vf, *uef, *uof;   // received t-faces (SH = 1)
    // folded CG (MODE 1 / 2, see eo_dhat_fused_kernel)
    const double2 *rold, *aold, *rf, *af;
    double2 *dnew, *rnew, *x;
    const double2 *aux2;
    CGScalars *sc;
    int first;
    double2 *out;
    const double2 *aux;
    double2 *partials;
    EoGeom g;
    int xchunk, NWT, TBk, XB;
    double mass;
};

struct ERow {                // one lane, one row: even input, even / odd links at (y, k)
    double2 v0, v1, et, ex, ot, ox;
};


//
// MODE 1 / 2: the two passes of the folded even-odd CG iteration j (the
// one-pass recurrence of cg_onepass_kernel on half-lattice vectors):
//   MODE 1 (DAG = 1): every loaded element forms r_j = r_{j-1} - alpha Ad_{j-1}
//     and d_j = d_{j-1} beta + r_j (v = d_{j-1}, rold, aold; first: d_j = r_j =
//     r_0); owned sites store r_j, d_j and x += alpha d_{j-1} and sum |r_j|^2;
//     out = Dhat^dag d_j. Partial: p[3b+2].x = |r_j|^2.
//   MODE 2 (DAG = 0, EPI_DOT): out = Ad_j = Dhat W; partials p[3b] = <d_j,Ad_j>
//     (aux = d_j), p[3b+1] = <r_j,Ad_j> (aux2 = r_j), p[3b+2].y = |Ad_j|^2.
// alpha, beta: sc (cg1_scalars after the previous pass B).
template <int DAG, int EPI, int SH, int MODE>
__global__ void __launch_bounds__(256) eo_dhat_fused_kernel(EoFArgs a) {
    __shared__ double2 sh[4];
    if (MODE != 0 && a.sc->done) return;                   // grid-uniform
    const int tb = blockIdx.x % a.TBk, xc = blockIdx.x / a.TBk;
    const int lane = threadIdx.x & 63;
    const int gw = tb * 4 + (threadIdx.x >> 6);
    const int x0 = xc * a.xchunk, xe = min(a.g.Nx, x0 + a.xchunk);
    double2 acc = make_double2(0.0, 0.0), acc_rA = make_double2(0.0, 0.0);
    double acc_nn = 0.0;                                   // MODE 1: |r|^2, MODE 2: |Ad|^2
    double2 alpha = make_double2(0.0, 0.0), beta = make_double2(0.0, 0.0);
    if (MODE == 1) {
        alpha = a.sc->alpha;
        beta = a.sc->beta;
    }
    if (gw < a.NWT && x0 < xe) {
        const int Wh = a.g.Wh, Nx = a.g.Nx;
        const long Vh = a.g.Vh;
        const int k = gw * EW - 2 + lane;
        int kw = k % Wh;
        if (kw < 0) kw += Wh;                                  // periodic in t (one shard)
        const bool own = lane >= 2 && lane < EW + 2 && k < Wh;
        // sharded: lanes outside the shard read the received faces
        const bool inside = k >= 0 && k < Wh;
        const int side = k < 0 ? 0 : 1;
        const int col = k < 0 ? k + 2 : min(k - Wh, 1);
        const double m = a.mass, hm = 0.5 / a.mass;
        auto wrapx = [Nx](int x) { int w = x % Nx; return w < 0 ? w + Nx : w; };
        auto load = [&](int y, ERow &R) {
            double2 r0, r1, A0, A1;
            if (!SH || inside) {
                const long h = (long)wrapx(y) * Wh + kw;
                R.v0 = a.v[h];
                R.v1 = a.v[h + Vh];
                if (MODE == 1) {
                    r0 = a.rold[h];
                    r1 = a.rold[h + Vh];
                    A0 = a.aold[h];
                    A1 = a.aold[h + Vh];
                }
                R.et = a.Ue[h];
                R.ex = a.Ue[h + Vh];
                R.ot = a.Uo[h];
                R.ox = a.Uo[h + Vh];
            } else {
                const long f0 = cb_face_at(Nx, side, 0, col, wrapx(y)), f1 = f0 + 2 * Nx;
                R.v0 = a.vf[f0];
                R.v1 = a.vf[f1];
                if (MODE == 1) {
                    r0 = a.rf[f0];
                    r1 = a.rf[f1];
                    A0 = a.af[f0];
                    A1 = a.af[f1];
                }
                R.et = a.uef[f0];
                R.ex = a.uef[f1];
                R.ot = a.uof[f0];
                R.ox = a.uof[f1];
            }
            if (MODE == 1) {
                // the reference's per-element updates (src/conjugate_gradient.cpp:36-39, 55-58)
                const double2 rj0 = a.first ? r0 : csub(r0, cmul(alpha, A0));
                const double2 rj1 = a.first ? r1 : csub(r1, cmul(alpha, A1));
                const double2 dj0 = a.first ? r0 : cadd(cmul(R.v0, beta), rj0);
                const double2 dj1 = a.first ? r1 : cadd(cmul(R.v1, beta), rj1);
                if (own && y >= x0 && y < xe) {
                    const long h = (long)y * Wh + kw;
                    st_nt(a.rnew + h, rj0);
                    st_nt(a.rnew + h + Vh, rj1);
                    st_nt(a.dnew + h, dj0);
                    st_nt(a.dnew + h + Vh, dj1);
                    if (!a.first) {
                        st_nt(a.x + h, cadd(a.x[h], cmul(alpha, R.v0)));
                        st_nt(a.x + h + Vh, cadd(a.x[h + Vh], cmul(alpha, R.v1)));
                    }
                    acc_nn += cmul(rj0, cconj(rj0)).x;  // Re dot(r, r)
                    acc_nn += cmul(rj1, cconj(rj1)).x;
                }
                R.v0 = dj0;
                R.v1 = dj1;
            }
        };
        // t: local, unwrapped (halo lanes of shard 0 / the last shard wrap
        // to the other end of the global lattice)
        auto signs = [&](int t, double &sr0, double &sl0) {
            int tg = a.g.t0 + t;
            if (tg < 0) tg += a.g.Ntg;
            else if (tg >= a.g.Ntg) tg -= a.g.Ntg;
            sr0 = tg == a.g.Ntg - 1 ? -1.0 : 1.0;
            sl0 = tg == 0 ? -1.0 : 1.0;
        };
        // T at odd site (y, k): neighbours v(y, k-1+s_o), v(y, k+s_o), v(y+-1, k); s_o = 1 - (y&1)
        auto todd = [&](int y, const Sp &vc, const Sp &vxm, const Sp &vxp, const ERow &Rc, double2 ex_m) {
            const bool ye = (wrapx(y) & 1) == 0;
            Sp pm, pp;
            double2 utm;
            if (ye) {
                pm = vc;
                pp = shl(vc);
                utm = Rc.et;
            } else {
                pm = shr(vc);
                pp = vc;
                utm = dpp_shr1(Rc.et);
            }
            double sr0, sl0;
            signs(2 * k + (ye ? 1 : 0), sr0, sl0);
            double2 h0, h1;
            dirac_bracket<DAG>(sr0, sl0, pp.a, pp.b, vxp.a, vxp.b, pm.a, pm.b, vxm.a, vxm.b, Rc.ot, Rc.ox, utm, ex_m,
                               h0, h1);
            return Sp{rmul(-0.5, h0), rmul(-0.5, h1)};
        };
        // out at even site (x, k): T(x, k-1+s_e), T(x, k+s_e), T(x+-1, k); s_e = x&1
        auto eout = [&](int x, const Sp &Tc, const Sp &Txm, const Sp &Txp, const ERow &Rc, double2 ox_m,
                        const Sp &vc) {
            const bool xe_ = (wrapx(x) & 1) == 0;
            Sp pm, pp;
            double2 utm;
            if (xe_) {
                pm = shr(Tc);
                pp = Tc;
                utm = dpp_shr1(Rc.ot);
            } else {
                pm = Tc;
                pp = shl(Tc);
                utm = Rc.ot;
            }
            double sr0, sl0;
            signs(2 * k + (xe_ ? 0 : 1), sr0, sl0);
            double2 h0, h1;
            dirac_bracket<DAG>(sr0, sl0, pp.a, pp.b, Txp.a, Txp.b, pm.a, pm.b, Txm.a, Txm.b, Rc.et, Rc.ex, utm, ox_m,
                               h0, h1);
            return Sp{cadd(rmul(m, vc.a), rmul(hm, h0)), cadd(rmul(m, vc.b), rmul(hm, h1))};
        };
        ERow R, Rm1, Rc, Rn;
        load(x0 - 2, R);
        const Sp vm2{R.v0, R.v1};
        const double2 exm2 = R.ex;
        load(x0 - 1, Rm1);
        Sp vm1{Rm1.v0, Rm1.v1};
        load(x0, Rc);
        Sp vc{Rc.v0, Rc.v1};
        load(x0 + 1, Rn);
        Sp vn{Rn.v0, Rn.v1};
        load(x0 + 2, R);
        Sp Tp = todd(x0 - 1, vm1, vm2, vc, Rm1, exm2);
        Sp Tc = todd(x0, vc, vm1, vn, Rc, Rm1.ex);
        double2 oxp = Rm1.ox;                                  // U_x(x-1) odd link
        for (int x = x0; x < xe; ++x) {
            const ERow R2 = R;                                 // row x+2
            load(min(x + 3, xe + 1), R);
            __builtin_amdgcn_sched_barrier(0);
            const Sp v2{R2.v0, R2.v1};
            const Sp Tn = todd(x + 1, vn, vc, v2, Rn, Rc.ex);
            const Sp o = eout(x, Tc, Tp, Tn, Rc, oxp, vc);
            if (own) {
                const long h = (long)x * Wh + kw;
                st_nt(a.out + h, o.a);
                st_nt(a.out + h + Vh, o.b);
                if (EPI == EPI_DOT) {
                    acc = cadd(acc, cmul(a.aux[h], cconj(o.a)));
                    acc = cadd(acc, cmul(a.aux[h + Vh], cconj(o.b)));
                }
                if (MODE == 2) {
                    acc_rA = cadd(acc_rA, cmul(a.aux2[h], cconj(o.a)));
                    acc_rA = cadd(acc_rA, cmul(a.aux2[h + Vh], cconj(o.b)));
                    acc_nn += cmul(o.a, cconj(o.a)).x;
                    acc_nn += cmul(o.b, cconj(o.b)).x;
                }
            }
            Tp = Tc;
            Tc = Tn;
            oxp = Rc.ox;
            vc = vn;
            vn = v2;
            Rc = Rn;
            Rn = R2;
        }
    }
    if (MODE == 1) {
        const double2 bs = block_sum(make_double2(acc_nn, 0.0), sh);
        if (threadIdx.x == 0) a.partials[3 * (long)blockIdx.x + 2].x = bs.x;
    } else if (MODE == 2) {
        const double2 s0 = block_sum(acc, sh);
        __syncthreads();
        const double2 s1 = block_sum(acc_rA, sh);
        __syncthreads();
        const double2 s2 = block_sum(make_double2(acc_nn, 0.0), sh);
        if (threadIdx.x == 0) {
            double2 *p = a.partials + 3 * (long)blockIdx.x;
            p[0] = s0;
            p[1] = s1;
            p[2].y = s2.x;
        }
    } else if (EPI == EPI_DOT) {
        const double2 bs = block_sum(acc, sh);
        if (threadIdx.x == 0) a.partials[blockIdx.x] = bs;
    }
}

namespace {
unsigned eo_grid(long n) {
    long nb = (n + 255) / 256;
    return (unsigned)(nb > 8192 ? 8192 : (nb < 1 ? 1 : nb));
}
EoGeom eo_geom(const Geometry &g) {
    EoGeom e;
    e.Nx = g.Nx;
    e.Wt = g.Wt;
    e.Wh = g.Wt / 2;
    e.t0 = g.t0;
    e.Ntg = g.Ntg;
    e.V = g.V;
    e.Vh = g.V / 2;
    return e;
}
}  // namespace

void launch_to_cb(hipStream_t s, const Geometry &g, const double2 *full, double2 *e, double2 *o) {
    hipLaunchKernelGGL(to_cb_kernel, dim3(eo_grid(g.V)), dim3(256), 0, s, eo_geom(g), full, e, o);
}

void launch_from_cb(hipStream_t s, const Geometry &g, const double2 *e, const double2 *o, double2 *full) {
    hipLaunchKernelGGL(from_cb_kernel, dim3(eo_grid(g.V)), dim3(256), 0, s, eo_geom(g), e, o, full);
}

EoFusedCfg eo_fused_config(const Geometry &g) {
    EoFusedCfg c;
    const int Wh = g.Wt / 2;
    c.NWT = (Wh + EW - 1) / EW;
    c.TBk = (c.NWT + 3) / 4;
    const int target = 4096;                              // blocks (as the fused CG pass)
    int nchunks = (target + c.TBk - 1) / c.TBk;
    if (nchunks > g.Nx / 2) nchunks = g.Nx / 2;
    if (nchunks < 1) nchunks = 1;
    int xchunk = (g.Nx + nchunks - 1) / nchunks;
    // but at least min(8, Nx/128) rows: short chunks re-read their 4 halo rows
    // too often (tools/tune_eo.py, one MI355X, ms per CG iteration, best
    // chunk: 512^2 4 rows 0.039 vs 0.043; 1024^2 8 rows 0.079 vs 0.096;
    // 2048^2 8 rows 0.243 vs 0.262; 4096^2 the 4096-block rule's 10 rows)
    int xmin = g.Nx / 128;
    xmin = xmin < 2 ? 2 : (xmin > 8 ? 8 : xmin);
    if (xchunk < xmin) xchunk = xmin;
    xchunk += xchunk & 1;                                 // even: every chunk starts on an even row
    c.xchunk = xchunk;
    c.XB = (g.Nx + c.xchunk - 1) / c.xchunk;
    return c;
}

int eo_fused_blocks(const EoFusedCfg &c) { return c.TBk * c.XB; }

void launch_pack_cb_faces(hipStream_t s, const Geometry &g, const double2 *f, double2 *out) {
    hipLaunchKernelGGL(pack_cb_faces_kernel, dim3((8 * g.Nx + 255) / 256), dim3(256), 0, s, eo_geom(g), f, out);
}

void launch_eo_dhat_fused(hipStream_t s, const Geometry &g, const EoFusedCfg &c, int dagger, const double2 *v,
                          const double2 *Ue, const double2 *Uo, double mass, double2 *out, const double2 *aux,
                          double2 *partials, const EoFaces &f) {
    EoFArgs a;
    a.v = v; a.Ue = Ue; a.Uo = Uo; a.out = out; a.aux = aux; a.partials = partials;
    a.vf = f.v; a.uef = f.ue; a.uof = f.uo;
    a.g = eo_geom(g);
    a.xchunk = c.xchunk; a.NWT = c.NWT; a.TBk = c.TBk; a.XB = c.XB;
    a.mass = mass;
    const dim3 grid(c.TBk * c.XB), block(256);
#define SM_EO_LAUNCH(D, E, H) hipLaunchKernelGGL((eo_dhat_fused_kernel<D, E, H, 0>), grid, block, 0, s, a)
    if (f.v) {
        if (dagger) {
            if (aux) SM_EO_LAUNCH(1, EPI_DOT, 1);
            else SM_EO_LAUNCH(1, EPI_NONE, 1);
        } else {
            if (aux) SM_EO_LAUNCH(0, EPI_DOT, 1);
            else SM_EO_LAUNCH(0, EPI_NONE, 1);
        }
    } else {
        if (dagger) {
            if (aux) SM_EO_LAUNCH(1, EPI_DOT, 0);
            else SM_EO_LAUNCH(1, EPI_NONE, 0);
        } else {
            if (aux) SM_EO_LAUNCH(0, EPI_DOT, 0);
            else SM_EO_LAUNCH(0, EPI_NONE, 0);
        }
    }
#undef SM_EO_LAUNCH
}

void launch_eo_cg_pass(hipStream_t s, const Geometry &g, const EoFusedCfg &c, int which, const EoCgPass &q,
                       const double2 *Ue, const double2 *Uo, double mass, const EoFaces &f, CGScalars *sc,
                       double2 *partials) {
    EoFArgs a = {};
    a.Ue = Ue; a.Uo = Uo; a.uef = f.ue; a.uof = f.uo;
    a.g = eo_geom(g);
    a.xchunk = c.xchunk; a.NWT = c.NWT; a.TBk = c.TBk; a.XB = c.XB;
    a.mass = mass;
    a.sc = sc;
    a.partials = partials;
    a.first = q.first;
    const dim3 grid(c.TBk * c.XB), block(256);
    if (which == 0) {  // pass A: d_j, r_j, x; W = Dhat^dag d_j
        a.v = q.dold; a.rold = q.rold; a.aold = q.ad;
        a.vf = f.v; a.rf = q.rf; a.af = q.af;
        a.dnew = q.dnew; a.rnew = q.rnew; a.x = q.x;
        a.out = q.W;
        if (f.v) hipLaunchKernelGGL((eo_dhat_fused_kernel<1, EPI_NONE, 1, 1>), grid, block, 0, s, a);
        else hipLaunchKernelGGL((eo_dhat_fused_kernel<1, EPI_NONE, 0, 1>), grid, block, 0, s, a);
    } else {           // pass B: Ad_j = Dhat W and the three dots
        a.v = q.W; a.vf = q.wf;
        a.aux = q.dnew; a.aux2 = q.rnew;
        a.out = q.ad;
        if (q.wf) hipLaunchKernelGGL((eo_dhat_fused_kernel<0, EPI_DOT, 1, 2>), grid, block, 0, s, a);
        else hipLaunchKernelGGL((eo_dhat_fused_kernel<0, EPI_DOT, 0, 2>), grid, block, 0, s, a);
    }
}

void launch_eo_hop(hipStream_t s, const Geometry &g, int dagger, int p, const double2 *in, const double2 *Up,
                   const double2 *Uq, const double2 *aux, double a, double b, double2 *out, const double2 *inf,
                   const double2 *uqf) {
    const EoGeom e = eo_geom(g);
    const dim3 grid(eo_grid(e.Vh)), block(256);
#define SM_EO_HOP(D, H) \
    hipLaunchKernelGGL((eo_hop_kernel<D, H>), grid, block, 0, s, e, p, in, Up, Uq, aux, a, b, out, inf, uqf)
    if (inf) {
        if (dagger) SM_EO_HOP(1, 1);
        else SM_EO_HOP(0, 1);
    } else {
        if (dagger) SM_EO_HOP(1, 0);
        else SM_EO_HOP(0, 0);
    }
#undef SM_EO_HOP
}

}  // namespace sm
