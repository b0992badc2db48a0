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
template <int DAG>
__global__ void __launch_bounds__(256) eo_hop_kernel(EoGeom g, int p, const double2 *in, const double2 *Up,
                                                     const double2 *Uq, const double2 *aux, double a, double b,
                                                     double2 *out) {
    const long Vh = g.Vh;
    for (long h = (long)blockIdx.x * blockDim.x + threadIdx.x; h < Vh; h += (long)gridDim.x * blockDim.x) {
        const int x = (int)(h / g.Wh), k = (int)(h - (long)x * g.Wh);
        const int s = (p + x) & 1;
        const int t = 2 * k + s;
        int kp = k + s, km = k + s - 1;            // t+1, t-1 in the opposite parity's row
        if (kp == g.Wh) kp = 0;
        if (km < 0) km = g.Wh - 1;
        const int xp = x + 1 == g.Nx ? 0 : x + 1, xm = x == 0 ? g.Nx - 1 : x - 1;
        const long row = (long)x * g.Wh;
        const long it = row + kp, im = row + km, ixp = (long)xp * g.Wh + k, ixm = (long)xm * g.Wh + k;
        const int tg = g.t0 + t;
        const double sr0 = tg == g.Ntg - 1 ? -1.0 : 1.0;
        const double sl0 = tg == 0 ? -1.0 : 1.0;
        double2 h0, h1;
        dirac_bracket<DAG>(sr0, sl0, in[it], in[it + Vh], in[ixp], in[ixp + Vh], in[im], in[im + Vh], in[ixm],
                           in[ixm + Vh], Up[h], Up[h + Vh], Uq[im], Uq[ixm + Vh], h0, h1);
        double2 o0 = rmul(b, h0), o1 = rmul(b, h1);
        if (aux) {
            o0 = cadd(rmul(a, aux[h]), o0);
            o1 = cadd(rmul(a, aux[h + Vh]), o1);
        }
        out[h] = o0;
        out[h + Vh] = o1;
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

void launch_eo_hop(hipStream_t s, const Geometry &g, int dagger, int p, const double2 *in, const double2 *Up,
                   const double2 *Uq, const double2 *aux, double a, double b, double2 *out) {
    const EoGeom e = eo_geom(g);
    if (dagger)
        hipLaunchKernelGGL(eo_hop_kernel<1>, dim3(eo_grid(e.Vh)), dim3(256), 0, s, e, p, in, Up, Uq, aux, a, b, out);
    else
        hipLaunchKernelGGL(eo_hop_kernel<0>, dim3(eo_grid(e.Vh)), dim3(256), 0, s, e, p, in, Up, Uq, aux, a, b, out);
}

}  // namespace sm
