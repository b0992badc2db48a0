// shape_tune.hip -- launch-geometry sweep of the two hot kernels at the
// lattice / shard shapes of the BASELINE configs (4096^2; 4096 x 4096/N for the
// t-sharded config 4; 8192^2 and 8192 x 1024 for config 5; 1024^2, 2048^2).
//
// Runs the product launchers (sm_kernels.hip launch_dslash, sm_cgra.hip
// launch_cg_ra) with explicit LaunchCfg / CGFusedCfg values on one shard and
// prints one JSON line per (shape, kernel, config): the median time per launch
// over R reps of K back-to-back launches (hipEvents on the launch stream).
// The CG pass is timed as one odd + one even pass (x update), with the link
// angles (UC) and with complex links.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I include -c tools/shape_tune.hip -o /tmp/st.o
//   hipcc --offload-arch=gfx950 /tmp/st.o build/sm_hip/sm_kernels.hip.o build/sm_hip/sm_cgra.hip.o -o tools/shape_tune
//   tools/shape_tune 4096x4096 4096x512 ...
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../schwingermodel_amd/csrc/sm_internal.h"

#define CHECK(x)                                                           \
    do {                                                                   \
        hipError_t e_ = (x);                                               \
        if (e_ != hipSuccess) {                                            \
            printf("%s: %s\n", #x, hipGetErrorString(e_));                 \
            exit(1);                                                       \
        }                                                                  \
    } while (0)

using namespace sm;

__global__ void fill_kernel(long n, double2 *p, double v) {
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
        const double th = v + 1e-7 * (double)(i & 4095);
        p[i] = make_double2(cos(th), sin(th));
    }
}

template <typename F>
static double time_us(hipStream_t s, int K, int R, F launch) {
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    for (int i = 0; i < 2; ++i) launch();
    std::vector<float> v;
    for (int r = 0; r < R; ++r) {
        CHECK(hipEventRecord(a, s));
        for (int i = 0; i < K; ++i) launch();
        CHECK(hipEventRecord(b, s));
        CHECK(hipEventSynchronize(b));
        float ms;
        CHECK(hipEventElapsedTime(&ms, a, b));
        v.push_back(ms * 1000.f / K);
    }
    std::sort(v.begin(), v.end());
    CHECK(hipEventDestroy(a));
    CHECK(hipEventDestroy(b));
    return v[v.size() / 2];
}

int main(int argc, char **argv) {
    hipStream_t s;
    CHECK(hipStreamCreate(&s));
    CGScalars *sc;
    CHECK(hipMalloc(&sc, sizeof(CGScalars)));
    CHECK(hipMemset(sc, 0, sizeof(CGScalars)));
    double2 *part;
    CHECK(hipMalloc(&part, sizeof(double2) * 2 * kMaxPartials));
    for (int ai = 1; ai < argc; ++ai) {
        int Nx, Nt;
        if (sscanf(argv[ai], "%dx%d", &Nx, &Nt) != 2) continue;
        const long V = (long)Nx * Nt;
        const int NF = 6;  // d1/in, U, dn/out, d2, x, angles
        double2 *pool;
        CHECK(hipMalloc(&pool, sizeof(double2) * NF * 2 * (size_t)V));
        hipLaunchKernelGGL(fill_kernel, dim3(4096), dim3(256), 0, s, (long)NF * 2 * V, pool, 0.3);
        CHECK(hipStreamSynchronize(s));
        double2 *f[NF];
        for (int k = 0; k < NF; ++k) f[k] = pool + (size_t)k * 2 * V;
        Geometry g;
        g.Nx = Nx;
        g.Wt = Nt;
        g.t0 = 0;
        g.Ntg = Nt;
        g.V = V;
        TFaces tf;
        tf.lo = f[0] + (Nt - 1);
        tf.lo_xs = Nt;
        tf.lo_ps = V;
        tf.hi = f[0];
        tf.hi_xs = Nt;
        tf.hi_ps = V;
        const int K = V >= (1L << 24) ? 10 : 30;
        // ---- Dirac apply -------------------------------------------------------
        const LaunchCfg d0 = dslash_config(g);
        for (int bt : {256, 128, 64}) {
            for (int xc : {0, 4, 8, 12, 16, 24, 32, 48, 64}) {
                LaunchCfg c = d0;
                c.bt = bt;
                if (xc) c.xchunk = xc;
                else if (bt != d0.bt) continue;  // xc = 0: the default config
                if (c.xchunk > Nx || dslash_blocks(g, c) > kMaxPartials) continue;
                const double us = time_us(s, K, 5, [&] {
                    launch_dslash(s, g, c, 0, f[0], f[2], f[1], f[1] + (Nt - 1), tf, -0.06, nullptr, nullptr, nullptr);
                });
                CHECK(hipGetLastError());
                printf("{\"shape\": \"%dx%d\", \"kernel\": \"dslash\", \"bt\": %d, \"xchunk\": %d, \"default\": %d, "
                       "\"blocks\": %d, \"us\": %.2f, \"GBps\": %.1f}\n",
                       Nx, Nt, c.bt, c.xchunk, xc == 0, dslash_blocks(g, c), us, 96.0 * V / us / 1e3);
                fflush(stdout);
            }
        }
        // ---- recompute-Ad CG pass -----------------------------------------------
        const CGFusedCfg r0 = cg_ra_config(g);
        const double *Ua = reinterpret_cast<const double *>(f[5]);
        for (int wpb : {4, 2, 1}) {
            for (int xc : {0, 8, 12, 16, 20, 24, 28, 32, 40, 48, 64}) {
                CGFusedCfg c = r0;
                c.wpb = wpb;
                c.TBk = (c.NWT + wpb - 1) / wpb;
                if (xc) c.xchunk = xc;
                else if (wpb != r0.wpb) continue;
                if (c.xchunk > Nx) continue;
                c.XB = (Nx + c.xchunk - 1) / c.xchunk;
                if (3L * (c.TBk * c.XB) > 2L * kMaxPartials) continue;
                for (int ang = 1; ang >= 0; --ang) {
                    const double *ua = ang ? Ua : nullptr;
                    const double us = time_us(s, K / 2, 5, [&] {
                        launch_cg_ra(s, g, c, 1, f[0], f[3], f[2], f[4], f[1], nullptr, nullptr, nullptr, -0.06, 3, sc,
                                     part, 0, c.TBk, nullptr, ua);
                        launch_cg_ra(s, g, c, 1, f[0], f[3], f[2], f[4], f[1], nullptr, nullptr, nullptr, -0.06, 4, sc,
                                     part, 0, c.TBk, nullptr, ua);
                    });
                    CHECK(hipGetLastError());
                    printf("{\"shape\": \"%dx%d\", \"kernel\": \"cg_ra\", \"angles\": %d, \"wpb\": %d, \"xchunk\": %d, "
                           "\"default\": %d, \"blocks\": %d, \"ms_per_iter\": %.4f, \"ps_per_site\": %.3f}\n",
                           Nx, Nt, ang, wpb, c.xchunk, xc == 0, (c.TBk * c.XB), us / 2e3, us / 2 / V * 1e6);
                    fflush(stdout);
                }
            }
        }
        CHECK(hipFree(pool));
    }
    return 0;
}
