// layout_probe.hip -- does the HBM placement of the fields move the Dirac
// apply / recompute-Ad CG pass off its ~5.7 TB/s plateau?
//
// The product kernels take the plane stride as a runtime value (Geometry.V),
// so this probe runs the unmodified launchers (sm_kernels.hip, sm_cgra.hip)
// on fields carved out of one pool with
//   PG: extra elements between plane 0 and plane 1 of every field
//       (plane stride V + PG instead of the power-of-two V = 4096^2), and
//   AG: extra elements between consecutive fields (ψ, U, out, ...).
// Timing: hipEvents on the launch stream, median of R reps of K launches.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I include \
//     tools/layout_probe.hip build/sm_hip/sm_kernels.hip.o build/sm_hip/sm_cgra.hip.o -o tools/layout_probe
//   tools/layout_probe 4096 "0,0" "16,0" "256,0" "0,4096" ...
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../schwingermodel_amd/csrc/sm_internal.h"

#define CHECK(x)                                                                \
    do {                                                                        \
        hipError_t e_ = (x);                                                    \
        if (e_ != hipSuccess) {                                                 \
            printf("%s: %s\n", #x, hipGetErrorString(e_));                      \
            exit(1);                                                            \
        }                                                                       \
    } while (0)

using namespace sm;

__global__ void fill_kernel(long n, double2 *p, double v) {
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
        p[i] = make_double2(v + 1e-9 * (double)(i & 1023), -v);
}

template <typename F>
static double time_us(hipStream_t s, int K, int R, F launch) {
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    for (int i = 0; i < 3; ++i) launch();
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
    // argv[1]: "N" (N x N) or "NxxNt"; the pool is sized for the largest lattice asked
    int N = 4096, NT = 4096;
    if (argc > 1 && sscanf(argv[1], "%dx%d", &N, &NT) != 2) NT = N = atoi(argv[1]);
    const long V = (long)N * NT;
    const long maxPG = 1 << 16, maxAG = 1 << 20;
    const int NF = 6;  // in/d1, U, out/dn, d2, x, spare
    const size_t pool_elems = (size_t)NF * (2 * (V + maxPG) + maxAG) + 4096;
    double2 *pool;
    CHECK(hipMalloc(&pool, pool_elems * sizeof(double2)));
    hipLaunchKernelGGL(fill_kernel, dim3(4096), dim3(256), 0, 0, (long)pool_elems, pool, 0.25);
    CHECK(hipDeviceSynchronize());
    hipStream_t s;
    CHECK(hipStreamCreate(&s));
    CGScalars *sc;
    CHECK(hipMalloc(&sc, sizeof(CGScalars)));
    CHECK(hipMemset(sc, 0, sizeof(CGScalars)));
    double2 *part;
    CHECK(hipMalloc(&part, sizeof(double2) * 2 * kMaxPartials));
    for (int ai = 2; ai < argc; ++ai) {
        long PG = 0, AG = 0;
        sscanf(argv[ai], "%ld,%ld", &PG, &AG);
        if (PG < 0 || PG > maxPG || AG < 0 || AG > maxAG) continue;
        const long PS = V + PG;
        double2 *f[NF];
        for (int k = 0; k < NF; ++k) f[k] = pool + (size_t)k * (2 * PS + AG);
        Geometry g;
        g.Nx = N;
        g.Wt = NT;
        g.t0 = 0;
        g.Ntg = NT;
        g.V = PS;
        LaunchCfg dc = dslash_config(g);
        TFaces tf;
        tf.lo = f[0] + (NT - 1);
        tf.lo_xs = NT;
        tf.lo_ps = PS;
        tf.hi = f[0];
        tf.hi_xs = NT;
        tf.hi_ps = PS;
        const double us_d = time_us(s, 20, 7, [&] {
            launch_dslash(s, g, dc, 0, f[0], f[2], f[1], f[1] + (NT - 1), tf, -0.06, nullptr, nullptr, nullptr);
        });
        CGFusedCfg rc = cg_ra_config(g);
        const double us_odd = time_us(s, 10, 5, [&] {
            launch_cg_ra(s, g, rc, 1, f[0], f[3], f[2], f[4], f[1], nullptr, nullptr, nullptr, -0.06, 3, sc, part, 0,
                         rc.TBk, nullptr);
        });
        const double us_even = time_us(s, 10, 5, [&] {
            launch_cg_ra(s, g, rc, 1, f[0], f[3], f[2], f[4], f[1], nullptr, nullptr, nullptr, -0.06, 4, sc, part, 0,
                         rc.TBk, nullptr);
        });
        // link angles (16 B/site instead of 32): the UC variant of the same passes
        const double *Ua = reinterpret_cast<const double *>(f[5]);
        const double us_odd_a = time_us(s, 10, 5, [&] {
            launch_cg_ra(s, g, rc, 1, f[0], f[3], f[2], f[4], f[1], nullptr, nullptr, nullptr, -0.06, 3, sc, part, 0,
                         rc.TBk, nullptr, Ua);
        });
        const double us_even_a = time_us(s, 10, 5, [&] {
            launch_cg_ra(s, g, rc, 1, f[0], f[3], f[2], f[4], f[1], nullptr, nullptr, nullptr, -0.06, 4, sc, part, 0,
                         rc.TBk, nullptr, Ua);
        });
        CHECK(hipGetLastError());
        const double ns_site = 1e3 / (double)V;  // us -> ns per site
        printf("{\"Nx\": %d, \"Nt\": %d, \"plane_gap\": %ld, \"array_gap\": %ld, \"dslash_us\": %.2f, "
               "\"dslash_GBps\": %.1f, \"cg_odd_us\": %.2f, \"cg_even_us\": %.2f, \"cg_iter_ms\": %.4f, "
               "\"angles_odd_us\": %.2f, \"angles_even_us\": %.2f, \"angles_iter_ms\": %.4f, "
               "\"ps_per_site\": {\"dslash\": %.3f, \"cg\": %.3f, \"cg_angles\": %.3f}}\n",
               N, NT, PG, AG, us_d, 96.0 * V / us_d / 1e3, us_odd, us_even, (us_odd + us_even) / 2e3, us_odd_a,
               us_even_a, (us_odd_a + us_even_a) / 2e3, 1e3 * us_d * ns_site,
               1e3 * (us_odd + us_even) / 2 * ns_site, 1e3 * (us_odd_a + us_even_a) / 2 * ns_site);
        fflush(stdout);
    }
    return 0;
}
