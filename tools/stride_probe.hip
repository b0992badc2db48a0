// stride_probe.hip -- does the HBM spacing of the CG pass's streams set its
// rate? (The same pass streams 11 % more bytes per second at 8192^2 than at
// 4096^2, 4096x8192 or 8192x4096: tools/shape_probe.py.)
//
// Runs the product launcher (sm_cgra.hip, launch_cg_ra: link angles, ticketed
// tail, the per-shape march schedule) the way sm_capi.cpp's one-shard pass
// does, with d_j rotating through three buffers, on fields carved out of one
// pool with a chosen plane stride PS (elements between plane 0 and plane 1 of
// every field, >= V) and field stride FS (elements between the starts of
// consecutive fields, >= 2 PS). Median of R reps of K passes, hipEvents.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I include -c tools/stride_probe.hip -o sp.o &&
//   hipcc --offload-arch=gfx950 sp.o build/sm_hip/sm_cgra.hip.o build/sm_hip/sm_kernels.hip.o -o tools/stride_probe
//   tools/stride_probe 4096x4096 "1,2" "4,8" "1,2,1,1,8" "1,2,0,0,0,2048" ...   (PS, FS in units of V[, random values, separate allocations[,
//     their size in V[, pool: extra KiB before field k, times k]]])
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
        p[i] = make_double2(v + 1e-9 * (double)(i & 1023), -v + 1e-10 * (double)(i & 511));
}

// uniform values in [-a, a) from a splitmix64 hash of the element index
__device__ inline double hash_unit(unsigned long long z) {
    z += 0x9e3779b97f4a7c15ull;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    z ^= z >> 31;
    return (double)(z >> 11) * (1.0 / 9007199254740992.0) * 2.0 - 1.0;
}
__global__ void fill_rand_kernel(long n, double2 *p, double a, unsigned long long seed) {
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
        p[i] = make_double2(a * hash_unit(seed + 2 * (unsigned long long)i), a * hash_unit(seed + 2 * (unsigned long long)i + 1));
}

int main(int argc, char **argv) {
    int N = 4096, NT = 4096;
    if (argc > 1 && sscanf(argv[1], "%dx%d", &N, &NT) != 2) NT = N = atoi(argv[1]);
    const long V = (long)N * NT;
    // fields: 3 direction buffers, x, angles (doubles: 2 planes of PS doubles fit in PS double2)
    const int NF = 5;
    long maxFS = 2 * V;
    for (int ai = 2; ai < argc; ++ai) {
        long ps = 1, fs = 2;
        sscanf(argv[ai], "%ld,%ld", &ps, &fs);
        maxFS = std::max(maxFS, std::max(fs, 2 * ps) * V + (8L << 30) / (long)sizeof(double2) / 5);
    }
    const size_t pool_elems = (size_t)NF * maxFS + 4096;
    double2 *pool;
    CHECK(hipMalloc(&pool, pool_elems * sizeof(double2)));
    hipLaunchKernelGGL(fill_kernel, dim3(4096), dim3(256), 0, 0, (long)pool_elems, pool, 0.25);
    CHECK(hipDeviceSynchronize());
    hipStream_t s;
    CHECK(hipStreamCreate(&s));
    CGScalars *sc;
    CHECK(hipMalloc(&sc, sizeof(CGScalars)));
    double2 *part, *gsum;
    unsigned *tick;
    CHECK(hipMalloc(&part, sizeof(double2) * 3 * kMaxPartials));
    CHECK(hipMalloc(&gsum, sizeof(double2) * 3 * kMaxTickGroups));
    CHECK(hipMalloc(&tick, sizeof(unsigned) * (1 + kMaxTickGroups)));
    CHECK(hipMemset(tick, 0, sizeof(unsigned) * (1 + kMaxTickGroups)));
    for (int ai = 2; ai < argc; ++ai) {
        long psm = 1, fsm = 2;
        int rnd = 0, sep = 0;  // rnd: random field values (angles in [-0.5, 0.5)); sep: one hipMalloc per field
        long asm_ = 0;         // sep: allocation size per field in units of V (default 2 PS)
        long offk = 0;         // pool: field k starts offk * k KiB further in
        sscanf(argv[ai], "%ld,%ld,%d,%d,%ld,%ld", &psm, &fsm, &rnd, &sep, &asm_, &offk);
        if (psm < 1 || fsm < 2 * psm) continue;
        const long PS = psm * V, FS = fsm * V;
        double2 *f[NF];
        // sep 1: every field its own allocation of asm_ V; 2: the same but x (k = 3) at its own size;
        // 3: the direction buffers in the pool, x and the angles in allocations of their own size
        bool own[NF];
        for (int k = 0; k < NF; ++k) {
            own[k] = sep == 1 || sep == 2 || (sep == 3 && k >= 3);
            const size_t bytes = sizeof(double2) * (size_t)(((sep == 2 && k == 3) || sep == 3) ? 2 * PS
                                                                                                : std::max(2 * PS, asm_ * V));
            if (own[k]) CHECK(hipMalloc(&f[k], bytes));
            else f[k] = pool + (size_t)k * FS + (size_t)(offk * k) * 1024 / sizeof(double2);
            if (rnd) hipLaunchKernelGGL(fill_rand_kernel, dim3(4096), dim3(256), 0, 0, 2 * PS, f[k], k == 4 ? 0.5 : 1.0,
                                        (unsigned long long)(k + 1) << 40);
            else if (own[k]) hipLaunchKernelGGL(fill_kernel, dim3(4096), dim3(256), 0, 0, 2 * PS, f[k], 0.25);
        }
        CHECK(hipDeviceSynchronize());
        Geometry g;
        g.Nx = N;
        g.Wt = NT;
        g.t0 = 0;
        g.Ntg = NT;
        g.V = PS;
        CGFusedCfg rc = cg_ra_config(g);
        const int nparts = rc.TBk * rc.XB;
        // tol 0, no stop: every pass does the full work
        CGScalars h;
        memset(&h, 0, sizeof(h));
        h.max_iter = 1 << 30;
        h.phi_norm = 1.0;
        CHECK(hipMemcpy(sc, &h, sizeof(h), hipMemcpyHostToDevice));
        const double *Ua = reinterpret_cast<const double *>(f[4]);
        long j = 0;
        auto pass = [&] {
            double2 *dn = f[j % 3], *d1 = f[(j + 2) % 3], *d2 = f[(j + 1) % 3];
            launch_cg_ra(s, g, rc, 1, d1, d2, dn, f[3], nullptr, nullptr, nullptr, nullptr, -0.06, j + 2, sc, part,
                         0, rc.TBk, nullptr, Ua, nullptr, nullptr, 0, tick, nparts, gsum, nullptr);
            ++j;
        };
        hipEvent_t a, b;
        CHECK(hipEventCreate(&a));
        CHECK(hipEventCreate(&b));
        for (int i = 0; i < 40; ++i) pass();
        std::vector<float> v;
        const int K = 40, R = 5;
        for (int r = 0; r < R; ++r) {
            CHECK(hipEventRecord(a, s));
            for (int i = 0; i < K; ++i) pass();
            CHECK(hipEventRecord(b, s));
            CHECK(hipEventSynchronize(b));
            float ms;
            CHECK(hipEventElapsedTime(&ms, a, b));
            v.push_back(ms * 1000.f / K);
        }
        CHECK(hipGetLastError());
        std::sort(v.begin(), v.end());
        const double us = v[v.size() / 2];
        printf("{\"Nx\": %d, \"Nt\": %d, \"plane_stride_V\": %ld, \"field_stride_V\": %ld, \"random\": %d, "
               "\"separate\": %d, \"alloc_V\": %ld, \"offset_KiB\": %ld, \"us_per_pass\": %.2f, \"ps_per_site\": %.2f, \"alg_TBps\": %.3f, \"min_us\": %.2f, "
               "\"max_us\": %.2f}\n",
               N, NT, psm, fsm, rnd, sep, asm_, offk, us, us * 1e6 / (double)V, 144.0 * V / us / 1e6, v.front(), v.back());
        for (int k = 0; k < NF; ++k)
            if (own[k]) CHECK(hipFree(f[k]));
        fflush(stdout);
        CHECK(hipEventDestroy(a));
        CHECK(hipEventDestroy(b));
    }
    return 0;
}
