// pool_offsets.hip -- can the CG pass's fast placement be had by RULE? The
// five streamed buffers (three directions, x, link codes) are carved out of
// ONE allocation requested as physically contiguous, at chosen offsets, so
// their relative physical placement is the relative virtual one (if the
// driver honours the flag). Each pattern is timed in interleaved rounds; a
// pattern that is fast in every process and on every box would replace the
// placement probe.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I include -c tools/pool_offsets.hip -o po.o &&
//   hipcc --offload-arch=gfx950 po.o build/sm_hip/sm_cgra.hip.o build/sm_hip/sm_kernels.hip.o -o tools/pool_offsets
//   tools/pool_offsets 4096 [rounds]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
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

int main(int argc, char **argv) {
    const int N = argc > 1 ? atoi(argv[1]) : 4096;
    const int R = argc > 2 ? atoi(argv[2]) : 3;
    const long V = (long)N * N;
    const size_t fb = sizeof(double2) * 2 * (size_t)V;
    const size_t G = size_t(1) << 30, M = size_t(1) << 20, K = size_t(1) << 10;
    const size_t pool_bytes = 16 * G;
    char *pool = nullptr;
    const bool contiguous = hipExtMallocWithFlags((void **)&pool, pool_bytes, hipDeviceMallocContiguous) == hipSuccess;
    if (!contiguous) {
        (void)hipGetLastError();
        CHECK(hipMalloc(&pool, pool_bytes));
    }
    hipLaunchKernelGGL(fill_kernel, dim3(8192), dim3(256), 0, 0, (long)(pool_bytes / sizeof(double2)), (double2 *)pool,
                       0.25);
    CHECK(hipDeviceSynchronize());
    // offsets of (d0, d1, d2, x, codes); every buffer takes fb (codes: fb too, generous)
    struct Pat {
        std::string name;
        size_t off[5];
    };
    std::vector<Pat> pats;
    auto stride = [&](const char *nm, size_t s) {
        Pat p{nm, {}};
        for (int k = 0; k < 5; ++k) p.off[k] = k * s;
        pats.push_back(p);
    };
    stride("packed", fb);
    stride("packed+2MiB", fb + 2 * M);
    stride("packed+64KiB", fb + 64 * K);
    stride("2GiB", 2 * G);
    stride("2GiB+2MiB", 2 * G + 2 * M);
    stride("2GiB+64KiB", 2 * G + 64 * K);
    stride("2GiB+256KiB", 2 * G + 256 * K);
    stride("2GiB+8MiB", 2 * G + 8 * M);
    stride("3GiB", 3 * G);
    stride("1GiB", 1 * G);
    std::mt19937_64 rng(12345);
    for (int r = 0; r < 10; ++r) {  // random slot order and 64-KiB jitter inside 3-GiB slots
        Pat p{"random" + std::to_string(r), {}};
        int perm[5] = {0, 1, 2, 3, 4};
        std::shuffle(perm, perm + 5, rng);
        for (int k = 0; k < 5; ++k) p.off[k] = perm[k] * 3 * G + (rng() % (1024 * M / (64 * K))) * 64 * K;
        pats.push_back(p);
    }
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
    CGScalars h;
    memset(&h, 0, sizeof(h));
    h.max_iter = 1 << 30;
    h.phi_norm = 1.0;
    CHECK(hipMemcpy(sc, &h, sizeof(h), hipMemcpyHostToDevice));
    Geometry g;
    g.Nx = N;
    g.Wt = N;
    g.t0 = 0;
    g.Ntg = N;
    g.V = V;
    const CGFusedCfg rc = cg_ra_config(g);
    const int nparts = rc.TBk * rc.XB;
    long j = 2;
    hipEvent_t ea, eb;
    CHECK(hipEventCreate(&ea));
    CHECK(hipEventCreate(&eb));
    auto time_pat = [&](const Pat &p) {
        double2 *f[5];
        for (int k = 0; k < 5; ++k) f[k] = (double2 *)(pool + p.off[k]);
        std::vector<float> v;
        for (int r = -1; r < 3; ++r) {
            CHECK(hipEventRecord(ea, s));
            for (int i = 0; i < 6; ++i, ++j)
                launch_cg_ra(s, g, rc, 1, f[(j + 2) % 3], f[(j + 1) % 3], f[j % 3], f[3], nullptr, nullptr, nullptr,
                             nullptr, 1.94, j, sc, part, 0, rc.TBk, nullptr, (const double *)f[4], nullptr, nullptr,
                             0, tick, nparts, gsum, nullptr, 0, 2);
            CHECK(hipEventRecord(eb, s));
            CHECK(hipEventSynchronize(eb));
            float ms;
            CHECK(hipEventElapsedTime(&ms, ea, eb));
            if (r >= 0) v.push_back(ms * 1000.f / 6);
        }
        std::sort(v.begin(), v.end());
        return (double)v[1];
    };
    std::vector<std::vector<double>> t(pats.size());
    for (int r = 0; r < R; ++r)
        for (size_t i = 0; i < pats.size(); ++i) t[i].push_back(time_pat(pats[i]));
    CHECK(hipGetLastError());
    for (size_t i = 0; i < pats.size(); ++i) {
        std::sort(t[i].begin(), t[i].end());
        printf("{\"N\": %d, \"contiguous\": %d, \"pattern\": \"%s\", \"offsets_MiB\": [", N, contiguous ? 1 : 0,
               pats[i].name.c_str());
        for (int k = 0; k < 5; ++k) printf("%s%.4f", k ? ", " : "", pats[i].off[k] / (double)M);
        printf("], \"us\": %.2f, \"min\": %.2f, \"max\": %.2f}\n", t[i][t[i].size() / 2], t[i].front(), t[i].back());
    }
    return 0;
}
