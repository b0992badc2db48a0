// membench2.hip -- which streaming form reaches the MI355X HBM ceiling for
// each access mix the Dirac/CG kernels use (16-B complex<double> per lane):
//   copy  (1 read, 1 write), axpy (2 reads, 1 write), dirac-like (3 reads,
//   1 write), read-only (1 read + per-block partial).
// Sweeps block size, grid size, per-thread unroll and nt on loads / stores.
//   hipcc --offload-arch=gfx950 -O3 -o tools/membench2 tools/membench2.hip
//   tools/membench2 [n_complex]
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

typedef double v2d __attribute__((ext_vector_type(2)));
template <bool NT>
__device__ __forceinline__ v2d ld(const v2d *p) {
    if (NT) return __builtin_nontemporal_load(p);
    return *p;
}
template <bool NT>
__device__ __forceinline__ void st(v2d *p, v2d v) {
    if (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}

// R reads, W (0/1) writes per element; contiguous chunk per block, U tiles
// of blockDim consecutive elements per step, all loads of a step first.
template <int R, int W, bool NTL, bool NTS, int U, int BS>
__global__ void __launch_bounds__(BS) k_chunk(long n, const v2d *a, const v2d *b, const v2d *c, v2d *o, double *part) {
    const long per = (n + gridDim.x - 1) / gridDim.x;
    const long beg = (long)blockIdx.x * per, end = min(n, beg + per);
    long i = beg + threadIdx.x;
    v2d acc = {0.0, 0.0};
    for (; i + (U - 1) * BS < end; i += U * BS) {
        v2d x[U], y[U], z[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            x[u] = ld<NTL>(a + i + u * BS);
            if (R > 1) y[u] = ld<NTL>(b + i + u * BS);
            if (R > 2) z[u] = ld<NTL>(c + i + u * BS);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            v2d v = x[u];
            if (R > 1) v = v - 0.5 * y[u];
            if (R > 2) v = v + 0.25 * z[u];
            if (W) st<NTS>(o + i + u * BS, v);
            else acc += v;
        }
    }
    for (; i < end; i += BS) {
        v2d v = ld<NTL>(a + i);
        if (R > 1) v = v - 0.5 * ld<NTL>(b + i);
        if (R > 2) v = v + 0.25 * ld<NTL>(c + i);
        if (W) st<NTS>(o + i, v);
        else acc += v;
    }
    if (!W && acc.x == 12345.678) part[blockIdx.x] = acc.y;  // keep the loads alive
}

typedef void (*kfn)(long, const v2d *, const v2d *, const v2d *, v2d *, double *);
struct V { std::string name; kfn f; int bs, blocks, streams; };

template <int R, int W, bool NTL, bool NTS, int U, int BS>
void add(std::vector<V> &vs, const char *mix, std::initializer_list<int> grids) {
    for (int g : grids) {
        char buf[128];
        snprintf(buf, sizeof buf, "%s ntl%d nts%d U%d bs%d g%d", mix, NTL, NTS, U, BS, g);
        vs.push_back({buf, k_chunk<R, W, NTL, NTS, U, BS>, BS, g, R + W});
    }
}

int main(int argc, char **argv) {
    long n = argc > 1 ? atol(argv[1]) : (1L << 25);  // 2^25 complex = 512 MiB per array
    v2d *a, *b, *c, *o;
    double *part;
    CHECK(hipMalloc(&a, n * 16));
    CHECK(hipMalloc(&b, n * 16));
    CHECK(hipMalloc(&c, n * 16));
    CHECK(hipMalloc(&o, n * 16));
    CHECK(hipMalloc(&part, 1 << 20));
    CHECK(hipMemset(a, 0, n * 16));
    CHECK(hipMemset(b, 0, n * 16));
    CHECK(hipMemset(c, 0, n * 16));
    std::vector<V> vs;
    // copy
    add<1, 1, true, true, 4, 256>(vs, "copy", {1024, 2048, 4096});
    add<1, 1, false, false, 4, 256>(vs, "copy", {2048});
    add<1, 1, true, true, 2, 512>(vs, "copy", {1024, 2048});
    add<1, 1, true, true, 8, 256>(vs, "copy", {1024, 2048});
    add<1, 1, false, true, 4, 256>(vs, "copy", {2048});
    // read only
    add<1, 0, true, false, 4, 256>(vs, "read", {1024, 2048, 4096});
    add<1, 0, false, false, 4, 256>(vs, "read", {2048});
    add<1, 0, true, false, 8, 256>(vs, "read", {2048});
    // axpy 2R1W
    add<2, 1, true, true, 4, 256>(vs, "axpy", {1024, 2048, 4096, 8192});
    add<2, 1, true, true, 2, 256>(vs, "axpy", {2048, 4096});
    add<2, 1, true, true, 8, 256>(vs, "axpy", {1024, 2048});
    add<2, 1, true, true, 2, 512>(vs, "axpy", {1024, 2048});
    add<2, 1, true, true, 1, 1024>(vs, "axpy", {1024, 2048});
    add<2, 1, false, true, 4, 256>(vs, "axpy", {2048});
    add<2, 1, true, false, 4, 256>(vs, "axpy", {2048});
    add<2, 1, false, false, 4, 256>(vs, "axpy", {2048});
    // 3R1W (Dirac-like mix)
    add<3, 1, true, true, 4, 256>(vs, "r3w1", {1024, 2048, 4096});
    add<3, 1, true, true, 2, 256>(vs, "r3w1", {2048, 4096});
    add<3, 1, false, true, 4, 256>(vs, "r3w1", {2048});
    add<3, 1, true, true, 2, 512>(vs, "r3w1", {2048});

    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    const int reps = 20, rounds = 5;
    std::vector<std::vector<float>> t(vs.size());
    for (int r = 0; r < rounds; ++r)
        for (size_t v = 0; v < vs.size(); ++v) {
            hipLaunchKernelGGL(vs[v].f, dim3(vs[v].blocks), dim3(vs[v].bs), 0, 0, n, a, b, c, o, part);
            CHECK(hipEventRecord(e0));
            for (int k = 0; k < reps; ++k)
                hipLaunchKernelGGL(vs[v].f, dim3(vs[v].blocks), dim3(vs[v].bs), 0, 0, n, a, b, c, o, part);
            CHECK(hipEventRecord(e1));
            CHECK(hipEventSynchronize(e1));
            float ms;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            t[v].push_back(ms / reps);
        }
    for (size_t v = 0; v < vs.size(); ++v) {
        std::sort(t[v].begin(), t[v].end());
        const float med = t[v][rounds / 2];
        printf("{\"variant\": \"%s\", \"us\": %.1f, \"GBps\": %.1f}\n", vs[v].name.c_str(), med * 1e3,
               16.0 * vs[v].streams * n / (med * 1e-3) / 1e9);
    }
    return 0;
}
