// membench.hip -- streaming-bandwidth micro-benchmark for MI355X (gfx950).
// Which load/store form reaches the HBM ceiling for the CG's BLAS-1 pattern
// (out = a - alpha*b, 2 reads + 1 write of 16-B complex<double>)?
//   hipcc --offload-arch=gfx950 -O3 -o tools/membench tools/membench.hip
//   tools/membench [n_complex]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

__device__ __forceinline__ double2 axpy(double2 a, double2 b, double s) { return make_double2(a.x - s * b.x, a.y - s * b.y); }

typedef double v2d __attribute__((ext_vector_type(2)));
template <bool NT>
__device__ __forceinline__ double2 ld(const double2 *p) {
    if (NT) {
        v2d v = __builtin_nontemporal_load(reinterpret_cast<const v2d *>(p));
        return make_double2(v.x, v.y);
    }
    return *p;
}
template <bool NT>
__device__ __forceinline__ void st(double2 *p, double2 v) {
    if (NT) {
        v2d w = {v.x, v.y};
        __builtin_nontemporal_store(w, reinterpret_cast<v2d *>(p));
    } else {
        *p = v;
    }
}

// V0: grid-stride, one element per iteration
template <bool NT>
__global__ void __launch_bounds__(256) k_gs1(long n, const double2 *a, const double2 *b, double2 *o, double s) {
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256)
        st<NT>(o + i, axpy(ld<NT>(a + i), ld<NT>(b + i), s));
}
// V1: grid-stride, U elements per thread per iteration, all loads first
template <bool NT, int U>
__global__ void __launch_bounds__(256) k_gsU(long n, const double2 *a, const double2 *b, double2 *o, double s) {
    const long stride = (long)gridDim.x * 256;
    long i = (long)blockIdx.x * 256 + threadIdx.x;
    for (; i + (U - 1) * stride < n; i += U * stride) {
        double2 x[U], y[U];
#pragma unroll
        for (int u = 0; u < U; ++u) { x[u] = ld<NT>(a + i + u * stride); y[u] = ld<NT>(b + i + u * stride); }
#pragma unroll
        for (int u = 0; u < U; ++u) st<NT>(o + i + u * stride, axpy(x[u], y[u], s));
    }
    for (; i < n; i += stride) st<NT>(o + i, axpy(ld<NT>(a + i), ld<NT>(b + i), s));
}
// V2: contiguous chunk per block, U consecutive 256-element tiles per step
template <bool NT, int U>
__global__ void __launch_bounds__(256) k_chunk(long n, const double2 *a, const double2 *b, double2 *o, double s) {
    const long per = (n + gridDim.x - 1) / gridDim.x;
    const long beg = (long)blockIdx.x * per, end = min(n, beg + per);
    long i = beg + threadIdx.x;
    for (; i + (U - 1) * 256 < end; i += U * 256) {
        double2 x[U], y[U];
#pragma unroll
        for (int u = 0; u < U; ++u) { x[u] = ld<NT>(a + i + u * 256); y[u] = ld<NT>(b + i + u * 256); }
#pragma unroll
        for (int u = 0; u < U; ++u) st<NT>(o + i + u * 256, axpy(x[u], y[u], s));
    }
    for (; i < end; i += 256) st<NT>(o + i, axpy(ld<NT>(a + i), ld<NT>(b + i), s));
}
// V3: each lane handles 2 adjacent complex (32 B), grid-stride
template <bool NT>
__global__ void __launch_bounds__(256) k_vec2(long n, const double2 *a, const double2 *b, double2 *o, double s) {
    const long n2 = n / 2;
    const long stride = (long)gridDim.x * 256;
    for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n2; i += stride) {
        double2 x0 = ld<NT>(a + 2 * i), x1 = ld<NT>(a + 2 * i + 1);
        double2 y0 = ld<NT>(b + 2 * i), y1 = ld<NT>(b + 2 * i + 1);
        st<NT>(o + 2 * i, axpy(x0, y0, s));
        st<NT>(o + 2 * i + 1, axpy(x1, y1, s));
    }
}

typedef void (*kfn)(long, const double2 *, const double2 *, double2 *, double);

int main(int argc, char **argv) {
    long n = argc > 1 ? atol(argv[1]) : (1L << 25);  // 2^25 complex = 512 MiB per array
    double2 *a, *b, *o;
    CHECK(hipMalloc(&a, n * 16));
    CHECK(hipMalloc(&b, n * 16));
    CHECK(hipMalloc(&o, n * 16));
    CHECK(hipMemset(a, 0, n * 16));
    CHECK(hipMemset(b, 0, n * 16));
    struct V { const char *name; kfn f; int blocks; };
    std::vector<V> vs = {
        {"gs1 2048", k_gs1<false>, 2048}, {"gs1 8192", k_gs1<false>, 8192}, {"gs1 nt 2048", k_gs1<true>, 2048},
        {"gsU4 2048", k_gsU<false, 4>, 2048}, {"gsU4 1024", k_gsU<false, 4>, 1024}, {"gsU4 4096", k_gsU<false, 4>, 4096},
        {"gsU4 nt 2048", k_gsU<true, 4>, 2048}, {"gsU8 1024", k_gsU<false, 8>, 1024},
        {"chunk4 1024", k_chunk<false, 4>, 1024}, {"chunk4 2048", k_chunk<false, 4>, 2048},
        {"chunk8 1024", k_chunk<false, 8>, 1024}, {"chunk4 nt 2048", k_chunk<true, 4>, 2048},
        {"vec2 4096", k_vec2<false>, 4096}, {"vec2 nt 4096", k_vec2<true>, 4096},
    };
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    const int reps = 20, rounds = 5;
    std::vector<std::vector<float>> t(vs.size());
    for (int r = 0; r < rounds; ++r)
        for (size_t v = 0; v < vs.size(); ++v) {
            hipLaunchKernelGGL(vs[v].f, dim3(vs[v].blocks), dim3(256), 0, 0, n, a, b, o, 0.5);
            CHECK(hipEventRecord(e0));
            for (int k = 0; k < reps; ++k) hipLaunchKernelGGL(vs[v].f, dim3(vs[v].blocks), dim3(256), 0, 0, n, a, b, o, 0.5);
            CHECK(hipEventRecord(e1));
            CHECK(hipEventSynchronize(e1));
            float ms;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            t[v].push_back(ms / reps);
        }
    for (size_t v = 0; v < vs.size(); ++v) {
        std::sort(t[v].begin(), t[v].end());
        float med = t[v][rounds / 2];
        printf("{\"variant\": \"%s\", \"us\": %.1f, \"GBps\": %.1f}\n", vs[v].name, med * 1e3, 48.0 * n / (med * 1e-3) / 1e9);
    }
    return 0;
}
