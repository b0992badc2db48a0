// membench4.hip -- membench3 plus scrambled oneshot order, staggered chunks and padded row strides.
// HBM ceiling?  membench2 only tried block-contiguous chunks (every block
// walks its own far-apart region).  Here the same 16-B-per-lane copy / axpy /
// 3R1W mixes run in three orders:
//   chunk  : block b owns [b*per, (b+1)*per), U tiles per step (membench2)
//   gstride: classic grid-stride sweep; all resident blocks touch one
//            contiguous window of grid*BS*U elements at a time
//   oneshot: one U-tile per block, grid = n/(BS*U) blocks (no loop)
// and, for the Dirac-like 2D access, a "rows" order: a block owns 256
// t-columns of R fields and marches X rows of stride Nt (like dslash).
//   hipcc --offload-arch=gfx950 -O3 -o tools/membench3 tools/membench3.hip
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
__device__ __forceinline__ v2d ld_(const v2d *p) { return ld<NT>(p); }
template <bool NT>
__device__ __forceinline__ void st(v2d *p, v2d v) {
    if (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}

template <int R, int U, int BS, bool NTL, bool NTS>
__device__ __forceinline__ void tile(long i, long step, const v2d *a, const v2d *b, const v2d *c, v2d *o) {
    v2d x[U], y[U], z[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        x[u] = ld<NTL>(a + i + u * step);
        if (R > 1) y[u] = ld<NTL>(b + i + u * step);
        if (R > 2) z[u] = ld<NTL>(c + i + u * step);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        v2d v = x[u];
        if (R > 1) v = v - 0.5 * y[u];
        if (R > 2) v = v + 0.25 * z[u];
        st<NTS>(o + i + u * step, v);
    }
}

template <int R, int U, int BS, bool NTL, bool NTS>
__global__ void __launch_bounds__(BS) k_chunk(long n, long, const v2d *a, const v2d *b, const v2d *c, v2d *o) {
    const long per = (n + gridDim.x - 1) / gridDim.x;
    const long beg = (long)blockIdx.x * per, end = min(n, beg + per);
    long i = beg + threadIdx.x;
    for (; i + (U - 1) * BS < end; i += U * BS) tile<R, U, BS, NTL, NTS>(i, BS, a, b, c, o);
}

template <int R, int U, int BS, bool NTL, bool NTS>
__global__ void __launch_bounds__(BS) k_gstride(long n, long, const v2d *a, const v2d *b, const v2d *c, v2d *o) {
    const long span = (long)gridDim.x * BS;
    long i = (long)blockIdx.x * BS + threadIdx.x;
    for (; i + (U - 1) * span < n; i += U * span) tile<R, U, BS, NTL, NTS>(i, span, a, b, c, o);
}

template <int R, int U, int BS, bool NTL, bool NTS>
__global__ void __launch_bounds__(BS) k_oneshot(long n, long, const v2d *a, const v2d *b, const v2d *c, v2d *o) {
    long i = (long)blockIdx.x * BS * U + threadIdx.x;
    if (i + (U - 1) * BS < n) tile<R, U, BS, NTL, NTS>(i, BS, a, b, c, o);
}

// rows: n = Nx*Nt with Nt = nt; block = (t-tile of BS columns, x-chunk of X rows)
template <int R, int X, int BS, bool NTL, bool NTS>
__global__ void __launch_bounds__(BS) k_rows(long n, long nt, const v2d *a, const v2d *b, const v2d *c, v2d *o) {
    const long ttiles = nt / BS;
    const long tt = blockIdx.x % ttiles, xc = blockIdx.x / ttiles;
    long i = xc * X * nt + tt * BS + threadIdx.x;
#pragma unroll 4
    for (int r = 0; r < X; ++r, i += nt) {
        v2d v = ld<NTL>(a + i);
        if (R > 1) v = v - 0.5 * ld<NTL>(b + i);
        if (R > 2) v = v + 0.25 * ld<NTL>(c + i);
        st<NTS>(o + i, v);
    }
}


// oneshot in a scrambled tile order: tile = (b * P) mod nblocks, P odd, so
// concurrently resident blocks touch addresses all over the arrays.
template <int R, int U, int BS, bool NTL, bool NTS>
__global__ void __launch_bounds__(BS) k_oneshotperm(long n, long, const v2d *a, const v2d *b, const v2d *c, v2d *o) {
    const long nb = gridDim.x;
    const long tb = ((long)blockIdx.x * 40503L) % nb;
    long i = tb * BS * U + threadIdx.x;
    if (i + (U - 1) * BS < n) tile<R, U, BS, NTL, NTS>(i, BS, a, b, c, o);
}
// chunk with block starts staggered by (b*13 mod 32) * 4 KiB inside a rotated range
template <int R, int U, int BS, bool NTL, bool NTS>
__global__ void __launch_bounds__(BS) k_chunkstag(long n, long, const v2d *a, const v2d *b, const v2d *c, v2d *o) {
    const long per = n / gridDim.x;
    const long beg = (long)blockIdx.x * per;
    const long rot = (((blockIdx.x * 13) & 31) * (long)(BS * U)) % per;  // per % (U*BS) == 0 (host-checked)
    for (long k = 0; k < per; k += U * BS) {
        long off = k + rot;
        if (off >= per) off -= per;
        tile<R, U, BS, NTL, NTS>(beg + off + threadIdx.x, BS, a, b, c, o);
    }
}
// rows with a padded row stride (PAD complex per row); n must cover Nx*(nt+PAD)
template <int R, int X, int BS, bool NTL, bool NTS, int PAD>
__global__ void __launch_bounds__(BS) k_rowspad(long n, long nt, const v2d *a, const v2d *b, const v2d *c, v2d *o) {
    const long ttiles = nt / BS, ld = nt + PAD;
    const long tt = blockIdx.x % ttiles, xc = blockIdx.x / ttiles;
    long i = xc * X * ld + tt * BS + threadIdx.x;
#pragma unroll 4
    for (int r = 0; r < X; ++r, i += ld) {
        v2d v = ld_<NTL>(a + i);
        if (R > 1) v = v - 0.5 * ld_<NTL>(b + i);
        if (R > 2) v = v + 0.25 * ld_<NTL>(c + i);
        st<NTS>(o + i, v);
    }
}

typedef void (*kfn)(long, long, const v2d *, const v2d *, const v2d *, v2d *);
struct V { std::string name; kfn f; int bs; long blocks; int streams; long elems = 0; };

int main(int argc, char **argv) {
    const long nt = 4096;
    long n = argc > 1 ? atol(argv[1]) : (1L << 24);  // 2^24 complex = 256 MiB/array (4096^2 plane)
    v2d *a, *b, *c, *o;
    CHECK(hipMalloc(&a, n * 16));
    CHECK(hipMalloc(&b, n * 16));
    CHECK(hipMalloc(&c, n * 16));
    CHECK(hipMalloc(&o, n * 16));
    // non-zero, non-uniform data (in case anything compresses)
    {
        std::vector<v2d> h(n);
        for (long i = 0; i < n; ++i) h[i] = v2d{(double)(i * 2654435761u % 1000003) * 1e-3, (double)i};
        CHECK(hipMemcpy(a, h.data(), n * 16, hipMemcpyHostToDevice));
        CHECK(hipMemcpy(b, h.data(), n * 16, hipMemcpyHostToDevice));
        CHECK(hipMemcpy(c, h.data(), n * 16, hipMemcpyHostToDevice));
    }
    std::vector<V> vs;
    char buf[160];
#define ADD(KIND, R, U, BS, NTL, NTS, G)                                                      \
    do {                                                                                    \
        snprintf(buf, sizeof buf, "%s R%d U%d bs%d ntl%d nts%d g%ld", #KIND, R, U, BS, NTL, NTS, (long)(G)); \
        vs.push_back({buf, k_##KIND<R, U, BS, NTL, NTS>, BS, (long)(G), R + 1, 0});            \
    } while (0)
    {
        const long nr = 4032;  // rows for padded variants: 4032*(4096+64) < 2^24
        ADD(oneshot, 2, 1, 256, 1, 1, n / 256);
        ADD(oneshotperm, 2, 1, 256, 1, 1, n / 256);
        ADD(oneshot, 1, 1, 256, 1, 1, n / 256);
        ADD(oneshotperm, 1, 1, 256, 1, 1, n / 256);
        ADD(chunk, 2, 4, 256, 1, 1, 2048);
        ADD(chunkstag, 2, 4, 256, 1, 1, 2048);
        ADD(chunkstag, 2, 4, 256, 1, 1, 4096);
        ADD(chunk, 2, 4, 256, 1, 1, 2000);
        ADD(chunk, 2, 4, 256, 1, 1, 1024);
        ADD(chunkstag, 2, 4, 256, 1, 1, 1024);
        ADD(rows, 2, 32, 256, 1, 1, n / (256 * 32));
        ADD(rows, 2, 8, 256, 1, 1, n / (256 * 8));
        ADD(rows, 2, 1, 256, 1, 1, n / 256);
#define ADDP(R, X, PAD, G)                                                                    \
    do {                                                                                    \
        snprintf(buf, sizeof buf, "rowspad R%d X%d pad%d g%ld", R, X, PAD, (long)(G));        \
        vs.push_back({buf, k_rowspad<R, X, 256, true, true, PAD>, 256, (long)(G), R + 1, nr * 4096}); \
    } while (0)
        ADDP(2, 32, 0, nr / 32 * 16);
        ADDP(2, 32, 16, nr / 32 * 16);
        ADDP(2, 32, 64, nr / 32 * 16);
        ADDP(2, 8, 0, nr / 8 * 16);
        ADDP(2, 8, 16, nr / 8 * 16);
        ADDP(2, 8, 64, nr / 8 * 16);
        ADDP(3, 32, 0, nr / 32 * 16);
        ADDP(3, 32, 64, nr / 32 * 16);
    }
    for (auto &v : vs)
        if (v.name.rfind("chunkstag", 0) == 0 && (n % v.blocks || (n / v.blocks) % 1024)) {
            printf("bad chunkstag grid %s\n", v.name.c_str());
            return 1;
        }
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    const int reps = 20, rounds = 5;
    std::vector<std::vector<float>> t(vs.size());
    for (int r = 0; r < rounds; ++r)
        for (size_t v = 0; v < vs.size(); ++v) {
            hipLaunchKernelGGL(vs[v].f, dim3(vs[v].blocks), dim3(vs[v].bs), 0, 0, n, nt, a, b, c, o);
            CHECK(hipEventRecord(e0));
            for (int k = 0; k < reps; ++k)
                hipLaunchKernelGGL(vs[v].f, dim3(vs[v].blocks), dim3(vs[v].bs), 0, 0, n, nt, a, b, c, o);
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
               16.0 * vs[v].streams * (vs[v].elems ? vs[v].elems : n) / (med * 1e-3) / 1e9);
    }
    return 0;
}
