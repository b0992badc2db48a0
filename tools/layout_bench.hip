// layout_bench.hip -- does interleaving the two spin planes of a field (site-
// major, 32 B per site contiguous) stream faster than the reference's planar
// layout (two planes V sites apart) for the CG pass's access shape?
//
// Each one-wave block owns 64 t-columns (one per lane) and marches `rows`
// x-rows of its chunk, like the recompute-Ad pass (sm_cgra.hip): per row it
// reads NR double2 fields (both planes), one link-code field of doubles (both
// planes) and writes one double2 field (both planes), non-temporal stores.
// planar:      field[p * V + x * Nt + t]            (p = plane)
// interleaved: field[(x * Nt + t) * 2 + p]          (a lane's two planes adjacent)
// The tiles are dealt to XCDs the way the pass deals them (consecutive ids of
// one XCD take t-adjacent tiles of its x-chunks). Median of R runs of K passes.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/layout_bench.hip -o tools/layout_bench
//   tools/layout_bench 4096 64 [NR=2]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                \
    do {                                                                        \
        hipError_t e_ = (x);                                                    \
        if (e_ != hipSuccess) {                                                 \
            printf("%s: %s\n", #x, hipGetErrorString(e_));                      \
            exit(1);                                                            \
        }                                                                       \
    } while (0)

struct Args {
    const double2 *in[3];
    const double *code;
    double2 *out;
    long V;
    int Nx, Nt, rows, nr, tiles_t, ntiles;
};

__device__ inline void st_nt(double2 *p, double2 v) {
    __builtin_nontemporal_store(v.x, &p->x);
    __builtin_nontemporal_store(v.y, &p->y);
}

template <int IL, int NR>
__global__ void __launch_bounds__(64) march(Args a) {
    int w = blockIdx.x;
    {  // XCD-aware: the tiles XCD k receives are a contiguous range
        const int n = a.ntiles, q = n >> 3, rr = n & 7, xcd = w & 7;
        w = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (w >> 3);
    }
    const int tb = w % a.tiles_t, xc = w / a.tiles_t;
    const int t = tb * 64 + threadIdx.x;
    const int x0 = xc * a.rows, xe = min(a.Nx, x0 + a.rows);
    double2 acc = make_double2(0.0, 0.0);
    for (int x = x0; x < xe; ++x) {
        const long n = (long)x * a.Nt + t;
        double2 s = make_double2(0.0, 0.0);
#pragma unroll
        for (int f = 0; f < NR; ++f) {
            double2 p0, p1;
            if (IL) {
                p0 = a.in[f][2 * n];
                p1 = a.in[f][2 * n + 1];
            } else {
                p0 = a.in[f][n];
                p1 = a.in[f][n + a.V];
            }
            s.x += p0.x * p1.y;
            s.y += p0.y - p1.x;
        }
        double c0, c1;
        if (IL) {
            const double2 cc = reinterpret_cast<const double2 *>(a.code)[n];
            c0 = cc.x;
            c1 = cc.y;
        } else {
            c0 = a.code[n];
            c1 = a.code[n + a.V];
        }
        s.x += c0;
        s.y += c1;
        acc.x += s.x;
        if (IL) {
            st_nt(a.out + 2 * n, s);
            st_nt(a.out + 2 * n + 1, acc);
        } else {
            st_nt(a.out + n, s);
            st_nt(a.out + n + a.V, acc);
        }
    }
}

__global__ void fill(long n, double2 *p) {
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
        p[i] = make_double2(1e-3 * (double)(i & 1023), 1.0);
}

int main(int argc, char **argv) {
    const int N = argc > 1 ? atoi(argv[1]) : 4096;
    const int rows = argc > 2 ? atoi(argv[2]) : 64;
    const int nr = argc > 3 ? atoi(argv[3]) : 2;
    const long V = (long)N * N;
    double2 *buf[5];
    for (auto &b : buf) {
        CHECK(hipMalloc(&b, sizeof(double2) * 2 * V));
        hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, 2 * V, b);
    }
    CHECK(hipDeviceSynchronize());
    Args a;
    a.in[0] = buf[0];
    a.in[1] = buf[1];
    a.in[2] = buf[2];
    a.code = reinterpret_cast<const double *>(buf[3]);
    a.out = buf[4];
    a.V = V;
    a.Nx = N;
    a.Nt = N;
    a.rows = rows;
    a.nr = nr;
    a.tiles_t = N / 64;
    a.ntiles = a.tiles_t * ((N + rows - 1) / rows);
    const double bytes = (32.0 * nr + 16.0 + 32.0) * V;
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    for (int round = 0; round < 3; ++round)
        for (int il = 0; il < 2; ++il) {
            auto go = [&] {
                if (il) {
                    if (nr == 2) hipLaunchKernelGGL((march<1, 2>), dim3(a.ntiles), dim3(64), 0, 0, a);
                    else hipLaunchKernelGGL((march<1, 3>), dim3(a.ntiles), dim3(64), 0, 0, a);
                } else {
                    if (nr == 2) hipLaunchKernelGGL((march<0, 2>), dim3(a.ntiles), dim3(64), 0, 0, a);
                    else hipLaunchKernelGGL((march<0, 3>), dim3(a.ntiles), dim3(64), 0, 0, a);
                }
            };
            for (int i = 0; i < 5; ++i) go();
            std::vector<float> v;
            for (int r = 0; r < 7; ++r) {
                CHECK(hipEventRecord(e0, 0));
                for (int i = 0; i < 20; ++i) go();
                CHECK(hipEventRecord(e1, 0));
                CHECK(hipEventSynchronize(e1));
                float ms;
                CHECK(hipEventElapsedTime(&ms, e0, e1));
                v.push_back(ms * 1000.f / 20);
            }
            CHECK(hipGetLastError());
            std::sort(v.begin(), v.end());
            printf("{\"N\": %d, \"rows\": %d, \"reads\": %d, \"layout\": \"%s\", \"round\": %d, \"us\": %.2f, "
                   "\"TBps\": %.3f}\n",
                   N, rows, nr, il ? "interleaved" : "planar", round, v[3], bytes / v[3] / 1e6);
        }
    return 0;
}
