// membench5.hip -- the Dirac apply's exact load/store pattern without its
// arithmetic, in "sequential front" order (membench3/4: a grid whose blocks
// each take one short tile, dispatched in address order, streams at
// 6.4-6.7 TB/s; long per-block marches cap near 5.5-5.8 TB/s).
//
// Fields are 4096 x 4096 sites, SoA: psi planes p0,p1, links u0 (U_t), u1 (U_x),
// out planes o0,o1 (16 B complex each, row stride 4096, t fastest).
// Per site: psi at (x,t), (x,t+-1), (x+-1,t); U_t(x,t), U_t(x,t-1), U_x(x,t),
// U_x(x-1,t); stores out(x,t). Algorithmic bytes 96/site.
// A block = 256 t-columns x RB rows, tiles ordered t-block fastest so the
// rows x-1, x+1 of a tile are tiles b -+ 16 (the same XCD under round-robin
// dealing when 16 % 8 == 0).
//   hipcc --offload-arch=gfx950 -O3 -o tools/membench5 tools/membench5.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

typedef double v2d __attribute__((ext_vector_type(2)));
template <bool NT>
__device__ __forceinline__ v2d ldg(const v2d *p) {
    if (NT) return __builtin_nontemporal_load(p);
    return *p;
}
__device__ __forceinline__ void stn(v2d *p, v2d v) { __builtin_nontemporal_store(v, p); }

constexpr int NX = 4096, NT = 4096;
constexpr long V = (long)NX * NT;

// F: psi 2 planes at [0,V) [V,2V); U planes same; out same.
// NTU: nt loads on U; RB rows per block; ORDER 0 = t-block fastest (front),
// 1 = scrambled tile order.
template <int RB, bool NTU, bool NTP, int ORDER>
__global__ void __launch_bounds__(256) k_stencil(const v2d *__restrict__ psi, const v2d *__restrict__ U,
                                                 v2d *__restrict__ out) {
    const int TB = NT / 256;
    long b = blockIdx.x;
    if (ORDER == 1) b = (b * 40503L) % gridDim.x;
    const int tb = b % TB, xg = b / TB;
    const int t = tb * 256 + threadIdx.x;
    const int tm = t == 0 ? NT - 1 : t - 1, tp = t == NT - 1 ? 0 : t + 1;
    const int x0 = xg * RB;
    v2d c0[RB + 2], c1[RB + 2], m0[RB], m1[RB], p0[RB], p1[RB], ut[RB], ux[RB + 1], utm[RB];
#pragma unroll
    for (int i = 0; i < RB + 2; ++i) {
        int x = x0 - 1 + i;
        x = x < 0 ? x + NX : (x >= NX ? x - NX : x);
        c0[i] = ldg<NTP>(psi + (long)x * NT + t);
        c1[i] = ldg<NTP>(psi + V + (long)x * NT + t);
    }
    {
        int x = x0 == 0 ? NX - 1 : x0 - 1;
        ux[0] = ldg<NTU>(U + V + (long)x * NT + t);
    }
#pragma unroll
    for (int i = 0; i < RB; ++i) {
        const long r = (long)(x0 + i) * NT;
        m0[i] = ldg<NTP>(psi + r + tm);
        m1[i] = ldg<NTP>(psi + V + r + tm);
        p0[i] = ldg<NTP>(psi + r + tp);
        p1[i] = ldg<NTP>(psi + V + r + tp);
        ut[i] = ldg<NTU>(U + r + t);
        utm[i] = ldg<NTU>(U + r + tm);
        ux[i + 1] = ldg<NTU>(U + V + r + t);
    }
#pragma unroll
    for (int i = 0; i < RB; ++i) {
        const long r = (long)(x0 + i) * NT + t;
        v2d s0 = c0[i + 1] * 0.5 - ut[i] * p0[i] + ux[i + 1] * c0[i + 2] + utm[i] * m0[i] + ux[i] * c0[i];
        v2d s1 = c1[i + 1] * 0.5 - ut[i] * p1[i] + ux[i + 1] * c1[i + 2] + utm[i] * m1[i] + ux[i] * c1[i];
        stn(out + r, s0);
        stn(out + V + r, s1);
    }
}

typedef void (*kfn)(const v2d *, const v2d *, v2d *);
struct Var { std::string name; kfn f; long blocks; };

int main() {
    v2d *psi, *U, *out;
    CHECK(hipMalloc(&psi, 2 * V * 16));
    CHECK(hipMalloc(&U, 2 * V * 16));
    CHECK(hipMalloc(&out, 2 * V * 16));
    {
        std::vector<v2d> h(2 * V);
        for (long i = 0; i < 2 * V; ++i) h[i] = v2d{(double)(i * 2654435761u % 1000003) * 1e-3, (double)(i & 1023)};
        CHECK(hipMemcpy(psi, h.data(), 2 * V * 16, hipMemcpyHostToDevice));
        CHECK(hipMemcpy(U, h.data(), 2 * V * 16, hipMemcpyHostToDevice));
    }
    std::vector<Var> vs;
#define ADD(RB, NTU, NTP, ORD) vs.push_back({"stencil RB" #RB " ntu" #NTU " ntp" #NTP " order" #ORD, k_stencil<RB, NTU, NTP, ORD>, V / (256L * RB)})
    ADD(1, false, false, 0);
    ADD(1, true, false, 0);
    ADD(1, true, true, 0);
    ADD(1, false, false, 1);
    ADD(2, false, false, 0);
    ADD(2, true, false, 0);
    ADD(4, false, false, 0);
    ADD(4, true, false, 0);
    ADD(8, true, false, 0);

    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    const int reps = 20, rounds = 5;
    std::vector<std::vector<float>> tm(vs.size());
    for (int r = 0; r < rounds; ++r)
        for (size_t v = 0; v < vs.size(); ++v) {
            hipLaunchKernelGGL(vs[v].f, dim3(vs[v].blocks), dim3(256), 0, 0, psi, U, out);
            CHECK(hipEventRecord(e0));
            for (int k = 0; k < reps; ++k) hipLaunchKernelGGL(vs[v].f, dim3(vs[v].blocks), dim3(256), 0, 0, psi, U, out);
            CHECK(hipEventRecord(e1));
            CHECK(hipEventSynchronize(e1));
            float ms;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            tm[v].push_back(ms / reps);
        }
    for (size_t v = 0; v < vs.size(); ++v) {
        std::sort(tm[v].begin(), tm[v].end());
        const float med = tm[v][rounds / 2];
        printf("{\"variant\": \"%s\", \"us\": %.1f, \"GBps\": %.1f}\n", vs[v].name.c_str(), med * 1e3,
               96.0 * V / (med * 1e-3) / 1e9);
    }
    return 0;
}
