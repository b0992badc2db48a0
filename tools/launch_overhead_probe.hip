// launch_overhead_probe.hip -- how long a kernel occupies its queue beyond its
// blocks' own run time (stream_gap_probe found 2048 one-wave blocks spinning
// 75 us take 122 us in rocprof), against the grid size and block size.
//
//   hipcc --offload-arch=gfx950 -O2 tools/launch_overhead_probe.hip -o tools/launch_overhead_probe
//
// Each launch: every block spins `us` on the 100-MHz wall clock and stamps its
// start / end (global atomics). HIP events around 20 back-to-back launches give
// the queue time per launch; the stamps give the blocks' window. One JSON line
// per (grid, block): ms per launch (events), the blocks' window (stamps).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                           \
        }                                                                                      \
    } while (0)

__global__ void spin(unsigned long long ticks, unsigned long long *stamp) {
    const unsigned long long t0 = wall_clock64();
    while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(2);
    if (threadIdx.x == 0) {
        atomicMin(&stamp[0], t0);
        atomicMax(&stamp[1], (unsigned long long)wall_clock64());
    }
}

__global__ void empty_kernel(int *p) {
    if (p && threadIdx.x == 1023) p[0] = 1;
}

int main() {
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    unsigned long long *st;
    const int N = 20;
    CK(hipMalloc(&st, N * 2 * 8));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    const int grids[] = {1, 64, 256, 1024, 2048, 4096, 8192};
    const int blocks[] = {64, 256};
    const int uss[] = {0, 20, 75};
    for (int us : uss)
        for (int bs : blocks)
            for (int g : grids) {
                if (bs == 256 && g > 2048) continue;
                std::vector<unsigned long long> h(N * 2);
                for (int i = 0; i < N; ++i) {
                    h[2 * i] = ~0ull;
                    h[2 * i + 1] = 0;
                }
                CK(hipMemcpy(st, h.data(), h.size() * 8, hipMemcpyHostToDevice));
                for (int w = 0; w < 3; ++w)
                    hipLaunchKernelGGL(spin, dim3(g), dim3(bs), 0, s, (unsigned long long)us * 100ull, st);
                CK(hipMemcpy(st, h.data(), h.size() * 8, hipMemcpyHostToDevice));
                CK(hipDeviceSynchronize());
                CK(hipEventRecord(a, s));
                for (int i = 0; i < N; ++i)
                    hipLaunchKernelGGL(spin, dim3(g), dim3(bs), 0, s, (unsigned long long)us * 100ull, st + 2 * i);
                CK(hipEventRecord(b, s));
                CK(hipEventSynchronize(b));
                float ms = 0;
                CK(hipEventElapsedTime(&ms, a, b));
                CK(hipMemcpy(h.data(), st, h.size() * 8, hipMemcpyDeviceToHost));
                double win = 0, period = 0;
                for (int i = 0; i < N; ++i) win += (double)(h[2 * i + 1] - h[2 * i]) / 100.0;
                for (int i = 1; i < N; ++i) period += (double)(h[2 * i] - h[2 * i - 2]) / 100.0;
                printf("{\"spin_us\": %d, \"block\": %d, \"grid\": %d, \"us_per_launch_events\": %.2f, "
                       "\"blocks_window_us\": %.2f, \"start_to_start_us\": %.2f}\n",
                       us, bs, g, 1000.0 * ms / N, win / N, period / (N - 1));
                fflush(stdout);
            }
    // an empty kernel, 2048 x 64
    CK(hipEventRecord(a, s));
    for (int i = 0; i < 100; ++i) hipLaunchKernelGGL(empty_kernel, dim3(2048), dim3(64), 0, s, nullptr);
    CK(hipEventRecord(b, s));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    printf("{\"empty_kernel\": \"2048x64\", \"us_per_launch_events\": %.2f}\n", 1000.0 * ms / 100);
    return 0;
}
