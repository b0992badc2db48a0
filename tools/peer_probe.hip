// peer_probe.hip -- feasibility and latency of a device-initiated shard
// transport on ONE GPU (round 6): two processes on the same device, each
// exporting an uncached region through hipIpcGetMemHandle and opening the
// other's; a one-block kernel per round writes a payload into the peer's
// region with system-scope stores, publishes a sequence flag there, then waits
// (bounded) for the peer's flag in its own region and checks the peer's payload.
// Modes:
//   loop   one process, the peer is itself (what a one-rank loopback pays)
//   ipc    two forked processes (fork before any HIP call)
// Prints one JSON line per process: round-trip us per round, payload errors,
// timeouts. Every wait gives up after ~1 s (wall clock), so every wave exits.
//   hipcc -O3 --offload-arch=gfx950 tools/peer_probe.hip -o tools/peer_probe
//   tools/peer_probe ipc [rounds] [payload_doubles] [uncached 1|0]
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <sys/wait.h>
#include <unistd.h>

#define CK(x)                                                                                     \
    do {                                                                                          \
        hipError_t e_ = (x);                                                                      \
        if (e_ != hipSuccess) {                                                                   \
            printf("{\"rank\": %d, \"error\": \"%s: %s\"}\n", g_rank, #x, hipGetErrorString(e_)); \
            fflush(stdout);                                                                       \
            _exit(2);                                                                             \
        }                                                                                         \
    } while (0)

static int g_rank = 0;

struct Region {  // one rank's receive area
    unsigned long long flag;
    unsigned long long pad[15];
    double data[1];
};

__device__ __forceinline__ void sys_store(double *p, double v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// errs[0] payload mismatches, errs[1] timeouts
__global__ void round_kernel(Region *mine, Region *peer, int n, unsigned long long seq, int rank, int check,
                             unsigned *errs) {
    // 1. payload into the peer's region
    for (int i = threadIdx.x; i < n; i += blockDim.x) sys_store(&peer->data[i], (double)(seq * 8 + rank) + i);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    __shared__ int ok;
    if (threadIdx.x == 0) {
        __hip_atomic_store(&peer->flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        // 2. wait for the peer's flag in my region
        const unsigned long long t0 = wall_clock64();
        int good = 1;
        while (__hip_atomic_load(&mine->flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < seq) {
            __builtin_amdgcn_s_sleep(1);
            if (wall_clock64() - t0 > 100000000ull) {  // 1 s at 100 MHz
                good = 0;
                atomicAdd(&errs[1], 1u);
                break;
            }
        }
        ok = good;
    }
    __syncthreads();
    if (!ok || !check) return;
    const int prank = rank ^ 1;
    unsigned bad = 0;
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        const double v = __hip_atomic_load(&mine->data[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (v != (double)(seq * 8 + prank) + i) ++bad;
    }
    if (bad) atomicAdd(&errs[0], bad);
}

static void run(const char *mode, int rank, int rounds, int n, int uncached, int rfd, int wfd) {
    g_rank = rank;
    CK(hipSetDevice(0));
    const size_t bytes = sizeof(Region) + sizeof(double) * n;
    Region *mine = nullptr, *peer = nullptr;
    if (uncached) CK(hipExtMallocWithFlags((void **)&mine, bytes, hipDeviceMallocUncached));
    else CK(hipMalloc(&mine, bytes));
    CK(hipMemset(mine, 0, bytes));
    CK(hipDeviceSynchronize());
    if (!strcmp(mode, "ipc")) {
        hipIpcMemHandle_t h, ph;
        CK(hipIpcGetMemHandle(&h, mine));
        if (write(wfd, &h, sizeof h) != (ssize_t)sizeof h || read(rfd, &ph, sizeof ph) != (ssize_t)sizeof ph) {
            printf("{\"rank\": %d, \"error\": \"handle pipe\"}\n", rank);
            _exit(2);
        }
        CK(hipIpcOpenMemHandle((void **)&peer, ph, hipIpcMemLazyEnablePeerAccess));
    } else {
        peer = mine;
    }
    unsigned *errs;
    CK(hipMalloc(&errs, 2 * sizeof(unsigned)));
    CK(hipMemset(errs, 0, 2 * sizeof(unsigned)));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    // a barrier round (seq 1), then warmup and the timed rounds
    unsigned long long seq = 1;
    hipLaunchKernelGGL(round_kernel, dim3(1), dim3(256), 0, s, mine, peer, n, seq++, rank, 1, errs);
    CK(hipStreamSynchronize(s));
    for (int i = 0; i < 20; ++i)
        hipLaunchKernelGGL(round_kernel, dim3(1), dim3(256), 0, s, mine, peer, n, seq++, rank, 1, errs);
    CK(hipStreamSynchronize(s));
    const auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < rounds; ++i)
        hipLaunchKernelGGL(round_kernel, dim3(1), dim3(256), 0, s, mine, peer, n, seq++, rank, 1, errs);
    CK(hipStreamSynchronize(s));
    const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    // an empty kernel on the same stream: the launch floor
    const auto t1 = std::chrono::steady_clock::now();
    for (int i = 0; i < rounds; ++i)
        hipLaunchKernelGGL(round_kernel, dim3(1), dim3(256), 0, s, mine, mine, 0, 0ull, rank, 0, errs);
    CK(hipStreamSynchronize(s));
    const double us0 = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t1).count();
    unsigned h_err[2];
    CK(hipMemcpy(h_err, errs, sizeof h_err, hipMemcpyDeviceToHost));
    printf("{\"mode\": \"%s\", \"rank\": %d, \"uncached\": %d, \"payload_doubles\": %d, \"rounds\": %d, "
           "\"us_per_round\": %.2f, \"us_per_empty_kernel\": %.2f, \"payload_errors\": %u, \"timeouts\": %u}\n",
           mode, rank, uncached, n, rounds, us / rounds, us0 / rounds, h_err[0], h_err[1]);
    fflush(stdout);
    if (peer != mine) CK(hipIpcCloseMemHandle(peer));
    CK(hipFree(mine));
}

int main(int argc, char **argv) {
    const char *mode = argc > 1 ? argv[1] : "loop";
    const int rounds = argc > 2 ? atoi(argv[2]) : 2000;
    const int n = argc > 3 ? atoi(argv[3]) : 8192;
    const int uncached = argc > 4 ? atoi(argv[4]) : 1;
    alarm(60);
    if (strcmp(mode, "ipc")) {
        run(mode, 0, rounds, n, uncached, -1, -1);
        return 0;
    }
    int a[2], b[2];  // a: 0 -> 1, b: 1 -> 0
    if (pipe(a) || pipe(b)) return 2;
    const pid_t pid = fork();  // before any HIP call
    if (pid == 0) {
        run(mode, 1, rounds, n, uncached, a[0], b[1]);
        _exit(0);
    }
    run(mode, 0, rounds, n, uncached, b[0], a[1]);
    int st = 0;
    waitpid(pid, &st, 0);
    return WIFEXITED(st) ? WEXITSTATUS(st) : 3;
}
