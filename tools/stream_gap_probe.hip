// stream_gap_probe.hip -- what a cross-stream join costs between two kernels
// of one stream (the RCCL t-shard CG pass's ~12-us gap between interior
// launches), on stand-in kernels that spin for a set time.
//
//   hipcc --offload-arch=gfx950 -O2 tools/stream_gap_probe.hip -o tools/stream_gap_probe
//   tools/stream_gap_probe [passes]
//
// Per pass j the schedules put an "interior" kernel K1 (2048 one-wave blocks,
// 75 us) on the main stream and an "edge" kernel K2 (512 blocks, 45 us) plus an
// "exchange" K3 (8 blocks, 15 us) on a second stream, with the library's event
// pattern or a variant of it. Every block stamps its start / end (100-MHz wall
// clock) with global atomics into one of 64 slots (one address for every block
// serialises ~12 ns per atomic: 2048 blocks would add ~47 us to each launch);
// the gap is min start of K1_{j+1} - max end of K1_j. One JSON line per
// schedule: median gap and median pass time in us.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <algorithm>
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

constexpr int kSlots = 64;

__global__ void spin(unsigned long long ticks, unsigned long long *stamp) {
    const unsigned long long t0 = wall_clock64();
    while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(2);
    if (threadIdx.x == 0) {
        unsigned long long *p = stamp + 2 * (blockIdx.x % kSlots);
        atomicMin(&p[0], t0);
        atomicMax(&p[1], (unsigned long long)wall_clock64());
    }
}

struct Run {
    hipStream_t m, c;
    hipEvent_t evR, evH, evI;
    unsigned long long *st;  // [3 kernels][passes][kSlots][2]
    int P;
    unsigned long long *s(int k, int j) { return st + ((size_t)k * P + j) * 2 * kSlots; }
    void K(int k, int j, hipStream_t s_, hipEvent_t stop = nullptr) {
        static const int grid[3] = {2048, 512, 8};
        static const unsigned long long us[3] = {75, 45, 15};
        if (stop)
            hipExtLaunchKernelGGL(spin, dim3(grid[k]), dim3(64), 0, s_, nullptr, stop, 0, us[k] * 100ull, s(k, j));
        else
            hipLaunchKernelGGL(spin, dim3(grid[k]), dim3(64), 0, s_, us[k] * 100ull, s(k, j));
    }
};

static void report(const char *name, Run &r) {
    std::vector<unsigned long long> h((size_t)3 * r.P * 2 * kSlots);
    CK(hipMemcpy(h.data(), r.st, h.size() * 8, hipMemcpyDeviceToHost));
    auto win = [&](int j, unsigned long long &lo, unsigned long long &hi) {  // K1_j over its slots
        lo = ~0ull;
        hi = 0;
        for (int q = 0; q < kSlots; ++q) {
            const unsigned long long *p = &h[((size_t)j * kSlots + q) * 2];
            lo = std::min(lo, p[0]);
            hi = std::max(hi, p[1]);
        }
    };
    std::vector<double> gap, pass;
    for (int j = 5; j + 1 < r.P; ++j) {  // skip the first passes
        unsigned long long a0, a1, b0, b1;
        win(j, a0, a1);
        win(j + 1, b0, b1);
        gap.push_back(((double)b0 - (double)a1) / 100.0);
        pass.push_back(((double)b0 - (double)a0) / 100.0);
    }
    std::sort(gap.begin(), gap.end());
    std::sort(pass.begin(), pass.end());
    printf("{\"schedule\": \"%s\", \"gap_us_median\": %.2f, \"gap_us_min\": %.2f, \"gap_us_max\": %.2f, "
           "\"pass_us_median\": %.2f}\n",
           name, gap[gap.size() / 2], gap.front(), gap.back(), pass[pass.size() / 2]);
    fflush(stdout);
}

static void reset(Run &r) {
    std::vector<unsigned long long> h((size_t)3 * r.P * 2 * kSlots);
    for (size_t i = 0; i < h.size(); i += 2) {
        h[i] = ~0ull;
        h[i + 1] = 0;
    }
    CK(hipMemcpy(r.st, h.data(), h.size() * 8, hipMemcpyHostToDevice));
    CK(hipDeviceSynchronize());
}

int main(int argc, char **argv) {
    Run r;
    r.P = argc > 1 ? atoi(argv[1]) : 60;
    CK(hipSetDevice(0));
    CK(hipStreamCreateWithFlags(&r.m, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&r.c, hipStreamNonBlocking));
    CK(hipMalloc(&r.st, (size_t)3 * r.P * 2 * kSlots * 8));
    const unsigned evf = hipEventDisableTiming;
    CK(hipEventCreateWithFlags(&r.evR, evf));
    CK(hipEventCreateWithFlags(&r.evH, evf));
    CK(hipEventCreateWithFlags(&r.evI, evf));

    // main stream only: K1 back to back
    reset(r);
    for (int j = 0; j < r.P; ++j) r.K(0, j, r.m);
    CK(hipDeviceSynchronize());
    report("K1 only", r);

    // K1 then a marker (event record) on main, nothing waits
    reset(r);
    for (int j = 0; j < r.P; ++j) {
        r.K(0, j, r.m);
        CK(hipEventRecord(r.evR, r.m));
    }
    CK(hipDeviceSynchronize());
    report("K1 + record", r);

    // K1 then a wait on an event of the other stream, long satisfied
    reset(r);
    CK(hipEventRecord(r.evH, r.c));
    CK(hipDeviceSynchronize());
    for (int j = 0; j < r.P; ++j) {
        r.K(0, j, r.m);
        CK(hipStreamWaitEvent(r.m, r.evH, 0));
    }
    CK(hipDeviceSynchronize());
    report("K1 + wait(satisfied)", r);

    // the library's schedule (sm_capi.cpp cg_ra_pass, pipelined faces):
    // main: record evR, K1, wait evH; comm: wait evR, K2, record evH, K3
    auto lib = [&](int j) {
        CK(hipEventRecord(r.evR, r.m));
        CK(hipStreamWaitEvent(r.c, r.evR, 0));
        r.K(1, j, r.c);
        CK(hipEventRecord(r.evH, r.c));
        r.K(0, j, r.m);
        r.K(2, j, r.c);
        CK(hipStreamWaitEvent(r.m, r.evH, 0));
    };
    reset(r);
    for (int j = 0; j < r.P; ++j) lib(j);
    CK(hipDeviceSynchronize());
    report("library: record evR | K1 | wait evH", r);

    // the fork event recorded right after K1 (before the join's wait)
    reset(r);
    for (int j = 0; j < r.P; ++j) {
        if (j == 0) CK(hipEventRecord(r.evI, r.m));
        CK(hipStreamWaitEvent(r.c, r.evI, 0));
        r.K(1, j, r.c);
        CK(hipEventRecord(r.evH, r.c));
        r.K(0, j, r.m);
        CK(hipEventRecord(r.evI, r.m));
        r.K(2, j, r.c);
        CK(hipStreamWaitEvent(r.m, r.evH, 0));
    }
    CK(hipDeviceSynchronize());
    report("fork after K1: K1 | record evI | wait evH", r);

    // the library's dependencies with the events carried by the kernels
    // themselves (hipExtLaunchKernelGGL stop events): no marker packet
    for (int timing = 0; timing < 2; ++timing) {
        hipEvent_t eI, eH;
        CK(hipEventCreateWithFlags(&eI, timing ? hipEventDefault : hipEventDisableTiming));
        CK(hipEventCreateWithFlags(&eH, timing ? hipEventDefault : hipEventDisableTiming));
        reset(r);
        for (int j = 0; j < r.P; ++j) {
            if (j > 0) CK(hipStreamWaitEvent(r.c, eI, 0));
            r.K(1, j, r.c, eH);
            r.K(0, j, r.m, eI);
            r.K(2, j, r.c);
            CK(hipStreamWaitEvent(r.m, eH, 0));
        }
        CK(hipDeviceSynchronize());
        report(timing ? "kernel stop events (timing events): K1 | wait evH"
                      : "kernel stop events (no timing): K1 | wait evH", r);
        CK(hipEventDestroy(eI));
        CK(hipEventDestroy(eH));
    }

    // the two halves of the library's schedule alone (dependencies
    // incomplete: timing only): the join without the fork, the fork without the join
    reset(r);
    for (int j = 0; j < r.P; ++j) {
        r.K(1, j, r.c);
        CK(hipEventRecord(r.evH, r.c));
        r.K(0, j, r.m);
        r.K(2, j, r.c);
        CK(hipStreamWaitEvent(r.m, r.evH, 0));
    }
    CK(hipDeviceSynchronize());
    report("join only: K1 | wait evH", r);
    reset(r);
    for (int j = 0; j < r.P; ++j) {
        CK(hipEventRecord(r.evR, r.m));
        CK(hipStreamWaitEvent(r.c, r.evR, 0));
        r.K(1, j, r.c);
        r.K(0, j, r.m);
        r.K(2, j, r.c);
    }
    CK(hipDeviceSynchronize());
    report("fork only: record evR | K1", r);

    // the library's schedule captured in a graph (12 passes), replayed
    reset(r);
    {
        const int G = 12;
        hipGraph_t g;
        hipGraphExec_t ge;
        int done = 0;
        while (done + G <= r.P) {
            CK(hipStreamBeginCapture(r.m, hipStreamCaptureModeGlobal));
            for (int j = done; j < done + G; ++j) lib(j);
            CK(hipEventRecord(r.evI, r.c));  // join the second stream back into the capture
            CK(hipStreamWaitEvent(r.m, r.evI, 0));
            CK(hipStreamEndCapture(r.m, &g));
            CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
            CK(hipGraphLaunch(ge, r.m));
            CK(hipStreamSynchronize(r.m));
            CK(hipGraphExecDestroy(ge));
            CK(hipGraphDestroy(g));
            done += G;
        }
        r.P = done;
    }
    CK(hipDeviceSynchronize());
    report("library schedule in a graph (12 passes a launch)", r);
    return 0;
}
