// sm_place.cpp -- placement of the buffers the recompute-Ad CG pass streams
// every iteration, and the placement probe run at context creation.
//
// Host code of libsm_hip.so (sm_capi.cpp owns the context; DESIGN.md §2 has
// the measurements behind both rules).

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <vector>

#include "sm_ctx.h"
#include "sm_internal.h"

using namespace sm;

namespace sm_host {

// Placement of the buffers the CG pass streams every iteration (the three
// direction buffers, x, the link codes). Buffers of 256 MiB and more get an
// allocation of their own of at least 2 GiB (a power of two), requested as
// physically contiguous, of which they use the start. The pass runs at one of
// two speeds depending on where the driver puts them (4096^2: ~456 against
// ~477 us per pass). Round 3 found that >= 2 GiB allocations reach the fast
// state where own-size ones and carved pools do not
// (profiles/r03_v_stride_probe.jsonl, r03_w_padded_alloc_ab.jsonl). Round 4
// (DESIGN §2): it is not address translation (zero UTCL1 misses either way,
// profiles/r04_b_alloc_counters.jsonl); the fast state issues the same reads
// with the same mean residency but keeps 5 % more in flight, with 8.5 %
// fewer DRAM-credit stall cycles (r04_c_alloc_rule_ab.jsonl). Over 60
// contexts on three boxes (tools/alloc_trials.py, r04_e_alloc_trials.jsonl)
// the >= 2 GiB allocations WITH the contiguous flag were the fastest rule on
// every box (2273 / 2172 it/s mean against 2193 / 2135 without the flag);
// own size, own-size physical memory at 2 GiB-aligned addresses, >= 1 GiB
// contiguous and one contiguous pool of exactly the buffers' size never
// reached the fast state.
size_t stream_alloc_bytes(size_t bytes, size_t floor_bytes) {
    if (bytes < (size_t(256) << 20)) return bytes;
    size_t a = floor_bytes;
    while (a < bytes) a <<= 1;
    return a;
}

static hipError_t contiguous_or_plain(void **p, size_t bytes) {
    if (hipExtMallocWithFlags(p, bytes, hipDeviceMallocContiguous) == hipSuccess) return hipSuccess;
    (void)hipGetLastError();  // clear the failed request's error state
    return hipMalloc(p, bytes);
}

// Allocate a streamed CG buffer by the context's placement rule (sm_ctx
// pad_alloc: 5 the default, 0 own size for A/B runs; the other rules measured
// in rounds 3-4 were slower and are gone, DESIGN Appendix A.4).
hipError_t stream_malloc(sm_ctx *c, void **p, size_t bytes) {
    if (bytes < (size_t(256) << 20) || c->pad_alloc == 0) return hipMalloc(p, bytes);
    // a contiguous request falls back to a plain allocation of the same size
    // when the driver cannot find contiguous memory
    return contiguous_or_plain(p, stream_alloc_bytes(bytes));
}

void stream_free(sm_ctx *, void *p) {
    if (p) (void)hipFree(p);
}

// Bytes of the codes of n links (sm_linkcode.h): n doubles (v), n flag words,
// then the packed form's flag bytes (one per site = per two links).
size_t link_code_bytes(long n) { return (sizeof(double) + sizeof(uint16_t)) * (size_t)n + (size_t)(n + 1) / 2; }

// Placement probe (round 5: coordinate descent over the buffers). The CG pass
// runs at one of two speeds (~430-438 against ~455-480 us at 4096^2)
// depending on where the driver physically puts its streamed buffers. Timing
// every set that differs from a base set in ONE buffer (tools/place_buffers,
// profiles/r05_a_place_buffers.jsonl) shows that each of the three direction
// buffers and x can flip the state while the link codes cannot, and that the
// effects do not add (the set of every buffer's best alternative was slower
// than the set of the worst ones on one box): the state belongs to the
// buffers' placement relative to each other. So the probe keeps the set and
// searches one buffer at a time -- x, d1, d0, d2 (F_X, F_D2, F_D, F_R) -- with
// up to place_probe fresh allocations of that buffer (held while it is
// searched, so the allocator cannot hand the same memory back), takes the
// fastest candidate if it beats the current set by more than 1 %, and frees
// the rest before the next buffer; a sweep that improved the pass by > 1 % is
// followed by another (at most 3). One sweep reached 430-439 us in 24 of 24
// trials on one box (r05_b_descent.jsonl) but stayed at 456-460 in 2 of 12 on
// another, where each of those had still moved (r05_l_probe_sweeps.jsonl).
// Each candidate is timed over 42 passes after a 40-pass warm burst (round 6),
// the clock state a solve sustains. Transient memory:
// place_probe allocations of one buffer (3 x 2 GiB at 4096^2), and only while
// 16 GiB stay free besides them; a candidate that cannot be allocated ends
// that buffer's search (not the context). Only where the rule applies (fields
// >= 256 MiB, the recompute-Ad pass with fused multiply-adds; not on
// host-staged contexts, where shard processes share one GPU). The timings run
// on drawn data (a field, its codes, Gaussian CG directions), so the kept
// buffers, U and the codes are zeroed again and the scalars and tickets reset. sm_placement_report returns the pass time of the
// initial set and after each buffer's search, and which buffers moved.
static int g_place_probe = 3;  // candidates per buffer for new contexts (sm_set_placement_probe)

// The streamed buffers in the pass's operand order (d[0..2], x), and the
// order the probe searches them in: entry i is bit i of place_chosen and of
// sm_placement_report's mask, with the name sm_placement_buffer_name(i) gives
// (bench.py reads the names from there). The one table for both.
static const int kOperandField[4] = {F_D, F_D2, F_R, F_X};
struct ProbeBuf {
    int operand;  // index into kOperandField
    const char *name;
};
static const ProbeBuf kProbeOrder[4] = {{3, "x"}, {1, "d1"}, {0, "d0"}, {2, "d2"}};

int placement_probe_default() { return g_place_probe; }

int placement_probe(sm_ctx *c, size_t fb) {
    const int M = c->place_probe;
    c->place_n = 0;
    c->place_chosen = 0;
    if (M < 1 || c->hosted || c->pad_alloc == 0 || fb < (size_t(c->place_min_mib) << 20) || c->cg_fused != 5 ||
        c->racfg.fold < 2)
        return SM_OK;
    const size_t ub = link_code_bytes(2 * c->g.V);
    // the link codes are the pass's fifth stream: allocated here so the probe
    // times the real pass (their placement does not move the state)
    if (!c->Uang) HIP_TRY(stream_malloc(c, (void **)&c->Uang, ub));
    Geometry g = c->g;
    g.t0 = 0;
    g.Ntg = g.Wt;  // one shard's pass over this shard's streams
    // The pass is timed on REAL data (round 6): a config-3-like field drawn
    // into the context's U (the caller's upload replaces it) and its packed
    // codes, and a CG started from complex-Gaussian directions and x, redrawn
    // before every set is timed. Round 5 timed zero / NaN data, whose lower
    // switching power let the capped board clock higher: the kept set's time
    // came out 2-3 % below the pass time the bench then sustained.
    launch_draw_gauge(c->own_stream, g, 0x9a1ce5eedull, 0.2374, c->U);
    (void)launch_link_codes(c->own_stream, 2 * c->g.V, c->U, c->Uang, c->partials);
    launch_link_nibbles(c->own_stream, c->g.V, c->Uang);
    void *cur[4];  // by operand
    for (int i = 0; i < 4; ++i) cur[i] = c->fields[kOperandField[i]];
    CGScalars *h = (CGScalars *)c->h_sc;
    memset(h, 0, sizeof(CGScalars));
    h->max_iter = 1 << 30;
    h->phi_norm = 1.0;
    const int nparts = cg_fused_blocks(c->racfg);
    const bool tail = (nparts + 63) / 64 <= kMaxTickGroups;
    hipEvent_t ev[2] = {nullptr, nullptr};
    auto drop_events = [&] {
        for (hipEvent_t e : ev)
            if (e) (void)hipEventDestroy(e);
    };
    if (hipEventCreate(&ev[0]) != hipSuccess || hipEventCreate(&ev[1]) != hipSuccess) {
        drop_events();
        return fail(SM_ERR_HIP, "placement probe: events");
    }
    long j = 2;
    // a fresh CG state on the set: d_{j-1}, d_{j-2}, d_j's buffer and x
    // Gaussian, zero scalars (pass j = 2 then runs r = d_{j-1}: a CG step)
    auto fresh = [&](void *const *f) -> int {
        for (int i = 0; i < 4; ++i) launch_draw_source(c->own_stream, g, 0x5eed0000ull + i, (double2 *)f[i]);
        if (hipMemcpyAsync(c->sc, h, sizeof(CGScalars), hipMemcpyHostToDevice, c->own_stream) != hipSuccess)
            return fail(SM_ERR_HIP, "placement probe: scalars");
        j = 2;
        return SM_OK;
    };
    // median us per pass of 3 rounds of 14 passes (one warm-up round first),
    // so every candidate is timed over 42 passes in the clock state of a
    // sustained solve (timed over 6-pass rounds, the kept
    // set's time was the burst clock's, 1.9-3 % below what the bench then
    // sustained); `burst` passes first warm the chip up to that state
    auto time_set = [&](void *const *f, double *us, int burst) -> int {
        constexpr int kRounds = 3, kPasses = 14;
        float t[kRounds];
        if (int rc = fresh(f); rc != SM_OK) return rc;
        for (int r = -1 - (burst > 0); r < kRounds; ++r) {
            double2 *d[3] = {(double2 *)f[0], (double2 *)f[1], (double2 *)f[2]};
            if (hipEventRecord(ev[0], c->own_stream) != hipSuccess) return fail(SM_ERR_HIP, "placement probe");
            const int np = r == -2 ? burst : kPasses;
            for (int p = 0; p < np; ++p, ++j)
                launch_cg_ra(c->own_stream, g, c->racfg, 1, d[(j + 2) % 3], d[(j + 1) % 3], d[j % 3], (double2 *)f[3],
                             nullptr, nullptr, nullptr, nullptr, 1.94, j, c->sc, c->partials, 0, c->racfg.TBk,
                             nullptr, c->Uang, nullptr, nullptr, 0, tail ? c->tick : nullptr, nparts, c->gsum,
                             nullptr, 0, 2);  // the packed flags: what fresh fields take
            float ms = 0.f;
            if (hipEventRecord(ev[1], c->own_stream) != hipSuccess || hipEventSynchronize(ev[1]) != hipSuccess ||
                hipEventElapsedTime(&ms, ev[0], ev[1]) != hipSuccess || hipGetLastError() != hipSuccess)
                return fail(SM_ERR_HIP, "placement probe timing");
            if (r >= 0) t[r] = ms * 1000.f / np;
        }
        std::sort(t, t + kRounds);
        *us = t[kRounds / 2];
        return SM_OK;
    };
    double now = 0.0;
    int rc = time_set(cur, &now, 40);
    c->place_us[c->place_n++] = now;
    const size_t bytes = stream_alloc_bytes(fb);
    // sweeps over the four buffers, another one while the last improved the
    // pass by > 1 % (at most kSweeps): a sweep that ends still slow has usually
    // moved, and the next one starts from there (profiles/r05_l_probe_sweeps.jsonl)
    constexpr int kSweeps = 3;
    double sweep_start = now;
    for (int step = 0; step < 4 * kSweeps && rc == SM_OK; ++step) {
        if (step > 0 && step % 4 == 0) {
            if (!(now < 0.99 * sweep_start)) break;
            sweep_start = now;
        }
        const int b = kProbeOrder[step % 4].operand;
        std::vector<void *> cand;
        int keep = -1;
        double best = now;
        for (int m = 0; m < M && rc == SM_OK; ++m) {
            size_t free_b = 0, total_b = 0;
            if (hipMemGetInfo(&free_b, &total_b) != hipSuccess || free_b < bytes + (size_t(16) << 30)) break;
            void *p = nullptr;
            if (stream_malloc(c, &p, fb) != hipSuccess) {
                (void)hipGetLastError();  // not fatal: this buffer's search ends
                break;
            }
            cand.push_back(p);
            void *trial[4] = {cur[0], cur[1], cur[2], cur[3]};
            trial[b] = p;
            double us = 0.0;
            rc = time_set(trial, &us, 0);
            if (rc == SM_OK && us < best) best = us, keep = (int)cand.size() - 1;
        }
        if (rc == SM_OK && keep >= 0 && best < 0.99 * now) {
            stream_free(c, cur[b]);
            cur[b] = cand[keep];
            c->fields[kOperandField[b]] = (double2 *)cur[b];
            now = best;
            c->place_chosen |= 1 << (step % 4);
        }
        for (void *p : cand)
            if (p != cur[b]) stream_free(c, p);
        c->place_us[c->place_n++] = now;
    }
    drop_events();
    if (rc != SM_OK) return rc;
    // clear the probe's iterates, field and codes, as fresh allocations would be
    // (pass 0 weights d_{-2} by a zero multiplier; the caller uploads U)
    for (void *p : cur) HIP_TRY(hipMemsetAsync(p, 0, fb, c->own_stream));
    HIP_TRY(hipMemsetAsync(c->Uang, 0, ub, c->own_stream));
    HIP_TRY(hipMemsetAsync(c->U, 0, sizeof(double2) * 2 * (size_t)c->g.V, c->own_stream));
    HIP_TRY(hipMemsetAsync(c->sc, 0, sizeof(CGScalars), c->own_stream));
    HIP_TRY(hipMemsetAsync(c->tick, 0, sizeof(unsigned) * (1 + kMaxTickGroups), c->own_stream));
    HIP_TRY(hipStreamSynchronize(c->own_stream));
    return SM_OK;
}

}  // namespace sm_host

using namespace sm_host;

extern "C" {

int sm_set_placement_probe(int candidates_per_buffer) {
    if (candidates_per_buffer < 0 || candidates_per_buffer > 8)
        return fail(SM_ERR_ARG, "placement probe candidates must be 0..8");
    g_place_probe = candidates_per_buffer;
    return SM_OK;
}

int sm_get_placement_probe(void) { return g_place_probe; }

const char *sm_placement_buffer_name(int i) { return i >= 0 && i < 4 ? kProbeOrder[i].name : nullptr; }

int sm_placement_report(const sm_ctx *c, double *us_per_pass, int *n, int *chosen) {
    if (!c || !n || !chosen) return fail(SM_ERR_ARG, "null argument");
    *n = c->place_n;
    *chosen = c->place_chosen;  // bit i: kProbeOrder[i] moved
    if (us_per_pass)
        for (int k = 0; k < c->place_n; ++k) us_per_pass[k] = c->place_us[k];
    return SM_OK;
}

}  // extern "C"
