// sm_peer.h -- the device-initiated shard transport (round 6, "peer").
//
// Every shard owns ONE region of uncached device memory (hipDeviceMallocUncached,
// so no L2 keeps a stale copy of what another device writes into it), exported
// with hipIpcGetMemHandle and opened by every other shard of the job. A shard
// sends by storing into the receiver's region with system-scope write-through
// stores and then publishing a sequence number there; the receiver waits for
// that number in its own region. No RCCL kernel, no proxy thread, no host step:
// one t-shard exchange or all-reduce is a few stores over xGMI plus a flag.
//
// Region layout (byte offsets from the region base; Nx rows):
//   PeerHdr                         flags and the all-reduce slots (4 KiB)
//   ring[3]    16 Nx complex each   the recompute-Ad CG pass's 4-deep faces of d_j,
//                                   slot j % 3, [col -4..-1, Wt..Wt+3][plane][x],
//                                   written by the neighbours' pass j itself
//   apply[4]   2 Nx complex each    spin-projected apply / force faces, slot seq % 4:
//                                   lo (t = -1) at +0, hi (t = Wt) at +Nx
//   mail[2][2] kMailDoubles Nx doubles each   generic face exchanges, slot seq % 2,
//                                   side 0 from the down neighbour, 1 from the up one
//
// Sequence numbers: the host keeps two counters per context (collectives,
// face exchanges) and every shard issues the same operations in the same
// order, so the n-th operation of a kind carries the same number everywhere.
// Flags only grow; a wait is `flag >= seq`. Every wait gives up after
// kPeerWaitTicks of the 100-MHz wall clock and records the timeout in the
// header's err word (sm_peer_status / sm_cg_finish report it), so every wave
// of every kernel exits.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sm {

constexpr int kPeerMaxRanks = 16;
constexpr long kPeerHdrBytes = 4096;
constexpr long kMailDoubles = 48;  // per x and side: up to 3 fields x 16 doubles (a 4-deep face)
constexpr unsigned long long kPeerWaitTicks = 1000000000ull;  // 10 s at 100 MHz (PeerView::wait_ticks default)

struct PeerHdr {
    unsigned long long coll[kPeerMaxRanks];  // all-reduce seq published by rank r
    unsigned long long face[2];              // exchange seq published by my down (0) / up (1) neighbour
    unsigned long long err;                  // set by MY kernels: a wait timed out (the seq waited for)
    unsigned long long pad[13];
    double gather[2][kPeerMaxRanks][8];      // all-reduce payloads by seq parity, [sender][value]
};
static_assert(sizeof(PeerHdr) <= kPeerHdrBytes, "peer header");

// Every shard's region base (this shard's own at base[me]), as the kernels see them.
struct PeerView {
    char *base[kPeerMaxRanks];
    int me, n, down, up;
    long Nx;
    unsigned long long wait_ticks;  // time limit of one wait (100-MHz ticks; kPeerWaitTicks unless a test sets it)
};

__host__ __device__ inline long peer_ring_off(long Nx, int slot) { return kPeerHdrBytes + (long)slot * 16 * Nx * 16; }
__host__ __device__ inline long peer_apply_off(long Nx, int slot) {
    return kPeerHdrBytes + 48 * Nx * 16 + (long)slot * 2 * Nx * 16;
}
__host__ __device__ inline long peer_mail_off(long Nx, int slot, int side) {
    return kPeerHdrBytes + 56 * Nx * 16 + (long)(2 * slot + side) * kMailDoubles * Nx * 8;
}
__host__ __device__ inline long peer_region_bytes(long Nx) { return peer_mail_off(Nx, 2, 0); }

#if defined(__HIPCC__)
__device__ __forceinline__ PeerHdr *peer_hdr(const PeerView &v, int r) { return reinterpret_cast<PeerHdr *>(v.base[r]); }

// Write-through system-scope stores: the store's completion (vmcnt) means the
// value has left this device's caches for the receiver's memory.
__device__ __forceinline__ void sys_st(double *p, double v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
// 16-byte write-through store at system scope (buffer_store_dwordx4 ... sc0
// sc1) at byte offset `off` of a raw buffer resource: the face payloads, one
// coalesced 16-B element per lane (a wave covers 1 KiB of consecutive rows).
typedef unsigned int sm_v4u __attribute__((ext_vector_type(4)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t sys_rsrc(void *base, unsigned bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(base, 0, (int)bytes, 0x00020000);  // gfx9 raw-buffer dword3
}
__device__ __forceinline__ void sys_st16(__amdgpu_buffer_rsrc_t r, int off, double2 v) {
    sm_v4u w;
    __builtin_memcpy(&w, &v, 16);
    __builtin_amdgcn_raw_buffer_store_b128(w, r, off, 0, 17);  // cache policy SC0 | SC1
}
__device__ __forceinline__ double sys_ld(const double *p) {
    return __hip_atomic_load(const_cast<double *>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
// Publish a sequence number: every store this thread's wave issued before is
// complete first (gfx9: vmcnt counts stores, and the payload went out as
// write-through system-scope stores), then the flag, itself a write-through
// store. No release fence: on gfx950 that writes back the XCD's whole dirty
// L2 (the CG pass's d_j and x lines), which the payload does not need (the
// same reasoning as sm_device.h's publish_partial, one scope wider).
__device__ __forceinline__ void peer_publish(unsigned long long *flag, unsigned long long seq) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_store(flag, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
// Wait (one thread) until *flag >= seq; false (and err recorded) after the
// time limit. The polls are system-scope loads (they bypass this device's
// caches); what the sender published is read afterwards with sys_ld, or by a
// later kernel from this region's uncached memory. Once a wait of this shard
// has timed out (err set), every later wait gives up at once: the results are
// already void, and the caller reaches sm_peer_status / sm_cg_finish's error
// after one time limit, not one per pass.
__device__ __forceinline__ bool peer_wait(unsigned long long *flag, unsigned long long seq, unsigned long long *err,
                                          unsigned long long limit) {
    if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) return false;
    const unsigned long long t0 = wall_clock64();
    while (__hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < seq) {
        __builtin_amdgcn_s_sleep(1);
        if (wall_clock64() - t0 > limit) {
            __hip_atomic_store(err, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            return false;
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no later load is issued before the poll that passed
    return true;
}

// All-reduce of n <= 8 doubles by ONE thread: my values into every shard's
// gather slot, my flag into every shard's header, wait for every shard's flag
// in mine, then the sum in rank order (rank 0's value, + rank 1's, ...), the
// same bits on every shard and the same order as the host-staged transport.
__device__ __forceinline__ void peer_allreduce_thread(const PeerView &v, unsigned long long seq, double *val, int n) {
    const int slot = (int)(seq & 1);
    for (int r = 0; r < v.n; ++r) {
        double *g = peer_hdr(v, r)->gather[slot][v.me];
        for (int i = 0; i < n; ++i) sys_st(g + i, val[i]);
    }
    for (int r = 0; r < v.n; ++r) peer_publish(&peer_hdr(v, r)->coll[v.me], seq);
    PeerHdr *mine = peer_hdr(v, v.me);
    for (int r = 0; r < v.n; ++r)
        if (!peer_wait(&mine->coll[r], seq, &mine->err, v.wait_ticks)) break;
    for (int i = 0; i < n; ++i) {
        double acc = sys_ld(&mine->gather[slot][0][i]);
        for (int r = 1; r < v.n; ++r) acc = acc + sys_ld(&mine->gather[slot][r][i]);
        val[i] = acc;
    }
}
#endif

}  // namespace sm
