// sm_peer.hip -- kernels of the device-initiated shard transport (sm_peer.h):
// the scalar all-reduce, generic face exchanges through the receivers'
// mailboxes, the Dirac apply's spin-projected faces stored straight into the
// neighbours' apply slots, and the pieces of a gather to shard 0. The CG
// pass's own faces and sums go through the same region from inside the pass
// (sm_cgra.hip: fsend / fsendh, cg_ticketed_tail's peer all-reduce).
//
// Each kernel that publishes ends with ONE waiting thread (the block that
// takes the last ticket), so a shard waiting for a slower one holds one wave,
// never the chip: the slower shard's kernels still find room when several
// shards share a GPU (the one-GPU tests), and every wait has a time limit.
#include "sm_device.h"
#include "sm_internal.h"
#include "sm_peer.h"

#pragma clang fp contract(off)

namespace sm {

__global__ void peer_allreduce_kernel(double *dev, int n, PeerView v, unsigned long long seq) {
    if (threadIdx.x != 0) return;
    double val[8];
    for (int i = 0; i < n; ++i) val[i] = dev[i];
    peer_allreduce_thread(v, seq, val, n);
    for (int i = 0; i < n; ++i) dev[i] = val[i];
}

void launch_peer_allreduce(hipStream_t s, double *dev, int n, const PeerView &v, unsigned long long seq) {
    hipLaunchKernelGGL(peer_allreduce_kernel, dim3(1), dim3(64), 0, s, dev, n, v, seq);
}

// The last block to arrive publishes this exchange to both neighbours (my
// down neighbour's "from up" flag, my up neighbour's "from down" flag) and
// waits for both of mine.
__device__ __forceinline__ void peer_face_handoff(const PeerView &v, unsigned long long seq, unsigned *tick) {
    __shared__ int last;
    if (!last_block_arrive(tick, gridDim.x, &last)) return;
    if (threadIdx.x == 0) {
        peer_publish(&peer_hdr(v, v.down)->face[1], seq);
        peer_publish(&peer_hdr(v, v.up)->face[0], seq);
        PeerHdr *me = peer_hdr(v, v.me);
        if (peer_wait(&me->face[0], seq, &me->err, v.wait_ticks)) peer_wait(&me->face[1], seq, &me->err, v.wait_ticks);
    }
}

// Generic exchange, step 1: slo[f] (my t = 0 side) into my down neighbour's
// mailbox side 1, shi[f] into my up neighbour's side 0, field after field.
__global__ void __launch_bounds__(256) peer_xin_kernel(PeerXfer x, PeerView v, unsigned long long seq, unsigned *tick) {
    const int slot = (int)(seq & 1);
    double *to_down = reinterpret_cast<double *>(v.base[v.down] + peer_mail_off(v.Nx, slot, 1));
    double *to_up = reinterpret_cast<double *>(v.base[v.up] + peer_mail_off(v.Nx, slot, 0));
    const long tot = (long)x.n * x.cnt;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < tot; i += (long)gridDim.x * blockDim.x) {
        const int f = (int)(i / x.cnt);
        const long k = i - (long)f * x.cnt;
        sys_st(to_down + i, x.slo[f][k]);
        sys_st(to_up + i, x.shi[f][k]);
    }
    peer_face_handoff(v, seq, tick);
}

// Step 2 (after step 1's wait): my mailbox into the caller's receive buffers.
__global__ void __launch_bounds__(256) peer_xout_kernel(PeerXfer x, PeerView v, unsigned long long seq) {
    const int slot = (int)(seq & 1);
    const double *from_down = reinterpret_cast<const double *>(v.base[v.me] + peer_mail_off(v.Nx, slot, 0));
    const double *from_up = reinterpret_cast<const double *>(v.base[v.me] + peer_mail_off(v.Nx, slot, 1));
    const long tot = (long)x.n * x.cnt;
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < tot; i += (long)gridDim.x * blockDim.x) {
        const int f = (int)(i / x.cnt);
        const long k = i - (long)f * x.cnt;
        x.rlo[f][k] = from_down[i];
        x.rhi[f][k] = from_up[i];
    }
}

static int peer_grid(long tot) {
    const long b = (tot + 1023) / 1024;
    return (int)(b < 1 ? 1 : (b > 256 ? 256 : b));
}

void launch_peer_exchange(hipStream_t s, const PeerXfer &x, const PeerView &v, unsigned long long seq,
                          unsigned *tick) {
    const int grid = peer_grid((long)x.n * x.cnt);
    hipLaunchKernelGGL(peer_xin_kernel, dim3(grid), dim3(256), 0, s, x, v, seq, tick);
    hipLaunchKernelGGL(peer_xout_kernel, dim3(grid), dim3(256), 0, s, x, v, seq);
}

// The Dirac apply's spin-projected faces (launch_pack_faces_proj's values,
// proj_face_value) stored straight into the neighbours' apply slot seq % 4:
// side 0 into the down neighbour's hi (its t = Wt), side 1 into the up
// neighbour's lo (its t = -1); then the handoff. The receiver's stencil reads
// its own slot (sm_comm.cpp halo) in the next kernel.
__global__ void __launch_bounds__(256) peer_pack_proj_kernel(int Nx, int Wt, long V, const double2 *f,
                                                             const double2 *U, int kind, PeerView v,
                                                             unsigned long long seq, unsigned *tick) {
    const int slot = (int)(seq & 3);
    double2 *down_hi = reinterpret_cast<double2 *>(v.base[v.down] + peer_apply_off(Nx, slot)) + Nx;
    double2 *up_lo = reinterpret_cast<double2 *>(v.base[v.up] + peer_apply_off(Nx, slot));
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < 2 * Nx) {  // side-major: a wave's 64 rows of one side, 1 KiB of consecutive stores
        const int side = i >= Nx, x = side ? i - Nx : i;
        const long n = (long)x * Wt + (side ? Wt - 1 : 0);
        const double2 val = proj_face_value(kind, side, f[n], f[n + V], U + n);
        sys_st16(sys_rsrc(side ? up_lo : down_hi, 16u * (unsigned)Nx), 16 * x, val);
    }
    peer_face_handoff(v, seq, tick);
}

void launch_peer_pack_proj(hipStream_t s, const Geometry &g, const double2 *field, const double2 *U, int kind,
                           const PeerView &v, unsigned long long seq, unsigned *tick) {
    hipLaunchKernelGGL(peer_pack_proj_kernel, dim3((2 * g.Nx + 255) / 256), dim3(256), 0, s, g.Nx, g.Wt, g.V, field,
                       U, kind, v, seq, tick);
}

// Gather to shard 0, one chunk of one sender: the sender's cnt doubles into
// shard 0's mailbox (then a collective barrier, shard 0 copies them out, and a
// second barrier frees the mailbox; sm_capi.cpp peer_gather_to0).
__global__ void __launch_bounds__(256) peer_put_kernel(const double *src, long cnt, double *dst) {
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < cnt; i += (long)gridDim.x * blockDim.x)
        sys_st(dst + i, src[i]);
}

__global__ void __launch_bounds__(256) peer_get_kernel(const double *src, long cnt, double *dst) {
    for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < cnt; i += (long)gridDim.x * blockDim.x)
        dst[i] = src[i];
}

void launch_peer_put(hipStream_t s, const double *src, long cnt, double *dst_remote) {
    hipLaunchKernelGGL(peer_put_kernel, dim3(peer_grid(cnt)), dim3(256), 0, s, src, cnt, dst_remote);
}

void launch_peer_get(hipStream_t s, const double *src_local, long cnt, double *dst) {
    hipLaunchKernelGGL(peer_get_kernel, dim3(peer_grid(cnt)), dim3(256), 0, s, src_local, cnt, dst);
}

}  // namespace sm
