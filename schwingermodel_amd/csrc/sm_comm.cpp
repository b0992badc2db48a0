// sm_comm.cpp -- the t-shard transports of libsm_hip.so (host side): RCCL
// (one communicator, operations in one total order), the host-staged
// transport (a caller's exchange / all-reduce callbacks) and the
// device-initiated peer transport (sm_peer.h, kernels in sm_peer.hip); the
// face exchanges and all-reduces every operator and CG path goes through,
// the halos of the Dirac apply (spin-projected), of the fused CG kernel
// (2-deep) and of the recompute-Ad pass (4-deep), the ghost links, and the
// setup of the peer regions and of the RCCL path's in-pass CG sums.
// (Split out of sm_capi.cpp, which keeps the context and the C-ABI entry
// points of the operators and the CG driver.)

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstddef>
#include <cstring>
#include <functional>
#include <vector>

#include "sm_fields.h"
#include "sm_ctx.h"
#include "sm_internal.h"

using namespace sm;
using namespace sm_host;

namespace sm_host {

int up_rank(const sm_ctx *c) { return (c->shard + 1) % c->nshard; }
int down_rank(const sm_ctx *c) { return (c->shard - 1 + c->nshard) % c->nshard; }

// Exchange the t-faces of `field` (both planes) with the t-1 / t+1 shards.
// My t = Wt-1 column goes up (it is the up-neighbour's t = -1), my t = 0
// column goes down (the down-neighbour's t = Wt). The face buffers are
// [plane][x], 4*Nx doubles.

// One communicator, RCCL operations in one total order.
// Every RCCL operation of a context -- face exchanges, scalar all-reduces, the
// gauge gather -- goes through the context's single communicator, and each
// one is ordered on the GPU after the one issued before it, so no two RCCL
// kernels of a context are ever in flight at once and nothing relies on two
// communicators' kernels being co-resident (round 5 split a second
// communicator off for the comm stream and argued that they always were).
// The operations still run on the stream whose work they belong to (the main
// stream, or the comm stream for the faces that travel under an interior
// launch): rccl_order makes an operation on stream s wait for the previous
// RCCL operation when that one ran on the other stream, by an event recorded
// there at issue time. Streams that already joined by the launch schedule's
// own events (rccl_joined) need no extra event. Measured on the RCCL loopback
// (profiles/r06_b_rccl_stream.jsonl): issuing every operation on ONE
// stream instead costs 15-31 us per CG iteration at 4096 x 512 .. 2048 (two
// ~10-us cross-stream hops per pass on the critical path, or the face
// exchange serialised behind the interior launch).
static int rccl_order(sm_ctx *c, hipStream_t s) {
    if (c->rccl_last && c->rccl_last != s && c->rccl_ordered) {
        // recorded now: the other stream's work so far ends with its last RCCL
        // operation wherever a schedule issues RCCL there last (the CG pass's
        // pipelined faces, the apply's overlapped faces)
        HIP_TRY(hipEventRecord(c->ev_rccl, c->rccl_last));
        HIP_TRY(hipStreamWaitEvent(s, c->ev_rccl, 0));
    }
    c->rccl_last = s;
    return SM_OK;
}

// `waiter` has just waited for an event recorded on `signaler` after its last
// RCCL operation: later operations on `waiter` are ordered after it already.
void rccl_joined(sm_ctx *c, hipStream_t waiter, hipStream_t signaler) {
    if (c->rccl_last == signaler) c->rccl_last = waiter;
}

int rccl_p2p_group(sm_ctx *c, hipStream_t s, int n, const double2 *const *send_up, double2 *const *recv_down,
                   const double2 *const *send_down, double2 *const *recv_up, size_t cnt) {
    TRY(rccl_order(c, s));
    NCCL_TRY(ncclGroupStart());
    for (int i = 0; i < n; ++i) {
        NCCL_TRY(ncclSend(send_up[i], cnt, ncclDouble, up_rank(c), c->comm, s));
        NCCL_TRY(ncclRecv(recv_down[i], cnt, ncclDouble, down_rank(c), c->comm, s));
        NCCL_TRY(ncclSend(send_down[i], cnt, ncclDouble, down_rank(c), c->comm, s));
        NCCL_TRY(ncclRecv(recv_up[i], cnt, ncclDouble, up_rank(c), c->comm, s));
    }
    NCCL_TRY(ncclGroupEnd());
    return SM_OK;
}

// ---- device-initiated transport (sm_peer.h, sm_peer.hip) ----
int peer_ready(const sm_ctx *c) {
    if (!c->peer_connected) return fail(SM_ERR_STATE, "peer transport: sm_peer_connect has not run on this context");
    return SM_OK;
}

// n (<= 3) exchanges through the receivers' mailboxes (generic faces)
static int peer_exchange(sm_ctx *c, hipStream_t s, int n, const double2 *const *slo, const double2 *const *shi,
                         double2 *const *rlo, double2 *const *rhi, size_t cnt) {
    TRY(peer_ready(c));
    if (n < 1 || n > 3 || (long)n * (long)cnt > kMailDoubles * (long)c->g.Nx)
        return fail(SM_ERR_ARG, "peer exchange of %d x %zu doubles exceeds the mailbox", n, cnt);
    PeerXfer x{};
    for (int i = 0; i < n; ++i) {
        x.slo[i] = (const double *)slo[i];
        x.shi[i] = (const double *)shi[i];
        x.rlo[i] = (double *)rlo[i];
        x.rhi[i] = (double *)rhi[i];
    }
    x.n = n;
    x.cnt = (long)cnt;
    launch_peer_exchange(s, x, c->peer_view, ++c->peer_face_seq, c->peer_tick);
    return SM_OK;
}

// Gather to shard 0 through its mailbox (cold path: the gauge field for a conf
// file): a barrier so no earlier exchange still needs shard 0's mailbox, then
// per sender and chunk: put, barrier, shard 0 copies out, barrier.
static int peer_gather_to0(sm_ctx *c, hipStream_t s, const double *send, double *recv, size_t cnt) {
    TRY(peer_ready(c));
    const long cap = 4 * kMailDoubles * (long)c->g.Nx;  // shard 0's four mailbox slots, contiguous
    double *mail0 = (double *)(c->peer_view.base[0] + peer_mail_off(c->g.Nx, 0, 0));
    double *scratch = (double *)(c->sums + 3);
    auto barrier = [&] { launch_peer_allreduce(s, scratch, 0, c->peer_view, ++c->peer_coll_seq); };
    if (c->shard == 0 && cnt) HIP_TRY(hipMemcpyAsync(recv, send, cnt * sizeof(double), hipMemcpyDeviceToDevice, s));
    barrier();
    for (int r = 1; r < c->nshard; ++r)
        for (size_t off = 0; off < cnt; off += (size_t)cap) {
            const long len = (long)std::min(cnt - off, (size_t)cap);
            if (c->shard == r) launch_peer_put(s, send + off, len, mail0);
            barrier();
            if (c->shard == 0) launch_peer_get(s, mail0, len, recv + (size_t)r * cnt + off);
            barrier();
        }
    HIP_TRY(hipGetLastError());
    return SM_OK;
}

int rccl_gather_to0(sm_ctx *c, hipStream_t s, const double *send, double *recv, size_t cnt) {
    if (c->peer) return peer_gather_to0(c, s, send, recv, cnt);
    TRY(rccl_order(c, s));
    NCCL_TRY(ncclGroupStart());
    if (c->shard == 0) {
        for (int r = 1; r < c->nshard; r++) NCCL_TRY(ncclRecv(recv + (size_t)r * cnt, cnt, ncclDouble, r, c->comm, s));
    } else {
        NCCL_TRY(ncclSend(send, cnt, ncclDouble, 0, c->comm, s));
    }
    NCCL_TRY(ncclGroupEnd());
    return SM_OK;
}

int exchange_faces_on(sm_ctx *c, hipStream_t s, double2 *slo, double2 *shi, double2 *rlo, double2 *rhi,
                      size_t cnt) {
    if (cnt > kMaxFaceDoubles * (size_t)c->g.Nx) return fail(SM_ERR_ARG, "face too large (%zu)", cnt);
    if (c->hosted) {
        double *h = c->h_face;
        HIP_TRY(hipMemcpyAsync(h, slo, cnt * 8, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipMemcpyAsync(h + cnt, shi, cnt * 8, hipMemcpyDeviceToHost, s));
        HIP_TRY(hipStreamSynchronize(s));
        if (c->tr.exchange(c->tr.user, h, h + cnt, h + 2 * cnt, h + 3 * cnt, (long)cnt) != 0)
            return fail(SM_ERR_ARG, "host transport exchange failed");
        HIP_TRY(hipMemcpyAsync(rlo, h + 2 * cnt, cnt * 8, hipMemcpyHostToDevice, s));
        HIP_TRY(hipMemcpyAsync(rhi, h + 3 * cnt, cnt * 8, hipMemcpyHostToDevice, s));
        HIP_TRY(hipStreamSynchronize(s));  // staging buffers are reused
        return SM_OK;
    }
    if (c->peer) {
        const double2 *sl[1] = {slo}, *sh[1] = {shi};
        double2 *rl[1] = {rlo}, *rh[1] = {rhi};
        return peer_exchange(c, s, 1, sl, sh, rl, rh, cnt);
    }
    const double2 *su[1] = {shi}, *sd[1] = {slo};
    double2 *rd[1] = {rlo}, *ru[1] = {rhi};
    return rccl_p2p_group(c, s, 1, su, rd, sd, ru, cnt);
}

int exchange_faces_multi(sm_ctx *c, hipStream_t s, int n, double2 *const *slo, double2 *const *shi,
                         double2 *const *rlo, double2 *const *rhi, size_t cnt) {
    if (c->hosted) {
        for (int i = 0; i < n; ++i) TRY(exchange_faces_on(c, s, slo[i], shi[i], rlo[i], rhi[i], cnt));
        return SM_OK;
    }
    if (cnt > kMaxFaceDoubles * (size_t)c->g.Nx) return fail(SM_ERR_ARG, "face too large (%zu)", cnt);
    if (c->peer) return peer_exchange(c, s, n, slo, shi, rlo, rhi, cnt);
    return rccl_p2p_group(c, s, n, shi, rlo, slo, rhi, cnt);
}

int exchange_faces(sm_ctx *c, double2 *slo, double2 *shi, double2 *rlo, double2 *rhi, size_t cnt) {
    return exchange_faces_on(c, c->stream, slo, shi, rlo, rhi, cnt);
}

// In-place global sum of n doubles resident on the device.
int allreduce_dev(sm_ctx *c, double *dev, int n) {
    if (!c->sharded()) return SM_OK;
    if (c->hosted) {
        HIP_TRY(hipMemcpyAsync(c->h_red, dev, sizeof(double) * n, hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(hipStreamSynchronize(c->stream));
        if (c->tr.allreduce_sum(c->tr.user, c->h_red, n) != 0)
            return fail(SM_ERR_ARG, "host transport allreduce failed");
        HIP_TRY(hipMemcpyAsync(dev, c->h_red, sizeof(double) * n, hipMemcpyHostToDevice, c->stream));
        HIP_TRY(hipStreamSynchronize(c->stream));
        return SM_OK;
    }
    if (c->peer) {
        TRY(peer_ready(c));
        if (n > 8) return fail(SM_ERR_ARG, "peer all-reduce of %d doubles (at most 8)", n);
        launch_peer_allreduce(c->stream, dev, n, c->peer_view, ++c->peer_coll_seq);
        return SM_OK;
    }
    TRY(rccl_order(c, c->stream));
    NCCL_TRY(ncclAllReduce(dev, dev, n, ncclDouble, ncclSum, c->comm, c->stream));
    return SM_OK;
}

// 1-deep t-faces of `field` for the operator `kind` (FaceKind): spin-projected,
// one complex per x and side (2 Nx doubles per message instead of 4 Nx).
int halo(sm_ctx *c, const double2 *field, int set, int kind, TFaces *f) {
    if (!c->sharded()) {
        *f = faces_for(c, field, nullptr, nullptr);
        return SM_OK;
    }
    if (c->peer) {  // packed straight into the neighbours' apply slots (sm_peer.hip)
        TRY(peer_ready(c));
        const unsigned long long seq = ++c->peer_face_seq;
        launch_peer_pack_proj(c->stream, c->g, field, c->U, kind, c->peer_view, seq, c->peer_tick);
        const double2 *slot = (const double2 *)(c->peer_region + peer_apply_off(c->g.Nx, (int)(seq & 3)));
        *f = faces_for(c, field, slot, slot + c->g.Nx);
        return SM_OK;
    }
    double2 *slo = face_buf(c, set, 0), *shi = face_buf(c, set, 1);
    double2 *rlo = face_buf(c, set, 2), *rhi = face_buf(c, set, 3);
    launch_pack_faces_proj(c->stream, c->g, field, c->U, kind, slo, shi);
    TRY(exchange_faces(c, slo, shi, rlo, rhi, (size_t)2 * c->g.Nx));
    *f = faces_for(c, field, rlo, rhi);
    return SM_OK;
}

// Global sum of per-block partials into c->sums[slot] (device).
int global_sum(sm_ctx *c, int nparts, const double2 *part, int slot) {
    launch_sum_partials(c->stream, nparts, part, c->sums + slot);
    return allreduce_dev(c, (double *)(c->sums + slot), 2);
}

// 2-deep faces of the fused CG kernel: 4 columns [-2,-1,Wt,Wt+1][plane][x].
// faces2 layout (complex, units of Nx): send slots of up to 3 fields at 8f
// (lo 4Nx, hi 4Nx), then receive slots at 24 + 8*which (which 0: d, 1: r,
// 2: U, 3: Ad), 56 Nx in all.
double2 *face2_recv(sm_ctx *c, int which) {  // 0: d, 1: r, 2: U, 3: Ad
    return c->faces2 + (size_t)(24 + 8 * which) * c->g.Nx;
}
double2 *face2_send(sm_ctx *c, int f, int hi) {  // send buffers of field slot f
    return c->faces2 + (size_t)(8 * f + 4 * hi) * c->g.Nx;
}

// Pack and exchange the 2-deep faces of nf (<= 2) fields in ONE transport
// round on stream s (RCCL: a single group of 4*nf p2p ops).
int halo2_multi(sm_ctx *c, hipStream_t s, const double2 *const *fields, double2 *const *faces, int nf) {
    if (!c->sharded()) return SM_OK;
    const size_t cnt = (size_t)8 * c->g.Nx;  // doubles: 2 columns x 2 planes x Nx complex
    for (int f = 0; f < nf; ++f) launch_pack_faces2(s, c->g, fields[f], face2_send(c, f, 0), face2_send(c, f, 1));
    if (c->hosted) {
        for (int f = 0; f < nf; ++f)
            TRY(exchange_faces_on(c, s, face2_send(c, f, 0), face2_send(c, f, 1), faces[f],
                                  faces[f] + (size_t)4 * c->g.Nx, cnt));
        return SM_OK;
    }
    if (c->peer) {
        const double2 *sl[3], *sh[3];
        double2 *rl[3], *rh[3];
        for (int f = 0; f < nf && f < 3; ++f) {
            sl[f] = face2_send(c, f, 0);
            sh[f] = face2_send(c, f, 1);
            rl[f] = faces[f];
            rh[f] = faces[f] + (size_t)4 * c->g.Nx;
        }
        return peer_exchange(c, s, nf, sl, sh, rl, rh, cnt);
    }
    const double2 *su[3], *sd[3];
    double2 *rd[3], *ru[3];
    if (nf > 3) return fail(SM_ERR_ARG, "halo2_multi: %d fields", nf);
    for (int f = 0; f < nf; ++f) {
        su[f] = face2_send(c, f, 1);
        sd[f] = face2_send(c, f, 0);
        rd[f] = faces[f];
        ru[f] = faces[f] + (size_t)4 * c->g.Nx;
    }
    return rccl_p2p_group(c, s, nf, su, rd, sd, ru, cnt);
}

int halo2(sm_ctx *c, const double2 *field, double2 *face) {
    const double2 *f[1] = {field};
    double2 *r[1] = {face};
    return halo2_multi(c, c->stream, f, r, 1);
}

// 4-deep faces of the recompute-Ad CG pass (sm_cgra.hip): [col -4..-1,
// Wt..Wt+3][plane][x], 16 Nx complex each. faces4 layout (complex, units of
// Nx): send lo 0, send hi 8, received d_{j-1} by pass parity at 16 and 32 (so
// pass j still holds d_{j-2}'s faces from pass j-1), U at 48; 64 Nx in all.
double2 *face4_send(sm_ctx *c, int hi) { return c->faces4 + (size_t)(8 * hi) * c->g.Nx; }
double2 *face4_recv_d(sm_ctx *c, long pass) { return c->faces4 + (size_t)(16 + 16 * (pass & 1)) * c->g.Nx; }
double2 *face4_recv_U(sm_ctx *c) { return c->faces4 + (size_t)48 * c->g.Nx; }
bool cg_ra_ok(const sm_ctx *c) { return !c->sharded() || c->g.Wt >= 4; }

// Pack and exchange the 4-deep t-faces of `field` into `recv` on stream s.
int halo4(sm_ctx *c, hipStream_t s, const double2 *field, double2 *recv) {
    launch_pack_faces_k(s, c->g, 4, field, face4_send(c, 0), face4_send(c, 1));
    return exchange_faces_on(c, s, face4_send(c, 0), face4_send(c, 1), recv, recv + (size_t)8 * c->g.Nx,
                             (size_t)16 * c->g.Nx);
}

int exchange_ghost_U(sm_ctx *c) {
    c->uang_state = 0;  // every change of U comes through here: the link codes are stale
    if (!c->sharded()) return SM_OK;
    // U_t(x, Wt-1) (plane 0 of my hi face) is the up-neighbour's U_t(x, -1)
    double2 *slo = face_buf(c, 1, 0), *shi = face_buf(c, 1, 1);
    double2 *rlo = face_buf(c, 1, 2), *rhi = face_buf(c, 1, 3);
    launch_pack_faces(c->stream, c->g, c->U, slo, shi);
    TRY(exchange_faces(c, slo, shi, rlo, rhi, (size_t)4 * c->g.Nx));
    HIP_TRY(hipMemcpyAsync(c->ghostU, rlo, sizeof(double2) * c->g.Nx, hipMemcpyDeviceToDevice, c->stream));
    // 2-deep ghost links for the fused CG kernel, 4-deep for the recompute-Ad pass
    TRY(halo2(c, c->U, face2_recv(c, 2)));
    if (cg_ra_ok(c)) TRY(halo4(c, c->stream, c->U, face4_recv_U(c)));
    return SM_OK;
}

// RCCL contexts, the CG pass's scalar sums: the recompute-Ad pass's last block
// all-reduces the shard's three sums itself (cg_ticketed_tail, the peer
// transport's in-pass all-reduce) through a 4-KiB uncached header per shard,
// instead of an ncclAllReduce after every pass; the halo exchange stays RCCL
// (north_star). The header handles are all-gathered over the context's own
// transport (the communicator; a host-staged context, test option
// hosted_psums=1, uses its all-reduce callback on byte values), and every
// shard's success (allocation, IPC open, a handshake all-reduce) is agreed by
// a min over shards, so all shards take the same path; any failure leaves
// the context on its transport's all-reduce. Every shard makes every
// collective call of this function whatever failed locally. Never fails the
// context on a local failure.
static int peer_sums_setup(sm_ctx *c, const std::function<int(char *, size_t)> &gather,
                           const std::function<int(int *)> &agree) {
    c->peer_sums = false;
    const int P = c->loop ? 1 : c->nshard, me = c->loop ? 0 : c->shard;
    const size_t hb = sizeof(hipIpcMemHandle_t);
    int ok = 1;
    std::vector<char> hh(hb * P, 0);
    if (hipExtMallocWithFlags((void **)&c->peer_region, kPeerHdrBytes, hipDeviceMallocUncached) != hipSuccess ||
        hipMemset(c->peer_region, 0, kPeerHdrBytes) != hipSuccess ||
        (!c->peer_view_dev && hipMalloc(&c->peer_view_dev, sizeof(PeerView)) != hipSuccess) ||
        hipIpcGetMemHandle(reinterpret_cast<hipIpcMemHandle_t *>(hh.data() + hb * me), c->peer_region) != hipSuccess)
        ok = 0;
    (void)hipGetLastError();
    int rc = gather(hh.data(), hb);
    for (int r = 0; rc == SM_OK && ok && r < P; ++r) {
        if (r == me) continue;
        void *p = nullptr;
        hipIpcMemHandle_t h;
        memcpy(&h, hh.data() + hb * r, hb);
        if (hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess) != hipSuccess) {
            ok = 0;
            (void)hipGetLastError();
        } else {
            c->peer_open[r] = (char *)p;
        }
    }
    if (rc == SM_OK) rc = agree(&ok);
    if (rc == SM_OK && ok) {
        PeerView &v = c->peer_view;
        v.me = me;
        v.n = P;
        v.down = c->loop ? 0 : down_rank(c);
        v.up = c->loop ? 0 : up_rank(c);
        v.Nx = c->g.Nx;
        v.wait_ticks = c->peer_wait_ticks;
        for (int r = 0; r < P; ++r) v.base[r] = r == me ? c->peer_region : c->peer_open[r];
        double *chk = (double *)(c->sums + 3);
        const double mine = (double)me;
        double got = -1.0;
        unsigned long long err = 0;
        if (hipMemcpy(c->peer_view_dev, &v, sizeof v, hipMemcpyHostToDevice) != hipSuccess ||
            hipMemcpy(chk, &mine, sizeof mine, hipMemcpyHostToDevice) != hipSuccess)
            ok = 0;
        launch_peer_allreduce(c->stream, chk, 1, v, ++c->peer_coll_seq);  // handshake (time-limited)
        if (hipStreamSynchronize(c->stream) != hipSuccess ||
            hipMemcpy(&got, chk, sizeof got, hipMemcpyDeviceToHost) != hipSuccess ||
            hipMemcpy(&err, c->peer_region + offsetof(PeerHdr, err), sizeof err, hipMemcpyDeviceToHost) != hipSuccess)
            ok = 0;
        if (err || got != 0.5 * P * (P - 1)) ok = 0;
        (void)hipGetLastError();
        rc = agree(&ok);
    }
    if (rc == SM_OK && ok) {
        c->peer_sums = true;
        return SM_OK;
    }
    for (char *&p : c->peer_open)
        if (p) {
            (void)hipIpcCloseMemHandle(p);
            p = nullptr;
        }
    if (c->peer_region) (void)hipFree(c->peer_region);
    c->peer_region = nullptr;
    (void)hipGetLastError();
    return rc;
}

int rccl_peer_sums_setup(sm_ctx *c) {
    c->peer_sums = false;
    if (!c->peer_sums_wish || !c->comm) return SM_OK;
    const int P = c->loop ? 1 : c->nshard, me = c->loop ? 0 : c->shard;
    char *dh = nullptr;  // the handles on the device for the all-gather
    int *flag = nullptr;
    HIP_TRY(hipMalloc(&dh, sizeof(hipIpcMemHandle_t) * P));
    if (hipMalloc(&flag, sizeof(int)) != hipSuccess) {
        (void)hipFree(dh);
        return fail(SM_ERR_HIP, "peer sums: allocation failed");
    }
    auto gather = [&](char *bytes, size_t nb) -> int {  // in place, over the communicator
        HIP_TRY(hipMemcpy(dh, bytes, nb * P, hipMemcpyHostToDevice));
        NCCL_TRY(ncclAllGather(dh + nb * me, dh, nb, ncclUint8, c->comm, c->stream));
        HIP_TRY(hipStreamSynchronize(c->stream));
        HIP_TRY(hipMemcpy(bytes, dh, nb * P, hipMemcpyDeviceToHost));
        return SM_OK;
    };
    auto agree = [&](int *ok) -> int {  // min over shards
        HIP_TRY(hipMemcpyAsync(flag, ok, sizeof *ok, hipMemcpyHostToDevice, c->stream));
        NCCL_TRY(ncclAllReduce(flag, flag, 1, ncclInt32, ncclMin, c->comm, c->stream));
        HIP_TRY(hipMemcpyAsync(ok, flag, sizeof *ok, hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(hipStreamSynchronize(c->stream));
        return SM_OK;
    };
    const int rc = peer_sums_setup(c, gather, agree);
    (void)hipFree(dh);
    (void)hipFree(flag);
    return rc;
}

// The same for a host-staged context (test option hosted_psums=1): the RCCL
// path's in-pass sums over its split launches with several shards on one GPU.
// The handle bytes travel as small integers through the all-reduce callback
// (each slot nonzero on one shard only: the sums are exact).
int hosted_peer_sums_setup(sm_ctx *c) {
    c->peer_sums = false;
    if (!c->hosted_psums) return SM_OK;
    const int P = c->nshard, me = c->shard;
    auto gather = [&](char *bytes, size_t nb) -> int {
        std::vector<double> v(nb * P, 0.0);
        for (size_t i = 0; i < nb; ++i) v[nb * me + i] = (double)(unsigned char)bytes[nb * me + i];
        if (c->tr.allreduce_sum(c->tr.user, v.data(), (long)v.size()) != 0)
            return fail(SM_ERR_ARG, "host transport allreduce failed");
        for (size_t i = 0; i < nb * P; ++i) bytes[i] = (char)(unsigned char)v[i];
        return SM_OK;
    };
    auto agree = [&](int *ok) -> int {
        double v = *ok ? 1.0 : 0.0;
        if (c->tr.allreduce_sum(c->tr.user, &v, 1) != 0) return fail(SM_ERR_ARG, "host transport allreduce failed");
        *ok = v == (double)P;
        return SM_OK;
    };
    return peer_sums_setup(c, gather, agree);
}

int peer_set_view(sm_ctx *c) {
    PeerView &v = c->peer_view;
    v.me = c->loop ? 0 : c->shard;
    v.n = c->loop ? 1 : c->nshard;
    v.down = c->loop ? 0 : down_rank(c);
    v.up = c->loop ? 0 : up_rank(c);
    v.Nx = c->g.Nx;
    v.wait_ticks = c->peer_wait_ticks;
    v.base[v.me] = c->peer_region;
    HIP_TRY(hipMemcpyAsync(c->peer_view_dev, &v, sizeof v, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    c->peer_connected = true;
    // handshake: one all-reduce of the shard numbers (every shard's region is
    // reachable and its flags move), checked here
    double *chk = (double *)(c->sums + 3);
    const double mine = (double)v.me;
    HIP_TRY(hipMemcpyAsync(chk, &mine, sizeof mine, hipMemcpyHostToDevice, c->stream));
    TRY(allreduce_dev(c, chk, 1));
    double got = -1.0;
    HIP_TRY(hipMemcpyAsync(&got, chk, sizeof got, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    TRY(sm_peer_status(c, nullptr));
    if (got != 0.5 * v.n * (v.n - 1))
        return fail(SM_ERR_STATE, "peer transport handshake: sum of shard numbers %g, expected %g", got,
                    0.5 * v.n * (v.n - 1));
    return SM_OK;
}
}  // namespace sm_host

extern "C" {

int sm_peer_connect(sm_ctx *c, const void *handles, int handle_bytes_each) {
    if (!c || !c->peer || c->loop) return fail(SM_ERR_ARG, "sm_peer_connect: not a peer-transport context");
    if (c->peer_connected) return fail(SM_ERR_STATE, "sm_peer_connect: already connected");
    if (!handles || handle_bytes_each < sm_peer_handle_bytes())
        return fail(SM_ERR_ARG, "sm_peer_connect: %d-byte handles expected", sm_peer_handle_bytes());
    HIP_TRY(hipSetDevice(c->device));
    for (int r = 0; r < c->nshard; ++r) {
        if (r == c->shard) continue;
        hipIpcMemHandle_t h;
        memcpy(&h, (const char *)handles + (size_t)r * handle_bytes_each, sizeof h);
        void *p = nullptr;
        const hipError_t e = hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess);
        if (e != hipSuccess) return fail(SM_ERR_HIP, "hipIpcOpenMemHandle of shard %d: %s", r, hipGetErrorString(e));
        c->peer_open[r] = (char *)p;
        c->peer_view.base[r] = (char *)p;
    }
    return peer_set_view(c);
}

int sm_peer_status(sm_ctx *c, unsigned long long *timed_out_seq) {
    if (!c) return fail(SM_ERR_ARG, "null context");
    unsigned long long err = 0;
    if ((c->peer || c->peer_sums) && c->peer_region) {
        HIP_TRY(hipStreamSynchronize(c->stream));
        HIP_TRY(hipMemcpy(&err, c->peer_region + offsetof(PeerHdr, err), sizeof err, hipMemcpyDeviceToHost));
    }
    if (timed_out_seq) *timed_out_seq = err;
    if (err) return fail(SM_ERR_RCCL, "peer transport: a wait timed out (sequence %llu)", err);
    return SM_OK;
}

}  // extern "C"
