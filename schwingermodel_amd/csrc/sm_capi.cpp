// sm_capi.cpp -- host side of libsm_hip.so: the C-ABI of include/sm_hip.h.
//
// Owns one t-shard of the lattice on one GPU: device-resident gauge field,
// CG work fields, halo faces, reduction partials and the device CG scalars;
// the operators, the CG driver and the context's life cycle. Kernels are in
// sm_kernels.hip / sm_cgra.hip / ...; the t-shard transports (RCCL over xGMI,
// host-staged, peer) and the halos are in sm_comm.cpp.

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <array>
#include <cstdarg>
#include <cstddef>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

#include "sm_fields.h"
#include "sm_ctx.h"
#include "sm_internal.h"

using namespace sm;
using namespace sm_host;

namespace {
thread_local std::string g_err;
}  // namespace

namespace sm_host {

int fail(int code, const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

// Neighbour sources for `in`: periodic aliases (1 GPU) or received faces.
TFaces faces_for(sm_ctx *c, const double2 *in, const double2 *recv_lo, const double2 *recv_hi) {
    TFaces f;
    if (!c->sharded()) {
        f.lo = in + (c->g.Wt - 1);
        f.lo_xs = c->g.Wt;
        f.lo_ps = c->g.V;
        f.hi = in;
        f.hi_xs = c->g.Wt;
        f.hi_ps = c->g.V;
    } else {
        // spin-projected faces (launch_pack_faces_proj): one complex per x
        f.lo = recv_lo;
        f.lo_xs = 1;
        f.lo_ps = 0;
        f.hi = recv_hi;
        f.hi_xs = 1;
        f.hi_ps = 0;
        f.proj = 1;
    }
    return f;
}

double2 *face_buf(sm_ctx *c, int set, int which) {
    // set 0/1: two independent spinor exchanges; which: 0 send_lo 1 send_hi 2 recv_lo 3 recv_hi
    return c->faces + (size_t)(set * 4 + which) * 2 * c->g.Nx;
}



const double2 *loU(sm_ctx *c) { return !c->sharded() ? c->U + (c->g.Wt - 1) : c->ghostU; }

int apply(sm_ctx *c, const double2 *in, double2 *out, double mass, int dagger, const double2 *aux,
          double2 *partials, const CGScalars *skip) {
    TFaces f;
    const int TB = (c->g.Wt + c->cfg.bt - 1) / c->cfg.bt;
    if (!c->sharded() || TB < 3 || !c->apply_split || c->peer) {
        // one shard, or a narrow t-shard: faces first, then one launch
        TRY(halo(c, in, 0, dagger ? FACE_DDAG : FACE_D, &f));
        launch_dslash(c->stream, c->g, c->cfg, dagger, in, out, c->U, loU(c), f, mass, aux, partials, skip);
    } else {
        // t-blocks 1..TB-2 never touch t = 0 / Wt-1: they run on the main
        // stream while the faces travel on the comm stream; the two edge
        // block-columns (TB-1, then 0 by wrap-around, one launch) follow the
        // faces there, concurrently with the interior launch
        double2 *slo = face_buf(c, 0, 0), *shi = face_buf(c, 0, 1);
        double2 *rlo = face_buf(c, 0, 2), *rhi = face_buf(c, 0, 3);
        HIP_TRY(hipEventRecord(c->ev_ready, c->stream));
        HIP_TRY(hipStreamWaitEvent(c->comm_stream, c->ev_ready, 0));
        rccl_joined(c, c->comm_stream, c->stream);
        launch_pack_faces_proj(c->comm_stream, c->g, in, c->U, dagger ? FACE_DDAG : FACE_D, slo, shi);
        TRY(exchange_faces_on(c, c->comm_stream, slo, shi, rlo, rhi, (size_t)2 * c->g.Nx));
        f = faces_for(c, in, rlo, rhi);
        launch_dslash(c->comm_stream, c->g, c->cfg, dagger, in, out, c->U, loU(c), f, mass, aux, partials, skip,
                      TB - 1, 2);
        HIP_TRY(hipEventRecord(c->ev_halo, c->comm_stream));
        launch_dslash(c->stream, c->g, c->cfg, dagger, in, out, c->U, loU(c), f, mass, aux, partials, skip,
                      1, TB - 2);
        HIP_TRY(hipStreamWaitEvent(c->stream, c->ev_halo, 0));
        rccl_joined(c, c->stream, c->comm_stream);
    }
    HIP_TRY(hipGetLastError());
    return SM_OK;
}


int check_ready(sm_ctx *c) {
    if (!c) return fail(SM_ERR_ARG, "null context");
    if (!c->have_gauge) return fail(SM_ERR_STATE, "no gauge field uploaded (sm_upload_gauge)");
    return SM_OK;
}

int upload_plane_pair(sm_ctx *c, double2 *dst, const double *p0, const double *p1) {
    const size_t bytes = sizeof(double2) * c->g.V;
    HIP_TRY(hipMemcpyAsync(dst, p0, bytes, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(dst + c->g.V, p1, bytes, hipMemcpyHostToDevice, c->stream));
    return SM_OK;
}

int download_plane_pair(sm_ctx *c, const double2 *src, double *p0, double *p1) {
    const size_t bytes = sizeof(double2) * c->g.V;
    HIP_TRY(hipMemcpyAsync(p0, src, bytes, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipMemcpyAsync(p1, src + c->g.V, bytes, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return SM_OK;
}



// Link codes for the recompute-Ad pass (cg_ra_kernel UC, sm_linkcode.h), rebuilt at the
// first solve after U changed (every change comes through exchange_ghost_U)
// or after the wish changed (sm_cg_link_codes). The codes rebuild every link
// BITWISE, so a pass reading them is the same arithmetic as one reading the
// complex links, and the choice needs no agreement between shards: each shard
// decides for itself from ITS links and the ghost links it received (the
// 4-deep face its pass reads), and shards deciding differently still compute
// the same iterates with the same collectives. The decision is a local host
// read (the counts of links not encodable and of flag words too wide for the
// packed form), no collective, and it runs only on a rebuild: a solve on an
// unchanged U and wish costs nothing here (round 4 all-reduced a
// stale count at every t-shard solve).
int ensure_link_angles(sm_ctx *c) {
    if (c->cg_fused != 5 || c->racfg.fold < 2 || !cg_ra_ok(c)) return SM_OK;
    if (c->uang_state != 0 || !c->link_angles) return SM_OK;
    if (!c->Uang) HIP_TRY(stream_malloc(c, (void **)&c->Uang, link_code_bytes(2 * c->g.V)));
    if (c->sharded() && !c->Uang_face) HIP_TRY(hipMalloc(&c->Uang_face, link_code_bytes(16 * (long)c->g.Nx)));
    // per block (links not rebuilt bitwise, links whose flag word needs 16 bits)
    int nb = launch_link_codes(c->stream, 2 * c->g.V, c->U, c->Uang, c->partials);
    if (c->sharded())
        nb += launch_link_codes(c->stream, 16 * (long)c->g.Nx, face4_recv_U(c), c->Uang_face, c->partials + nb);
    launch_sum_partials(c->stream, nb, c->partials, c->sums);
    HIP_TRY(hipMemcpyAsync(c->h_sums, c->sums, sizeof(double2), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    c->uang_state = c->h_sums[0].x == 0.0 ? 1 : 2;
    // the packed flags (one byte per site) when every flag word fits a nibble,
    // else the 16-bit flag words
    c->link_fmt = c->h_sums[0].y == 0.0 ? 2 : 1;
    if (c->uang_state == 1 && c->link_fmt == 2) {
        launch_link_nibbles(c->stream, c->g.V, c->Uang);
        if (c->sharded()) launch_face_nibbles(c->stream, c->g.Nx, c->Uang_face);
    }
    HIP_TRY(hipGetLastError());
    return SM_OK;
}

// alpha / beta from per-block partials (local sum, all-reduce over shards, scalar)
int cg_scalar(sm_ctx *c, int nparts, int which) {
    if (!c->sharded()) {
        if (which == 0) launch_cg_alpha(c->stream, nparts, c->partials, c->sc);
        else launch_cg_beta(c->stream, nparts, c->partials, c->sc);
        return SM_OK;
    }
    launch_sum_to_scalar(c->stream, nparts, c->partials, c->sc);
    TRY(allreduce_dev(c, (double *)&c->sc->sum, 2));
    if (which == 0) launch_cg_alpha_from_sum(c->stream, c->sc);
    else launch_cg_beta_from_sum(c->stream, c->sc);
    return SM_OK;
}
}  // namespace sm_host

// ============================================================================
extern "C" {

int sm_abi_version(void) { return 1; }
const char *sm_last_error(void) { return g_err.c_str(); }

int sm_shard_plan(int Nt, int nshard, int shard, int *t0, int *Wt) {
    if (Nt <= 0 || nshard <= 0 || shard < 0 || shard >= nshard)
        return fail(SM_ERR_ARG, "bad shard plan Nt=%d nshard=%d shard=%d", Nt, nshard, shard);
    // the reference enforces equal blocks (include/mpi_setup.h:14-19)
    if (Nt % nshard != 0) return fail(SM_ERR_ARG, "Nt=%d not divisible by nshard=%d", Nt, nshard);
    if (t0) *t0 = shard * (Nt / nshard);
    if (Wt) *Wt = Nt / nshard;
    return SM_OK;
}

int sm_device_count(int *n) {
    if (!n) return fail(SM_ERR_ARG, "null argument");
    *n = 0;
    HIP_TRY(hipGetDeviceCount(n));
    return SM_OK;
}

int sm_comm_unique_id(void *id_out, int id_bytes) {
    if (!id_out || id_bytes < (int)sizeof(ncclUniqueId))
        return fail(SM_ERR_ARG, "unique id buffer must hold %d bytes", (int)sizeof(ncclUniqueId));
    ncclUniqueId id;
    NCCL_TRY(ncclGetUniqueId(&id));
    memcpy(id_out, &id, sizeof id);
    return SM_OK;
}

// Test-only switches. Every production choice above is a per-shape rule or
// table; the tests force the alternatives through ONE environment variable,
// read when a context is created: SM_TEST_OPTS="key=value,key=value". The
// keys and the choice each forces:
//   cg=0|4|5            CG path (six launches / stored Ad / recompute Ad)
//   tail=0              scalar kernel instead of the ticketed tail
//   red_shards=0        t-shards: scalar kernel after the all-reduce
//   face_pipe=0|1|2     t-shards: d_j's faces packed by a kernel at the next
//                       pass (0), packed by the edge launch and sent right
//                       behind it (1), or packed by it and sent at the start of
//                       the next pass, after the all-reduce (2)
//   edge_xchunk=N       t-shards: rows per edge block (0: the interior's; -1: rule)
//   ra_red_max_blocks=N one shard: redundant scalars up to N blocks
//   fold=0|1|2          recompute-Ad pass arithmetic (2: fused multiply-adds)
//   apply_split=0|1     t-shard Dirac apply: interior / edge launches around
//                       the faces on the comm stream (1; default from Wt 2048)
//                       or faces first, then one launch (0)
//   rccl_order=0        no ordering events between RCCL operations on the two
//                       streams (A/B only: the one communicator then relies on
//                       RCCL's own ordering)
//   rccl_sums=1         RCCL contexts: the CG pass's scalar sums through
//                       ncclAllReduce instead of the in-pass peer all-reduce
//   hosted_psums=1      host-staged contexts: the CG pass's sums in-pass as on
//                       RCCL contexts (the multi-shard test of that path)
//   peer_wait_ms=N      peer transport: time limit of one wait (default 10000)
//   peer_store=0|1|2    peer transport: the CG pass's face stores as 16-B
//                       write-through buffer stores (0), 8-B atomic stores (1)
//                       or plain stores into the uncached ring (2)
//   ra_strip=0|1        recompute-Ad pass: the block's 4 waves share one t-strip
//                       (one shard; ignored on t-shards)
//   ra_xbal=0|1         recompute-Ad pass: balanced x-chunks (Nx / XB rows)
//   ra_remap=0|1        recompute-Ad pass tile order (1: each XCD takes a
//                       contiguous range of x-adjacent chunks, t-adjacent
//                       tiles consecutive; 0: round-robin dispatch order)
//   rev=0|1|2           recompute-Ad pass march schedule (0 all forward; 1 odd
//                       passes backward; 2, the default, x-adjacent chunks in
//                       opposite directions and odd passes flipped)
//   pad_alloc=0|5       placement of the streamed CG buffers (sm_ctx.h:
//                       5 >= 2 GiB each + contiguous flag, the default;
//                       0 own size)
//   place_probe=N       candidates per buffer of the placement probe (0: none;
//                       sm_set_placement_probe sets the default)
//   probe_min_mib=N     smallest field (MiB) whose context runs the probe
//   link_angles=0|1     recompute-Ad pass reads the links as one-double codes
//   ra_xchunk=N         recompute-Ad pass: N rows per tile (with ra_xbal=1: ceil(Nx/N) balanced chunks)
//   kernel_events=0|1   t-shard CG pass: hand-offs between the streams on events
//                       recorded by the launches themselves (1, the default) or markers
//   bt=64|128|256       Dirac apply t-columns per block
//   eo_fused=0, eo_cg_td=0, eo_cg_folded=1   even-odd operator / CG forms
//   debug_cg=1          CG host loops print their status (stderr)
// An unknown key or a malformed value fails the creation.
static int apply_test_opts(sm_ctx *c) {
    const char *env = getenv("SM_TEST_OPTS");
    if (!env || !*env) return SM_OK;
    std::string all(env);
    size_t pos = 0;
    while (pos < all.size()) {
        size_t end = all.find(',', pos);
        if (end == std::string::npos) end = all.size();
        const std::string kv = all.substr(pos, end - pos);
        pos = end + 1;
        if (kv.empty()) continue;
        const size_t eq = kv.find('=');
        char *tail = nullptr;
        const long v = eq == std::string::npos ? 0 : strtol(kv.c_str() + eq + 1, &tail, 10);
        if (eq == std::string::npos || !tail || *tail || tail == kv.c_str() + eq + 1)
            return fail(SM_ERR_ARG, "SM_TEST_OPTS: malformed '%s'", kv.c_str());
        const std::string k = kv.substr(0, eq);
        const int iv = (int)v;
        if (k == "cg") {
            if (iv != 0 && iv != 4 && iv != 5) return fail(SM_ERR_ARG, "SM_TEST_OPTS: cg must be 0, 4 or 5");
            c->cg_fused = iv;
        } else if (k == "tail") {
            c->cg_tail = iv;
        } else if (k == "red_shards") {
            c->cg_red_shards = iv;
        } else if (k == "face_pipe") {
            c->cg_face_pipe = iv;
        } else if (k == "edge_xchunk") {
            c->cg_edge_xchunk = iv;
        } else if (k == "ra_red_max_blocks") {
            c->cg_ra_red_max_blocks = iv;
        } else if (k == "fold") {
            c->racfg.fold = iv;
        } else if (k == "rev") {
            c->racfg.rev_odd = iv;
        } else if (k == "apply_split") {
            c->apply_split = iv ? 1 : 0;
        } else if (k == "rccl_order") {
            c->rccl_ordered = iv ? 1 : 0;
        } else if (k == "rccl_sums") {
            c->peer_sums_wish = iv ? 0 : 1;
        } else if (k == "hosted_psums") {
            c->hosted_psums = iv ? 1 : 0;
        } else if (k == "peer_wait_ms") {
            if (iv < 1) return fail(SM_ERR_ARG, "SM_TEST_OPTS: peer_wait_ms must be >= 1");
            c->peer_wait_ticks = 100000ull * (unsigned long long)iv;  // 100-MHz wall clock
        } else if (k == "peer_store") {
            if (iv < 0 || iv > 2) return fail(SM_ERR_ARG, "SM_TEST_OPTS: peer_store must be 0, 1 or 2");
            c->peer_store = iv;
        } else if (k == "ra_strip") {
            cg_ra_set_strip(c->racfg, c->g, iv);
        } else if (k == "kernel_events") {
            c->kernel_events = iv ? 1 : 0;
        } else if (k == "ra_xchunk") {  // rows per tile of the recompute-Ad pass (XB follows)
            if (iv < 2 || iv > c->g.Nx) return fail(SM_ERR_ARG, "SM_TEST_OPTS: ra_xchunk must be 2..Nx");
            c->racfg.xchunk = iv;
            c->racfg.XB = (c->g.Nx + iv - 1) / iv;
        } else if (k == "ra_xbal") {
            c->racfg.xbal = iv ? 1 : 0;
        } else if (k == "ra_remap") {
            if (iv < 0 || iv > 1) return fail(SM_ERR_ARG, "SM_TEST_OPTS: ra_remap must be 0 or 1");
            c->racfg.remap = iv;

        } else if (k == "probe_min_mib") {
            if (iv < 1) return fail(SM_ERR_ARG, "SM_TEST_OPTS: probe_min_mib must be >= 1");
            c->place_min_mib = iv;
        } else if (k == "place_probe") {
            if (iv < 0 || iv > 8) return fail(SM_ERR_ARG, "SM_TEST_OPTS: place_probe must be 0..8");
            c->place_probe = iv;
        } else if (k == "pad_alloc") {
            if (iv != 0 && iv != 5) return fail(SM_ERR_ARG, "SM_TEST_OPTS: pad_alloc must be 0 or 5");
            c->pad_alloc = iv;
        } else if (k == "link_angles") {
            c->link_angles = iv ? 1 : 0;
        } else if (k == "bt") {
            if (iv != 64 && iv != 128 && iv != 256) return fail(SM_ERR_ARG, "SM_TEST_OPTS: bt must be 64, 128 or 256");
            c->cfg.bt = iv;
            c->nparts_dslash = dslash_blocks(c->g, c->cfg);
        } else if (k == "eo_fused") {
            c->eo_fused = iv;
        } else if (k == "eo_cg_td") {
            c->eo_cg_td = iv;
        } else if (k == "eo_cg_folded") {
            c->eo_cg_folded = iv;
        } else if (k == "debug_cg") {
            c->debug_cg = iv;
        } else {
            return fail(SM_ERR_ARG, "SM_TEST_OPTS: unknown key '%s'", k.c_str());
        }
    }
    return SM_OK;
}


static int create_common(sm_ctx **out, int Nx, int Nt_global, int nshard, int shard, int device,
                         const void *unique_id, const sm_host_transport *tr, bool loop = false, bool peer = false) {
    if (!out) return fail(SM_ERR_ARG, "null out");
    *out = nullptr;
    int t0, Wt;
    if (Nx < 1) return fail(SM_ERR_ARG, "Nx=%d", Nx);
    TRY(sm_shard_plan(Nt_global, nshard, shard, &t0, &Wt));
    if (nshard > 1 && !unique_id && !tr && !peer) return fail(SM_ERR_ARG, "nshard > 1 needs a unique id or a transport");
    if (tr && (!tr->exchange || !tr->allreduce_sum)) return fail(SM_ERR_ARG, "incomplete host transport");
    int ndev = 0;
    HIP_TRY(hipGetDeviceCount(&ndev));
    if (device < 0 || device >= ndev) return fail(SM_ERR_ARG, "device %d of %d", device, ndev);
    HIP_TRY(hipSetDevice(device));
    sm_ctx *c = new sm_ctx();
    c->device = device;
    if (hipDeviceGetAttribute(&c->n_cu, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || c->n_cu <= 0)
        c->n_cu = 256;
    c->loop = loop;
    c->peer = peer;
    c->nshard = nshard;
    c->shard = shard;
    c->g.Nx = Nx;
    c->g.Wt = Wt;
    c->g.t0 = t0;
    c->g.Ntg = Nt_global;
    c->g.V = (long)Nx * Wt;
    c->cfg = dslash_config(c->g);
    c->nparts_dslash = dslash_blocks(c->g, c->cfg);
    c->nparts_red = reduce_blocks(2 * c->g.V);
    c->fcfg = cg_fused_config(c->g);
    c->racfg = cg_ra_config(c->g);
    // every per-tile partial slot must fit c->partials (2 kMaxPartials complex;
    // the one-pass CG grids write 3 per tile): tall shards march longer chunks
    // instead of writing past it
    auto fit = [Nx](CGFusedCfg &f) {
        while (3L * cg_fused_blocks(f) > 2L * kMaxPartials && f.xchunk < Nx) {
            f.xchunk = std::min(Nx, 2 * f.xchunk);
            f.XB = (Nx + f.xchunk - 1) / f.xchunk;
        }
        return 3L * cg_fused_blocks(f) <= 2L * kMaxPartials;
    };
    // Per-shape choices (measured):
    // * CG path: the recompute-Ad pass from 256^2 sites per shard, the
    //   stored-Ad pass below (latency-bound grids; tools/small_cg.py).
    c->cg_fused = c->g.V >= (1L << 16) ? 5 : 4;
    // * t-shard apply: faces first, then one launch, on shards narrower than
    //   2048 (RCCL loopback, us per apply: 4096x1024 79 vs 91 split; 4096x2048
    //   166 vs 164, 4096^2 296 vs 292; profiles/r02_v8_apply_split.log).
    c->apply_split = c->g.Wt >= 2048 ? 1 : 0;
    // * link codes from 4M sites per shard: below, the fields of a pass sit
    //   largely in the 256 MB MALL and the pass is bound by its VALU work,
    //   where decoding the links cost more than the 16 B it saves (round 2's
    //   angle form, tools/tune_shapes.py: 4096x512 0.080 vs 0.068 ms per
    //   iteration, 4096x1024 0.141 vs 0.147; tools/link_probe.py re-measures
    //   it for the codes).
    c->link_angles = c->g.V >= (1L << 22) ? 1 : 0;
    c->place_probe = placement_probe_default();
    if (int rc = apply_test_opts(c); rc != SM_OK) {
        delete c;
        return rc;
    }
    if (c->sharded() && c->racfg.strip) cg_ra_set_strip(c->racfg, c->g, 0);  // t-strips: one-shard contexts only
    while (c->nparts_dslash > kMaxPartials && c->cfg.xchunk < Nx) {
        c->cfg.xchunk = std::min(Nx, 2 * c->cfg.xchunk);
        c->nparts_dslash = dslash_blocks(c->g, c->cfg);
    }
    if (!fit(c->fcfg) || !fit(c->racfg) || c->nparts_dslash > kMaxPartials) {
        delete c;
        return fail(SM_ERR_ARG, "shard %dx%d too wide for the partial-sum buffer", Nx, Wt);
    }
    const int np = kMaxPartials;
    const size_t fb = sizeof(double2) * 2 * (size_t)c->g.V;
    hipError_t e = hipSuccess;
    auto chk = [&](hipError_t x) { if (e == hipSuccess) e = x; };
    chk(hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking));
    c->stream = c->own_stream;
    c->hosted = nshard > 1 && tr;
    // The host-staged transport synchronises the stream inside every exchange
    // and all-reduce, so a second stream buys it no overlap: its contexts run
    // on ONE stream (one hardware queue per process, the fewest when several
    // shards share a GPU). RCCL contexts overlap faces and edge blocks with
    // the interior on a separate comm stream.
    if (c->hosted || c->peer) {
        c->comm_stream = c->own_stream;
    } else {
        chk(hipStreamCreateWithFlags(&c->comm_stream, hipStreamNonBlocking));
        c->own_comm_stream = true;
    }
    chk(hipMalloc(&c->U, fb));
    chk(hipMalloc(&c->ghostU, sizeof(double2) * (size_t)Nx));
    for (int i = 0; i < NFIELDS; ++i) {
        // the recompute-Ad pass's three direction buffers and the x it updates
        const bool hot = i == F_D || i == F_D2 || i == F_R || i == F_X;
        chk(hot ? stream_malloc(c, (void **)&c->fields[i], fb) : hipMalloc(&c->fields[i], fb));
    }
    // the passes update F_X (placed as above) on every field from 256 MiB up,
    // including fields that are themselves a power of two >= 2 GiB (8192^2 on
    // one GPU): the caller's x is wherever its allocator put it
    c->x_internal = fb >= (size_t(256) << 20);
    chk(hipMalloc(&c->faces, sizeof(double2) * 2 * (size_t)Nx * 8));
    chk(hipMalloc(&c->faces2, sizeof(double2) * 56 * (size_t)Nx));
    chk(hipMalloc(&c->faces4, sizeof(double2) * 64 * (size_t)Nx));
    chk(hipEventCreateWithFlags(&c->ev_ready, hipEventDisableTiming));
    chk(hipEventCreateWithFlags(&c->ev_halo, hipEventDisableTiming));
    chk(hipEventCreateWithFlags(&c->ev_int, hipEventDisableTiming));
    chk(hipEventCreateWithFlags(&c->ev_rccl, hipEventDisableTiming));
    chk(hipMalloc(&c->partials, sizeof(double2) * 2 * (size_t)np));
    chk(hipMalloc(&c->sums, sizeof(double2) * 4));
    chk(hipMalloc(&c->Fbuf, sizeof(double) * 2 * (size_t)c->g.V));
    chk(hipMalloc(&c->sc, sizeof(CGScalars)));
    chk(hipMalloc(&c->tick, sizeof(unsigned) * (1 + kMaxTickGroups)));
    chk(hipMalloc(&c->gsum, sizeof(double2) * 3 * kMaxTickGroups));
    chk(hipHostMalloc(&c->h_sc, sizeof(CGScalars)));
    chk(hipHostMalloc(&c->h_sums, sizeof(double2) * 4));
    chk(hipHostMalloc(&c->h_face, sizeof(double) * 4 * kMaxFaceDoubles * (size_t)Nx));
    chk(hipHostMalloc(&c->h_red, sizeof(double) * 8));
    if (c->peer) {  // the region the other shards store into (sm_peer.h), uncached
        chk(hipExtMallocWithFlags((void **)&c->peer_region, (size_t)peer_region_bytes(Nx), hipDeviceMallocUncached));
        chk(hipMalloc(&c->peer_tick, sizeof(unsigned)));
        chk(hipMalloc(&c->peer_view_dev, sizeof(PeerView)));
        if (e == hipSuccess) chk(hipMemsetAsync(c->peer_region, 0, (size_t)peer_region_bytes(Nx), c->own_stream));
        if (e == hipSuccess) chk(hipMemsetAsync(c->peer_tick, 0, sizeof(unsigned), c->own_stream));
    }
    // on the context's stream, not the null stream (which would be one more
    // hardware queue per process); face slots start as zeros, not whatever
    // the allocator hands back
    if (e == hipSuccess) chk(hipMemsetAsync(c->sc, 0, sizeof(CGScalars), c->own_stream));
    if (e == hipSuccess) chk(hipMemsetAsync(c->tick, 0, sizeof(unsigned) * (1 + kMaxTickGroups), c->own_stream));
    if (e == hipSuccess) chk(hipMemsetAsync(c->faces, 0, sizeof(double2) * 2 * (size_t)Nx * 8, c->own_stream));
    if (e == hipSuccess) chk(hipMemsetAsync(c->faces2, 0, sizeof(double2) * 56 * (size_t)Nx, c->own_stream));
    if (e == hipSuccess) chk(hipMemsetAsync(c->faces4, 0, sizeof(double2) * 64 * (size_t)Nx, c->own_stream));
    if (e == hipSuccess) chk(hipStreamSynchronize(c->own_stream));
    if (e != hipSuccess) {
        sm_destroy(c);
        return fail(SM_ERR_HIP, "allocation failed: %s", hipGetErrorString(e));
    }
    if (int rc = placement_probe(c, fb); rc != SM_OK) {
        sm_destroy(c);
        return rc;
    }
    if (c->hosted) {
        c->tr = *tr;
        if (int rc = hosted_peer_sums_setup(c); rc != SM_OK) {
            sm_destroy(c);
            return rc;
        }
    } else if (c->peer) {
        // connected by sm_peer_connect (the loopback: here, to itself)
    } else if (c->sharded()) {
        // RCCL's mixing of graph-captured and eager launches on one communicator
        // costs every launch a cross-stream dependency; nothing here is captured
        // (RCCL loopback, ms per CG iteration: 4096x512 0.0911 against 0.0944,
        // 4096x1024 0.1542 against 0.1613; profiles/r06_j_rccl_launch_env.jsonl).
        // A caller's own setting wins.
        setenv("NCCL_GRAPH_MIXING_SUPPORT", "0", 0);
        ncclUniqueId id;
        memcpy(&id, unique_id, sizeof id);
        ncclResult_t r = ncclCommInitRank(&c->comm, nshard, id, shard);
        if (r != ncclSuccess) {
            c->comm = nullptr;
            sm_destroy(c);
            return fail(SM_ERR_RCCL, "ncclCommInitRank: %s", ncclGetErrorString(r));
        }
        if (int rc = rccl_peer_sums_setup(c); rc != SM_OK) {
            sm_destroy(c);
            return rc;
        }
    }
    *out = c;
    return SM_OK;
}


int sm_create(sm_ctx **out, int Nx, int Nt_global, int nshard, int shard, int device,
              const void *unique_id) {
    return create_common(out, Nx, Nt_global, nshard, shard, device, unique_id, nullptr);
}

int sm_create_loopback(sm_ctx **out, int Nx, int Nt_global, int device, const void *unique_id) {
    if (!unique_id) return fail(SM_ERR_ARG, "loopback needs an RCCL unique id (sm_comm_unique_id)");
    return create_common(out, Nx, Nt_global, 1, 0, device, unique_id, nullptr, true);
}

// ---- the peer transport (sm_peer.h) ----
int sm_peer_handle_bytes(void) { return (int)sizeof(hipIpcMemHandle_t); }


int sm_create_peer(sm_ctx **out, int Nx, int Nt_global, int nshard, int shard, int device, void *handle_out,
                   int handle_bytes) {
    if (nshard < 2 || nshard > kPeerMaxRanks)
        return fail(SM_ERR_ARG, "peer transport: 2..%d shards (one shard: sm_create_peer_loopback)", kPeerMaxRanks);
    if (!handle_out || handle_bytes < sm_peer_handle_bytes())
        return fail(SM_ERR_ARG, "peer transport: the handle buffer must hold %d bytes", sm_peer_handle_bytes());
    TRY(create_common(out, Nx, Nt_global, nshard, shard, device, nullptr, nullptr, false, true));
    hipIpcMemHandle_t h;
    const hipError_t e = hipIpcGetMemHandle(&h, (*out)->peer_region);
    if (e != hipSuccess) {
        sm_destroy(*out);
        *out = nullptr;
        return fail(SM_ERR_HIP, "hipIpcGetMemHandle: %s", hipGetErrorString(e));
    }
    memcpy(handle_out, &h, sizeof h);
    return SM_OK;
}


int sm_create_peer_loopback(sm_ctx **out, int Nx, int Nt_global, int device) {
    TRY(create_common(out, Nx, Nt_global, 1, 0, device, nullptr, nullptr, true, true));
    const int rc = peer_set_view(*out);
    if (rc != SM_OK) {
        sm_destroy(*out);
        *out = nullptr;
    }
    return rc;
}


int sm_create_hosted(sm_ctx **out, int Nx, int Nt_global, int nshard, int shard, int device,
                     const sm_host_transport *transport) {
    if (!transport) return fail(SM_ERR_ARG, "null transport");
    return create_common(out, Nx, Nt_global, nshard, shard, device, nullptr, transport);
}

int sm_destroy(sm_ctx *c) {
    if (!c) return SM_OK;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    if (c->comm_stream) (void)hipStreamSynchronize(c->comm_stream);  // e.g. a CG's trailing face exchange
    if (c->comm) ncclCommDestroy(c->comm);
    for (char *&p : c->peer_open)
        if (p) {
            (void)hipIpcCloseMemHandle(p);
            p = nullptr;
        }
    if (c->peer_region) (void)hipFree(c->peer_region);
    if (c->peer_tick) (void)hipFree(c->peer_tick);
    if (c->peer_view_dev) (void)hipFree(c->peer_view_dev);
    for (double2 *&f : c->fields)
        if (f) {
            stream_free(c, f);
            f = nullptr;
        }
    stream_free(c, c->Uang);
    c->Uang = nullptr;
    void *dev[] = {c->U, c->ghostU, c->faces, c->faces2, c->faces4, c->partials, c->sums, c->Fbuf, c->sc,
                   c->U_alt, c->Pmd, c->Fmd, c->eo, c->Ucb, c->eo_faces, c->eo_faces4, c->Uang_face,
                   c->tick, c->gsum};
    for (void *p : dev)
        if (p) (void)hipFree(p);
    if (c->h_sc) (void)hipHostFree(c->h_sc);
    if (c->h_sums) (void)hipHostFree(c->h_sums);
    if (c->h_face) (void)hipHostFree(c->h_face);
    if (c->h_red) (void)hipHostFree(c->h_red);
    if (c->comm_stream) (void)hipStreamSynchronize(c->comm_stream);
    for (hipEvent_t ev : {c->ev_ready, c->ev_halo, c->ev_int, c->ev_rccl})
        if (ev) (void)hipEventDestroy(ev);
    if (c->comm_stream && c->own_comm_stream) (void)hipStreamDestroy(c->comm_stream);
    if (c->own_stream) (void)hipStreamDestroy(c->own_stream);
    delete c;
    return SM_OK;
}

int sm_tune_cg(sm_ctx *c, int fused, int xchunk) {
    if (!c) return fail(SM_ERR_ARG, "null context");
    if (fused > 5 || (fused >= 1 && fused <= 3))
        return fail(SM_ERR_ARG, "CG path must be 0 (reference sequence), 4 (stored Ad) or 5 (recompute Ad)");
    if (fused >= 0) c->cg_fused = fused;
    if (xchunk > 0) {
        CGFusedCfg &cur = c->cg_fused == 5 ? c->racfg : c->fcfg;  // the active pass's geometry
        CGFusedCfg f = cur;
        f.xchunk = xchunk;
        f.XB = (c->g.Nx + xchunk - 1) / xchunk;
        if (3 * cg_fused_blocks(f) > 2 * kMaxPartials) return fail(SM_ERR_ARG, "too many blocks");
        cur = f;
    }
    return SM_OK;
}

int sm_tune_cg_geometry(sm_ctx *c, int waves_per_block, int xchunk) {
    if (!c) return fail(SM_ERR_ARG, "null context");
    CGFusedCfg f = c->racfg;
    if (waves_per_block > 0) {
        if (waves_per_block != 1 && waves_per_block != 2 && waves_per_block != 4)
            return fail(SM_ERR_ARG, "waves per block must be 1, 2 or 4");
        if (f.strip && waves_per_block == 1) return fail(SM_ERR_ARG, "t-strip blocks are 2 or 4 waves");
        f.wpb = waves_per_block;
        cg_ra_set_strip(f, c->g, f.strip);
    }
    if (xchunk > 0) f.xchunk = xchunk;
    f.XB = (c->g.Nx + f.xchunk - 1) / f.xchunk;
    if (3L * cg_fused_blocks(f) > 2L * kMaxPartials) return fail(SM_ERR_ARG, "too many blocks");
    c->racfg = f;
    for (int &n : c->cg_shard_blocks_per_cu) n = -1;  // the block size may have changed
    return SM_OK;
}

int sm_tune_cg_strip(sm_ctx *c, int strip, int balanced) {
    if (!c) return fail(SM_ERR_ARG, "null context");
    CGFusedCfg f = c->racfg;
    if (strip >= 0) {
        if (strip && c->sharded()) return fail(SM_ERR_ARG, "t-strip blocks run on one-shard contexts");
        if (strip && f.fold < 2) return fail(SM_ERR_ARG, "t-strip blocks take the fused multiply-add pass (fold 2)");
        cg_ra_set_strip(f, c->g, strip);
    }
    if (balanced >= 0) f.xbal = balanced ? 1 : 0;
    f.XB = (c->g.Nx + f.xchunk - 1) / f.xchunk;
    if (3L * cg_fused_blocks(f) > 2L * kMaxPartials) return fail(SM_ERR_ARG, "too many blocks");
    c->racfg = f;
    for (int &n : c->cg_shard_blocks_per_cu) n = -1;
    return SM_OK;
}

int sm_cg_link_angles(sm_ctx *c, int on, int *in_use) { return sm_cg_link_codes(c, on, in_use); }

int sm_cg_link_bytes(const sm_ctx *c, int *bytes_per_site) {
    if (!c || !bytes_per_site) return fail(SM_ERR_ARG, "null argument");
    // recorded by the passes as they were launched: a later gauge
    // upload, a Metropolis reject or a change of wish does not rewrite it
    *bytes_per_site = c->cg_link_bytes_last;
    return SM_OK;
}

int sm_link_code_check(sm_ctx *c, double *U_out, double *max_err, long *n_bad) {
    TRY(check_ready(c));
    if (!max_err || !n_bad) return fail(SM_ERR_ARG, "null argument");
    // per block: (links beyond the bound, largest error)
    const int nb = launch_link_code_check(c->stream, 2 * c->g.V, c->U, (double2 *)U_out, c->partials);
    std::vector<double2> h(nb);
    HIP_TRY(hipMemcpyAsync(h.data(), c->partials, sizeof(double2) * nb, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    double bad = 0.0, mx = 0.0;
    for (const double2 &b : h) {
        bad += b.x;
        mx = b.y > mx || b.y != b.y ? b.y : mx;  // a NaN error stays NaN
    }
    *n_bad = (long)bad;
    *max_err = mx;
    return SM_OK;
}

int sm_cg_link_codes(sm_ctx *c, int on, int *in_use) {
    if (!c) return fail(SM_ERR_ARG, "null context");
    if (on >= 0 && (on ? 1 : 0) != c->link_angles) {
        c->link_angles = on ? 1 : 0;
        c->uang_state = 0;  // decided again (by this shard) at the next solve
    }
    if (in_use) *in_use = c->link_angles && c->cg_fused == 5 && c->uang_state == 1 ? 1 : 0;
    return SM_OK;
}

int sm_tune(sm_ctx *c, int bt, int xchunk, int xcd_remap, int variant) {
    if (!c) return fail(SM_ERR_ARG, "null context");
    LaunchCfg cfg = c->cfg;
    if (bt > 0) cfg.bt = bt;
    if (xchunk > 0) cfg.xchunk = xchunk;
    if (xcd_remap >= 0) cfg.xcd_remap = xcd_remap;
    if (variant >= 0) cfg.variant = variant;
    if (cfg.bt % 64 || cfg.bt > 256 || cfg.xchunk < 1)
        return fail(SM_ERR_ARG, "bad launch config bt=%d xchunk=%d", cfg.bt, cfg.xchunk);
    if (dslash_blocks(c->g, cfg) > kMaxPartials) return fail(SM_ERR_ARG, "too many blocks");
    c->cfg = cfg;
    c->nparts_dslash = dslash_blocks(c->g, cfg);
    return SM_OK;
}

int sm_bench_stream(sm_ctx *c, int two_reads, long n, const double *a, const double *b, double *out,
                    int blocks) {
    if (!c || !a || !out || (two_reads && !b)) return fail(SM_ERR_ARG, "null argument");
    launch_stream(c->stream, two_reads, n, (const double2 *)a, (const double2 *)b, (double2 *)out, blocks);
    HIP_TRY(hipGetLastError());
    return SM_OK;
}

int sm_set_stream(sm_ctx *c, void *s) {
    if (!c) return fail(SM_ERR_ARG, "null context");
    // the old stream's work completes before any is issued on the new one
    // (its RCCL operations have completed: the next one needs no ordering
    // event on it)
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (c->rccl_last == c->stream) c->rccl_last = nullptr;
    c->stream = s ? (hipStream_t)s : c->own_stream;
    if (c->hosted || c->peer) c->comm_stream = c->stream;  // hosted and peer contexts run on one stream
    return SM_OK;
}

int sm_comm_info(const sm_ctx *c, int *transport, int *nranks, int *rank) {
    if (!c) return fail(SM_ERR_ARG, "null context");
    int t = 0, n = 1, r = 0;
    if (c->hosted) {
        t = 1;
    } else if (c->peer) {
        t = 3;  // the shards the peer view holds (sm_peer_connect)
        n = c->peer_view.n;
        r = c->peer_view.me;
    } else if (c->comm) {
        t = 2;
        NCCL_TRY(ncclCommCount(c->comm, &n));  // what the communicator itself holds, not the creation arguments
        NCCL_TRY(ncclCommUserRank(c->comm, &r));
    }
    if (transport) *transport = t;
    if (nranks) *nranks = n;
    if (rank) *rank = r;
    return SM_OK;
}

int sm_cg_sums_in_pass(const sm_ctx *c, int *in_pass) {
    if (!c || !in_pass) return fail(SM_ERR_ARG, "null argument");
    *in_pass = c->peer || c->peer_sums ? 1 : 0;
    return SM_OK;
}

int sm_synchronize(sm_ctx *c) {
    if (!c) return fail(SM_ERR_ARG, "null context");
    HIP_TRY(hipStreamSynchronize(c->stream));
    return SM_OK;
}

int sm_local_sites(const sm_ctx *c, long *V, int *Nx, int *Wt, int *t0) {
    if (!c) return fail(SM_ERR_ARG, "null context");
    if (V) *V = c->g.V;
    if (Nx) *Nx = c->g.Nx;
    if (Wt) *Wt = c->g.Wt;
    if (t0) *t0 = c->g.t0;
    return SM_OK;
}

int sm_upload_gauge(sm_ctx *c, const double *U0, const double *U1) {
    if (!c || !U0 || !U1) return fail(SM_ERR_ARG, "null argument");
    HIP_TRY(hipSetDevice(c->device));
    TRY(upload_plane_pair(c, c->U, U0, U1));
    TRY(exchange_ghost_U(c));
    HIP_TRY(hipStreamSynchronize(c->stream));
    c->have_gauge = true;
    return SM_OK;
}

int sm_upload_gauge_dev(sm_ctx *c, const double *U) {
    if (!c || !U) return fail(SM_ERR_ARG, "null argument");
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipMemcpyAsync(c->U, U, sizeof(double2) * 2 * c->g.V, hipMemcpyDeviceToDevice, c->stream));
    TRY(exchange_ghost_U(c));
    c->have_gauge = true;
    return SM_OK;
}

// ---- device-resident operators -------------------------------------------
int sm_dirac_dev(sm_ctx *c, const double *in, double *out, double m0, int dagger) {
    TRY(check_ready(c));
    return apply(c, (const double2 *)in, (double2 *)out, m0 + 2, dagger ? 1 : 0, nullptr, nullptr, nullptr);
}

int sm_ddag_dev(sm_ctx *c, const double *in, double *out, double m0) {
    TRY(check_ready(c));
    double2 *tmp = c->field(F_TMP);   // the reference's DTEMP
    TRY(apply(c, (const double2 *)in, tmp, m0 + 2, 1, nullptr, nullptr, nullptr));
    return apply(c, tmp, (double2 *)out, m0 + 2, 0, nullptr, nullptr, nullptr);
}

int sm_force_dev(sm_ctx *c, const double *l, const double *r, double *F) {
    TRY(check_ready(c));
    TFaces fl, fr;
    TRY(halo(c, (const double2 *)l, 0, FACE_FORCE_L, &fl));
    TRY(halo(c, (const double2 *)r, 1, FACE_FORCE_R, &fr));
    launch_force(c->stream, c->g, c->U, (const double2 *)l, (const double2 *)r, fl, fr, F);
    HIP_TRY(hipGetLastError());
    return SM_OK;
}

int sm_dot_dev(sm_ctx *c, const double *a, const double *b, double *out) {
    if (!c || !out) return fail(SM_ERR_ARG, "null argument");
    launch_dot_partial(c->stream, 2 * c->g.V, (const double2 *)a, (const double2 *)b, c->partials);
    TRY(global_sum(c, c->nparts_red, c->partials, 0));
    HIP_TRY(hipMemcpyAsync(c->h_sums, c->sums, sizeof(double2), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    out[0] = c->h_sums[0].x;
    out[1] = c->h_sums[0].y;
    return SM_OK;
}

// ---- CG on D D^dagger (src/conjugate_gradient.cpp:4-66) ---------------------
int sm_cg_begin(sm_ctx *c, const double *phi, double *x, double m0, double tol) {
    TRY(check_ready(c));
    TRY(ensure_link_angles(c));
    const long n = 2 * c->g.V;
    const double2 *ph = (const double2 *)phi;
    double2 *xx = (double2 *)x;
    c->cg_mass = m0 + 2;
    c->cg_phi = ph;
    // On large fields the passes update x in F_X, an allocation laid out like
    // the direction buffers (stream_alloc_bytes), and sm_cg_finish copies it
    // to the caller's x: the caller's buffer is wherever its allocator put it.
    c->cg_x_user = nullptr;
    if (c->x_internal && xx != c->field(F_X) && ph != c->field(F_X)) {
        c->cg_x_user = xx;
        xx = c->field(F_X);
    }
    c->cg_x = xx;
    double2 *r = c->field(F_R), *d = c->field(F_D), *Ad = c->field(F_AD), *t = c->field(F_T);
    if ((const double2 *)xx != ph) launch_copy(c->stream, n, ph, xx);          // x = phi
    TRY(apply(c, xx, t, c->cg_mass, 1, nullptr, nullptr, nullptr));            // DD^dag x
    TRY(apply(c, t, Ad, c->cg_mass, 0, nullptr, nullptr, nullptr));
    double2 *prr = c->partials, *ppp = c->partials + c->nparts_red;
    launch_cg_init(c->stream, n, ph, Ad, r, d, prr, ppp);                        // r = phi - Ax; d = r
    if (!c->sharded()) {
        launch_cg_finalize_init(c->stream, c->nparts_red, prr, ppp, c->sc, tol);
    } else {
        launch_sum_partials(c->stream, c->nparts_red, prr, c->sums);
        launch_sum_partials(c->stream, c->nparts_red, ppp, c->sums + 1);
        TRY(allreduce_dev(c, (double *)c->sums, 4));
        launch_cg_init_from_sums(c->stream, c->sums, c->sc, tol);
    }
    HIP_TRY(hipGetLastError());
    c->cg_active = 1;
    c->cg_issued = 0;
    c->cg_flush_pass = -1;
    c->cg_flush_sums = 0;
    c->cg_pending_x = 0;
    c->cg_faces_for = -1;
    c->cg_faces_packed = 0;
    return SM_OK;
}


// One pass of the two-direction CG with a stored Ad (cg_fused == 4,
// sm_cgfused.hip: cg_onepass_kernel): pass j reads d_{j-1}, d_{j-2} and
// Ad_{j-1}, writes d_j and Ad_j, updates x on even passes (so after an odd
// final pass sm_cg_finish adds the pending alpha_{j-1} d_{j-1}), then the
// scalar kernel forms err / stop, alpha_j and beta_j. d rotates through three
// buffers (cg_dbuf), Ad ping-pongs.
static double2 *cg_dbuf(sm_ctx *c, long i) {  // d_i (d_0 from cg_init in F_D)
    static const int slot[3] = {F_D2, F_R, F_D};
    return c->field(slot[((i % 3) + 3) % 3]);
}

static int cg_onepass(sm_ctx *c) {
    const long j = c->cg_issued;
    const bool odd = j & 1, first = j == 0;
    // pass 0 reads d_0 from F_D and stores it to cg_dbuf(0)
    const double2 *dold = first ? c->field(F_D) : cg_dbuf(c, j - 1);
    const double2 *d2 = cg_dbuf(c, j - 2);
    double2 *dnew = cg_dbuf(c, j);
    double2 *aold = c->field(odd ? F_AD2 : F_AD), *anew = c->field(odd ? F_AD : F_AD2);
    const CGFusedCfg &fc = c->fcfg;
    const int nparts = cg_fused_blocks(fc);
    // redundant scalars on small one-shard grids: partials by pass parity,
    // evaluated by every block of the next pass; sm_cg_iterate flushes the last
    const bool redundant = !c->sharded() && nparts <= c->cg_red_max_blocks;
    double2 *part = redundant ? c->partials + (j & 1) * 3 * (size_t)nparts : c->partials;
    const double2 *prev = redundant ? c->partials + ((j + 1) & 1) * 3 * (size_t)nparts : nullptr;
    auto pass = [&](int tb0, int tbn, hipStream_t st) {
        launch_cg_onepass(st, c->g, fc, c->kshards(), dold, d2, aold, dnew, anew, c->cg_x, c->U, face2_recv(c, 0),
                          face2_recv(c, 1), face2_recv(c, 3), face2_recv(c, 2), c->cg_mass, first, c->sc, part, tb0,
                          tbn, prev, j);
    };
    c->cg_pending_x = 1;  // sm_cg_finish checks the device's final pass parity
    if (!c->sharded()) {
        pass(0, fc.TBk, c->stream);
        if (!redundant) launch_cg1_scalars(c->stream, nparts, c->partials, c->sc, first);
        c->cg_flush_pass = redundant ? j : -1;
        c->cg_flush_nparts = nparts;
        return SM_OK;
    }
    // interior t-blocks while the 2-deep faces of d_{j-1}, d_{j-2}, Ad_{j-1} travel (one round)
    const double2 *flds[3] = {dold, d2, aold};
    double2 *fcs[3] = {face2_recv(c, 0), face2_recv(c, 1), face2_recv(c, 3)};
    auto interior = [&](int tb) {
        const int g_lo = 4 * tb, g_hi = std::min(4 * tb + 3, fc.NWT - 1);
        return kFusedWaveCols * g_lo - 2 >= 0 && kFusedWaveCols * g_hi + kFusedWaveCols + 1 <= c->g.Wt - 1;
    };
    int tb_lo = 0, tb_hi = -1;
    for (int tb = 0; tb < fc.TBk; ++tb)
        if (interior(tb)) {
            if (tb_hi < 0) tb_lo = tb;
            tb_hi = tb;
        }
    const bool split = tb_hi >= tb_lo && tb_hi >= 0;
    HIP_TRY(hipEventRecord(c->ev_ready, c->stream));
    HIP_TRY(hipStreamWaitEvent(c->comm_stream, c->ev_ready, 0));
    rccl_joined(c, c->comm_stream, c->stream);
    TRY(halo2_multi(c, c->comm_stream, flds, fcs, 3));
    // edge t-blocks (tb_hi, TBk) and [0, tb_lo), wrapping: one launch, on the
    // comm stream behind the faces, concurrent with the interior launch
    if (split) pass(tb_hi + 1, fc.TBk - 1 - tb_hi + tb_lo, c->comm_stream);
    HIP_TRY(hipEventRecord(c->ev_halo, c->comm_stream));
    if (split) pass(tb_lo, tb_hi - tb_lo + 1, c->stream);
    HIP_TRY(hipStreamWaitEvent(c->stream, c->ev_halo, 0));
    rccl_joined(c, c->stream, c->comm_stream);
    if (!split) pass(0, fc.TBk, c->stream);
    launch_cg1_local_sum(c->stream, nparts, c->partials, c->sc);
    TRY(allreduce_dev(c, (double *)c->sc->sum3, 6));
    launch_cg1_from_sums(c->stream, c->sc, first);
    return SM_OK;
}

// One pass of the recompute-Ad CG (cg_fused == 5, sm_cgra.hip): the
// two-direction pass without the Ad vector, d_i in cg_dbuf(i). t-shards: the
// 4-deep faces of d_{j-1} arrive in slot j & 1 on the comm stream while the
// interior t-blocks run; d_{j-2}'s faces are still in slot (j-1) & 1.
// The blocks owning columns 0..3 and Wt-4..Wt-1 (the 4-deep faces) are all
// edge blocks (outside [tb_lo, tb_hi]), so the edge launch can pack the faces.
static bool ra_edge_owns_faces(const sm_ctx *c, const CGFusedCfg &fc, int tb_lo, int tb_hi) {
    const int Wt = c->g.Wt;
    if (Wt < 8) return false;  // lo and hi columns would overlap
    auto blk = [&](int col) { return col / kRAWaveCols / fc.wpb; };
    for (int col : {0, 3, Wt - 4, Wt - 1})
        if (blk(col) >= tb_lo && blk(col) <= tb_hi) return false;
    return true;
}

// The recompute-Ad pass on t-shards over the peer transport: ONE launch over
// every t-block on the main stream. The blocks owning columns 0..3 / Wt-4..Wt-1
// store d_j's 4-deep faces straight into ring slot j % 3 of the down / up
// neighbour's region, and the pass's last block all-reduces the shard's sums
// in-kernel (cg_ticketed_tail) -- it returns only once every shard's sums of
// pass j are in, and every shard's pass j has written its faces before its own
// sums, so pass j+1 finds d_j's faces in its ring when it starts. Pass 0 reads
// d_0's faces from a generic exchange into slot 2 (= -1 mod 3); shards narrower
// than 8 columns (the lo and hi face columns overlap) exchange d_{j-1} at every
// pass that way. Ring slots by j % 3: pass j reads slots j-1, j-2 and its
// neighbours write slot j, which nobody reads before pass j+1.
static double2 *peer_ring(const sm_ctx *c, int r, long j) {
    return (double2 *)(c->peer_view.base[r] + peer_ring_off(c->g.Nx, (int)(((j % 3) + 3) % 3)));
}

static int cg_ra_pass_peer(sm_ctx *c, const double2 *d1, const double2 *d2, double2 *dn, const double *ua) {
    TRY(peer_ready(c));
    const long j = c->cg_issued;
    const bool first = j == 0;
    const CGFusedCfg &fc = c->racfg;
    const int nparts = cg_fused_blocks(fc);
    if (fc.fold < 2 || (nparts + 63) / 64 > kMaxTickGroups)
        return fail(SM_ERR_STATE, "peer transport: the recompute-Ad pass needs the ticketed tail");
    const int me = c->peer_view.me;
    double2 *f1 = peer_ring(c, me, j - 1), *f2 = first ? f1 : peer_ring(c, me, j - 2);
    const bool direct = c->g.Wt >= 8;
    if (first || !direct) TRY(halo4(c, c->stream, d1, f1));
    const long Nx = c->g.Nx;
    double2 *fs = direct ? peer_ring(c, c->peer_view.down, j) + 8 * Nx : nullptr;  // my columns 0..3: its Wt..Wt+3
    double2 *fsh = direct ? peer_ring(c, c->peer_view.up, j) : nullptr;             // my Wt-4..Wt-1: its -4..-1
    double2 *sums = &c->sc->sumr[j & 1][0];
    const int lb = launch_cg_ra(c->stream, c->g, fc, c->kshards(), d1, d2, dn, c->cg_x, c->U, f1, f2, face4_recv_U(c),
                                c->cg_mass, j, c->sc, c->partials, 0, fc.TBk, nullptr, ua, c->Uang_face, fs, 0,
                                c->tick, nparts, c->gsum, sums, 1, c->link_fmt, fsh, c->peer_view_dev,
                                ++c->peer_coll_seq, c->peer_store,
                                // the shape's march schedule where a one-shard pass of this grid takes it
                                // (the ticketed tail, not the redundant scalars of small grids)
                                nparts > c->cg_ra_red_max_blocks ? 1 : 0);
    if (lb) c->cg_link_bytes_last = lb;
    c->cg_flush_pass = j;
    c->cg_flush_sums = 1;
    return SM_OK;
}

static int cg_ra_pass(sm_ctx *c) {
    const long j = c->cg_issued;
    const bool first = j == 0;
    const double2 *d1 = first ? c->field(F_D) : cg_dbuf(c, j - 1);
    const double2 *d2 = cg_dbuf(c, j - 2);
    double2 *dn = cg_dbuf(c, j);
    const CGFusedCfg &fc = c->racfg;
    const int nparts = cg_fused_blocks(fc);
    c->cg_pending_x = 2;  // sm_cg_finish adds the rows still pending (by the final pass parity)
    c->cg_flush_pass = -1;
    c->cg_flush_sums = 0;
    const bool one = !c->sharded();
    const bool angles = c->link_angles && c->uang_state == 1;
    const double *ua = angles ? c->Uang : nullptr;
    if (one) {
        // redundant scalars on small grids (partials by pass parity; every block
        // of the next pass evaluates them; sm_cg_iterate flushes the last pass)
        const bool red = fc.fold >= 2 && !fc.strip && nparts <= c->cg_ra_red_max_blocks;  // (t-strips: the tail)
        double2 *part = red ? c->partials + (j & 1) * 3 * (size_t)nparts : c->partials;
        const double2 *prev = red ? c->partials + ((j + 1) & 1) * 3 * (size_t)nparts : nullptr;
        const bool tail = !red && (c->cg_tail || fc.strip) && fc.fold >= 2 && (nparts + 63) / 64 <= kMaxTickGroups;
        c->cg_link_bytes_last =
            launch_cg_ra(c->stream, c->g, fc, 1, d1, d2, dn, c->cg_x, c->U, nullptr, nullptr, nullptr, c->cg_mass, j,
                         c->sc, part, 0, fc.TBk, prev, ua, nullptr, nullptr, 0, tail ? c->tick : nullptr, nparts,
                         c->gsum, nullptr, 0, c->link_fmt);
        if (red) {
            c->cg_flush_pass = j;
            c->cg_flush_nparts = nparts;
        } else if (!tail) {
            launch_cg1_scalars(c->stream, nparts, c->partials, c->sc, first);
        }
        return SM_OK;
    }
    if (c->peer) return cg_ra_pass_peer(c, d1, d2, dn, ua);
    // pass 0 has no d_{-2}: its (zero-weighted) faces are d_0's own, never the
    // other slot, which holds nothing of this solve yet (the zero multiplier
    // beta2 = 0 would turn a stale NaN there into a NaN iterate)
    double2 *f1 = face4_recv_d(c, j), *f2 = first ? f1 : face4_recv_d(c, j - 1);
    // interior t-blocks: every lane's column (56g-4 .. 56g+59) inside [0, Wt)
    auto interior = [&](int tb) {
        const int g_lo = fc.wpb * tb, g_hi = std::min(fc.wpb * tb + fc.wpb - 1, fc.NWT - 1);
        return kRAWaveCols * g_lo - 4 >= 0 && kRAWaveCols * g_hi + kRAWaveCols + 3 <= c->g.Wt - 1;
    };
    int tb_lo = 0, tb_hi = -1;
    for (int tb = 0; tb < fc.TBk; ++tb)
        if (interior(tb)) {
            if (tb_hi < 0) tb_lo = tb;
            tb_hi = tb;
        }
    const bool split = tb_hi >= tb_lo && tb_hi >= 0;
    const int nint = split ? tb_hi - tb_lo + 1 : 0, nedge = fc.TBk - nint;
    // Pipelined faces (t-shards, edge launch concurrent): the edge blocks write
    // d_j's 4-deep send faces themselves, and the exchange for pass j+1 follows
    // them on the comm stream, under the interior launch and the scalar step;
    // the edge launch marches short chunks so it ends long before the interior
    // one (its blocks otherwise run as long as the whole pass, AFTER the faces).
    // Edge rows per block: 8 where those tiles still join the interior ones
    // in one residency round, else 16, or 32 where only the longer chunks let
    // the edge tiles join the interior ones in one residency round (the resident
    // blocks per CU come from the runtime's occupancy of the launched kernel,
    // cg_ra_shard_blocks_per_cu: 8 one-wave blocks at 2 waves per SIMD for
    // the round-5 kernel). RCCL loopback, ms per
    // iteration, 16 / 32 / 24 rows (profiles/r05_q_edge_chunk_long.jsonl):
    // 4096x1024 (1751 interior tiles + 512 / 256 / 342 edge ones against 2048
    // slots) 0.159 / 0.150 / 0.173; 4096x512 (all fit) 0.085 / 0.093 / 0.088;
    // 4096x2048 (the interior alone overflows) 0.257 / 0.261-0.271 / 0.260.
    CGFusedCfg ec = fc;
    const bool pipe = split && c->cg_face_pipe && ra_edge_owns_faces(c, fc, tb_lo, tb_hi);
    // face_pipe 2 (deferred): the edge launch still packs d_j's faces, but
    // they are SENT at the start of pass j+1, after this pass's all-reduce in
    // the communicator's order (comm stream behind ev_ready), so the RCCL
    // operations alternate exchange, all-reduce, exchange, ... and the
    // launch schedule's own events order them (no ordering event on the
    // critical path: the all-reduce waits only for the edge launch it needs
    // anyway, ev_halo, which follows the exchange)
    const bool deferred = pipe && c->cg_face_pipe == 2;
    int exc = c->cg_edge_xchunk;
    if (exc < 0) {
        const int form = angles ? c->link_fmt : 0;
        int &per_cu = c->cg_shard_blocks_per_cu[form];
        if (per_cu < 0) per_cu = cg_ra_shard_blocks_per_cu(fc, form);
        const long slots = (long)c->n_cu * (per_cu > 0 ? per_cu : 8 / fc.wpb), inner = (long)nint * fc.XB;
        auto tiles = [&](int r) { return inner + (long)nedge * ((c->g.Nx + r - 1) / r); };
        // 8 rows where even those tiles join the interior ones in one round
        // (round 6, with the RCCL order: 4096x512 0.0951 against 0.0987 ms
        // per iteration for 16, profiles/r06_f_chunk_alignment_edge_rows.jsonl)
        exc = tiles(8) <= slots ? 8 : (tiles(16) > slots && tiles(32) <= slots ? 32 : 16);
    }
    if (pipe && exc > 0 && exc < fc.xchunk) {
        ec.xchunk = exc;
        ec.XB = (c->g.Nx + ec.xchunk - 1) / ec.xchunk;
        if (3L * (nint * fc.XB + nedge * ec.XB) > 2L * kMaxPartials) ec = fc;
    }
    const int nparts_pass = split ? nint * fc.XB + nedge * ec.XB : nparts;
    // ticketed tail: the pass's last block forms the scalars (one shard) or
    // this shard's sums, instead of a separate kernel
    const bool tail = c->cg_tail && fc.fold >= 2 && (nparts_pass + 63) / 64 <= kMaxTickGroups;
    // t-shard redundant scalars (with the tail): every block of pass j
    // evaluates pass j-1's scalars from its all-reduced sums (kept by pass
    // parity), so no scalar kernel sits between the all-reduce and the next pass
    const bool red = tail && c->cg_red_shards;
    double2 *sums = red ? &c->sc->sumr[j & 1][0] : c->sc->sum3;  // this shard's sums (all-reduced below)
    // RCCL contexts with peer sums (rccl_peer_sums_setup): the pass's last block
    // all-reduces the sums itself, one collective number for both launches
    const bool psums = c->peer_sums && red;
    const PeerView *pv = psums ? c->peer_view_dev : nullptr;
    const unsigned long long pseq = psums ? ++c->peer_coll_seq : 0;
    auto pass = [&](const CGFusedCfg &cf, int tb0, int tbn, hipStream_t st, int pbase, double2 *fsend,
                    hipEvent_t stop = nullptr) {
        const int lb = launch_cg_ra(st, c->g, cf, c->kshards(), d1, d2, dn, c->cg_x, c->U, f1, f2, face4_recv_U(c),
                                    c->cg_mass, j, c->sc, c->partials, tb0, tbn, nullptr, ua, c->Uang_face, fsend,
                                    pbase, tail ? c->tick : nullptr, nparts_pass, c->gsum, sums, red ? 1 : 0,
                                    c->link_fmt, nullptr, pv, pseq, 2 /* faces: plain stores, local */, 0, stop);
        if (lb) c->cg_link_bytes_last = lb;
    };
    // Kernel-carried events (kernel_events): when this pass enqueues nothing on
    // the main stream after its interior launch (in-pass sums, ticketed tail,
    // scalars in the next pass), that launch records ev_int itself, and the
    // next pass's comm stream waits on it -- everything the edge launch needs
    // from the main stream -- instead of on a marker recorded behind it; the
    // edge launch likewise records ev_halo. ~3 us off each pass's critical
    // path (tools/stream_gap_probe.hip). Any other pass (the first of an
    // sm_cg_iterate call, or one enqueueing more) records the marker.
    const bool kev = c->kernel_events && split && psums && red && tail && !deferred;
    if (kev && c->ev_int_pass == j - 1 && !first) {
        HIP_TRY(hipStreamWaitEvent(c->comm_stream, c->ev_int, 0));
    } else {
        HIP_TRY(hipEventRecord(c->ev_ready, c->stream));
        HIP_TRY(hipStreamWaitEvent(c->comm_stream, c->ev_ready, 0));
    }
    c->ev_int_pass = -1;
    rccl_joined(c, c->comm_stream, c->stream);
    // d_{j-1}'s faces: already in slot j & 1 if pass j-1 sent them (pipe), or
    // packed by pass j-1's edge launch and sent now (deferred)
    if (!(pipe && c->cg_faces_for == j)) {
        TRY(halo4(c, c->comm_stream, d1, f1));
    } else if (c->cg_faces_packed) {
        TRY(exchange_faces_on(c, c->comm_stream, face4_send(c, 0), face4_send(c, 1), f1, f1 + (size_t)8 * c->g.Nx,
                              (size_t)16 * c->g.Nx));
    }
    c->cg_faces_for = -1;
    c->cg_faces_packed = 0;
    // edge t-blocks (tb_hi, TBk) and [0, tb_lo), wrapping: one launch on the
    // comm stream behind the faces, concurrent with the interior launch
    if (split)
        pass(ec, tb_hi + 1, nedge, c->comm_stream, nint * fc.XB, pipe ? face4_send(c, 0) : nullptr,
             kev ? c->ev_halo : nullptr);
    if (!kev) HIP_TRY(hipEventRecord(c->ev_halo, c->comm_stream));
    if (split) pass(fc, tb_lo, nint, c->stream, 0, nullptr, kev ? c->ev_int : nullptr);
    if (kev) c->ev_int_pass = j;
    if (deferred) {  // d_j's faces stay packed until pass j+1
        c->cg_faces_for = j + 1;
        c->cg_faces_packed = 1;
    } else if (pipe) {  // d_j's faces into slot (j+1) & 1 (d_{j-2}'s, read by this pass's edge launch above)
        double2 *r = face4_recv_d(c, j + 1);
        TRY(exchange_faces_on(c, c->comm_stream, face4_send(c, 0), face4_send(c, 1), r, r + (size_t)8 * c->g.Nx,
                              (size_t)16 * c->g.Nx));
        c->cg_faces_for = j + 1;
    }
    HIP_TRY(hipStreamWaitEvent(c->stream, c->ev_halo, 0));
    // (face_pipe 1: ev_halo precedes the face exchange issued after it)
    if (!pipe || deferred) rccl_joined(c, c->stream, c->comm_stream);
    if (!split) pass(fc, 0, fc.TBk, c->stream, 0, nullptr);
    if (!tail) launch_cg1_local_sum(c->stream, nparts_pass, c->partials, c->sc);
    if (!psums) TRY(allreduce_dev(c, (double *)sums, 6));
    if (red) {
        c->cg_flush_pass = j;
        c->cg_flush_sums = 1;
        return SM_OK;
    }
    launch_cg1_from_sums(c->stream, c->sc, first);
    return SM_OK;
}

int sm_cg_iterate(sm_ctx *c, int niter) {
    TRY(check_ready(c));
    if (!c->cg_active) return fail(SM_ERR_STATE, "sm_cg_iterate before sm_cg_begin");
    const long n = 2 * c->g.V;
    double2 *r = c->field(F_R), *Ad = c->field(F_AD), *t = c->field(F_T);
    double2 *x = c->cg_x;
    for (int i = 0; i < niter; ++i) {
        if (c->cg_fused == 5 && cg_ra_ok(c)) {
            TRY(cg_ra_pass(c));
        } else if (c->cg_fused >= 4) {
            TRY(cg_onepass(c));
            c->cg_link_bytes_last = 32;
        } else {
            c->cg_link_bytes_last = 32;
            // the reference's sequence, six launches (src/conjugate_gradient.cpp:31-63):
            // Ad = D D^dag d with fused partials of <d, Ad>; alpha; x, r; beta; d
            double2 *d = c->field(F_D);
            TRY(apply(c, d, t, c->cg_mass, 1, nullptr, nullptr, c->sc));
            TRY(apply(c, t, Ad, c->cg_mass, 0, d, c->partials, c->sc));
            TRY(cg_scalar(c, c->nparts_dslash, 0));
            launch_cg_update_xr(c->stream, n, x, r, d, Ad, c->sc, c->partials);
            TRY(cg_scalar(c, c->nparts_red, 1));
            launch_cg_update_d(c->stream, n, d, r, c->sc);
        }
        c->cg_issued++;
    }
    c->ev_int_pass = -1;  // whatever follows on the main stream is not behind ev_int
    if (c->cg_fused >= 4 && c->cg_flush_pass >= 0) {  // redundant scalars: evaluate the last pass for the host
        const long J = c->cg_flush_pass;
        const int nparts = c->cg_flush_nparts;
        if (c->cg_flush_sums) launch_cg_ra_flush_sums(c->stream, c->sc, J);
        else launch_cg1_flush(c->stream, nparts, c->partials + (J & 1) * 3 * (size_t)nparts, c->sc, J);
        c->cg_flush_pass = -1;
        c->cg_flush_sums = 0;
    }
    HIP_TRY(hipGetLastError());
    return SM_OK;
}

int sm_cg_finish(sm_ctx *c, sm_cg_result *res) {
    if (!c || !res) return fail(SM_ERR_ARG, "null argument");
    if (c->cg_active && c->sharded()) {  // the last pass's face exchange (pipelined faces) joins the main stream
        HIP_TRY(hipEventRecord(c->ev_halo, c->comm_stream));
        HIP_TRY(hipStreamWaitEvent(c->stream, c->ev_halo, 0));
        rccl_joined(c, c->stream, c->comm_stream);
    }
    if (c->cg_active && c->cg_pending_x == 2) {  // recompute-Ad pass: x rows by parity
        launch_cg_ra_finish_x(c->stream, c->g, c->cg_x, cg_dbuf(c, 0), cg_dbuf(c, 1), cg_dbuf(c, 2), c->sc);
        HIP_TRY(hipGetLastError());
        c->cg_pending_x = 0;
    } else if (c->cg_active && c->cg_pending_x) {
        launch_cg_td_finish_x(c->stream, 2 * c->g.V, c->cg_x, cg_dbuf(c, 0), cg_dbuf(c, 1), cg_dbuf(c, 2), c->sc);
        HIP_TRY(hipGetLastError());
        c->cg_pending_x = 0;
    }
    if (c->cg_active && c->cg_x_user) {
        launch_copy(c->stream, 2 * c->g.V, c->cg_x, c->cg_x_user);
        HIP_TRY(hipGetLastError());
        c->cg_x_user = nullptr;
    }
    c->cg_active = 0;
    TRY(sm_cg_status(c, res));
    if (c->peer || c->peer_sums) return sm_peer_status(c, nullptr);  // a timed-out wait makes the solve an error
    return SM_OK;
}

int sm_cg_status(sm_ctx *c, sm_cg_result *res) {
    if (!c || !res) return fail(SM_ERR_ARG, "null argument");
    HIP_TRY(hipMemcpyAsync(c->h_sc, c->sc, sizeof(CGScalars), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    res->converged = c->h_sc->converged;
    res->iterations = c->h_sc->k;
    res->residual = c->h_sc->err;
    res->phi_norm = c->h_sc->phi_norm;
    return SM_OK;
}

int sm_cg_dev(sm_ctx *c, const double *phi, double *x, double m0, double tol, int max_iter,
              sm_cg_result *res) {
    if (!res) return fail(SM_ERR_ARG, "null result");
    TRY(sm_cg_begin(c, phi, x, m0, tol));
    // Enqueue iterations in chunks; each CG kernel is a no-op once the device
    // flag `done` is set, so overshooting a chunk costs only empty launches.
    // The one-pass paths run max_iter + 1 passes (pass 0 forms Ad_0) and stop
    // themselves at k == max_iter.
    int passes = max_iter;
    if (c->cg_fused >= 4) {
        HIP_TRY(hipMemsetD32Async((hipDeviceptr_t)&c->sc->max_iter, max_iter, 1, c->stream));
        passes = max_iter + 1;
    }
    CgChunker plan;
    int issued = 0, chunk = plan.chunk;
    while (issued < passes) {
        const int nb = (passes - issued) < chunk ? (passes - issued) : chunk;
        TRY(sm_cg_iterate(c, nb));
        issued += nb;
        TRY(sm_cg_status(c, res));
        if (c->debug_cg)
            fprintf(stderr, "[sm cg shard %d/%d] passes %d k %d err %.3e\n", c->shard, c->nshard, issued,
                    res->iterations, res->residual);
        if (res->converged) break;
        chunk = plan.next(res->iterations, res->residual, tol * res->phi_norm);
    }
    return sm_cg_finish(c, res);
}

// ---- host-pointer (drop-in) operators ---------------------------------------
int sm_dirac(sm_ctx *c, const double *in0, const double *in1, double *out0, double *out1, double m0,
             int dagger) {
    TRY(check_ready(c));
    HIP_TRY(hipSetDevice(c->device));
    double2 *in = c->field(F_IN), *out = c->field(F_OUT);
    TRY(upload_plane_pair(c, in, in0, in1));
    TRY(sm_dirac_dev(c, (const double *)in, (double *)out, m0, dagger));
    return download_plane_pair(c, out, out0, out1);
}

int sm_ddag(sm_ctx *c, const double *in0, const double *in1, double *out0, double *out1, double m0) {
    TRY(check_ready(c));
    HIP_TRY(hipSetDevice(c->device));
    double2 *in = c->field(F_IN), *out = c->field(F_OUT);
    TRY(upload_plane_pair(c, in, in0, in1));
    TRY(sm_ddag_dev(c, (const double *)in, (double *)out, m0));
    return download_plane_pair(c, out, out0, out1);
}

int sm_force(sm_ctx *c, const double *l0, const double *l1, const double *r0, const double *r1,
             double *F0, double *F1) {
    TRY(check_ready(c));
    HIP_TRY(hipSetDevice(c->device));
    double2 *l = c->field(F_L), *r = c->field(F_RR);
    TRY(upload_plane_pair(c, l, l0, l1));
    TRY(upload_plane_pair(c, r, r0, r1));
    TRY(sm_force_dev(c, (const double *)l, (const double *)r, c->Fbuf));
    const size_t bytes = sizeof(double) * c->g.V;
    HIP_TRY(hipMemcpyAsync(F0, c->Fbuf, bytes, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipMemcpyAsync(F1, c->Fbuf + c->g.V, bytes, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return SM_OK;
}

int sm_dot(sm_ctx *c, const double *a0, const double *a1, const double *b0, const double *b1,
           double *out) {
    if (!c) return fail(SM_ERR_ARG, "null context");
    HIP_TRY(hipSetDevice(c->device));
    double2 *a = c->field(F_IN), *b = c->field(F_OUT);
    TRY(upload_plane_pair(c, a, a0, a1));
    TRY(upload_plane_pair(c, b, b0, b1));
    return sm_dot_dev(c, (const double *)a, (const double *)b, out);
}

int sm_cg(sm_ctx *c, const double *phi0, const double *phi1, double *x0, double *x1, double m0,
          double tol, int max_iter, sm_cg_result *res) {
    TRY(check_ready(c));
    HIP_TRY(hipSetDevice(c->device));
    double2 *phi = c->field(F_PHI), *x = c->field(F_X);
    TRY(upload_plane_pair(c, phi, phi0, phi1));
    TRY(sm_cg_dev(c, (const double *)phi, (double *)x, m0, tol, max_iter, res));
    return download_plane_pair(c, x, x0, x1);
}

}  // extern "C"
