// sm_ctx.h -- private host-side state of one lattice shard (the opaque
// sm_ctx of include/sm_hip.h) and the transport / launch helpers shared by
// sm_capi.cpp (operators, CG) and sm_md.cpp (gauge field, MD, HMC).
#pragma once
#include "../../include/sm_hip.h"

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cmath>
#include <cstddef>
#include <vector>

#include "sm_internal.h"
#include "sm_peer.h"

namespace sm_host {

int fail(int code, const char *fmt, ...);

#define HIP_TRY(expr)                                                                   \
    do {                                                                                \
        hipError_t e_ = (expr);                                                         \
        if (e_ != hipSuccess)                                                           \
            return ::sm_host::fail(SM_ERR_HIP, "%s failed: %s (%s:%d)", #expr,           \
                                   hipGetErrorString(e_), __FILE__, __LINE__);          \
    } while (0)

#define NCCL_TRY(expr)                                                                     \
    do {                                                                                   \
        ncclResult_t r_ = (expr);                                                          \
        if (r_ != ncclSuccess)                                                             \
            return ::sm_host::fail(SM_ERR_RCCL, "%s failed: %s (%s:%d)", #expr,             \
                                   ncclGetErrorString(r_), __FILE__, __LINE__);            \
    } while (0)

#define TRY(expr)                     \
    do {                              \
        int rc_ = (expr);             \
        if (rc_ != SM_OK) return rc_; \
    } while (0)

}  // namespace sm_host


// Work fields, each 2*V complex (plane mu0 then mu1).
// F_D, F_D2, F_R: the three d buffers of the one-pass CG paths (F_R is r in the
// six-launch path); F_AD2: the second Ad buffer of the stored-Ad pass (ping-pong with F_AD).
enum { F_IN, F_OUT, F_TMP, F_X, F_R, F_D, F_D2, F_T, F_AD, F_PHI, F_L, F_RR, F_AD2, NFIELDS };

struct sm_ctx {
    int device = 0;
    int nshard = 1, shard = 0;
    // RCCL loopback (sm_create_loopback): one shard driven through the t-shard
    // code path, faces and scalar sums over a one-rank communicator (self
    // send/recv). Tests the RCCL data path on a single GPU.
    bool loop = false;
    int debug_cg = 0;  // test option debug_cg=1: the CG host loops print their status at each check (stderr)
    bool sharded() const { return nshard > 1 || loop; }  // faces + collectives (else periodic wrap)
    int kshards() const { return sharded() ? 2 : 1; }    // the kernels' view: > 1 reads faces
    sm::Geometry g{};
    sm::LaunchCfg cfg{};
    sm::CGFusedCfg fcfg{};
    sm::CGFusedCfg racfg{};        // recompute-Ad CG pass (sm_cgra.hip)
    // CG iteration: 0 the reference's six-launch sequence (576 B/site), 4 the
    // two-direction one-pass form with a stored Ad (sm_cgfused.hip: no r
    // vector, x every other pass, 224 B/site), 5 the two-direction pass that
    // recomputes Ad instead of storing it (sm_cgra.hip, 160 B/site). Chosen at
    // creation: 5 from 256^2 sites per shard, 4 below (latency-bound grids).
    int cg_fused = 4;
    int cg_red_max_blocks = sm::kRedundantMaxBlocks;  // stored-Ad pass: redundant scalars up to this grid
    long cg_flush_pass = -1;        // last one-pass pass whose scalars still await evaluation
    int cg_flush_nparts = 0;        // its partial count (the one-pass or the recompute-Ad grid)
    int cg_ra_red_max_blocks = 512; // recompute-Ad pass: redundant scalars up to this many blocks (one shard)
    // recompute-Ad pass with compact links (sm_cgra.hip UC): U enters the CG as
    // one double + one 16-bit flag word per link (sm_linkcode.h, 20 B/site),
    // rebuilt bitwise in registers.
    // Built at the first solve after U changes (uang_state 0); state 1 = in
    // use, 2 = some link is not encodable (far off the unit circle, NaN), so
    // the complex links are used.
    int link_angles = 1;
    int uang_state = 0;
    int link_fmt = 1;               // codes in use: 2 = flag nibbles, one byte per site; 1 = 16-bit flag words
    int cg_link_bytes_last = 0;     // link bytes per site the last CG pass launched read (sm_cg_link_bytes; 0: none yet)
    // Placement of the buffers the CG pass streams (stream_malloc): 5 = an
    // allocation of >= 2 GiB each with hipDeviceMallocContiguous (the
    // default; plain allocation of that size when the driver has no
    // contiguous memory), 0 = own size (A/B). Test option pad_alloc=N; DESIGN
    // §2 and profiles/r04_e_alloc_trials.jsonl give the measurements.
    int pad_alloc = 5;
    // Placement probe at creation (sm_place.cpp placement_probe): candidates
    // per streamed buffer (0 = no probe; sm_set_placement_probe, test option
    // place_probe=N), the pass time of the initial set and after each
    // buffer's search (us per pass), and which buffers moved (bit mask).
    int place_probe = 3;
    long place_min_mib = 256;       // smallest field (MiB) that is probed; test option probe_min_mib=N
    int place_n = 0, place_chosen = 0;
    double place_us[16] = {};       // the initial set, then one per buffer searched (up to 3 sweeps of 4)
    double *Uang = nullptr;         // 2V link codes (plane mu0 then mu1)
    double *Uang_face = nullptr;    // t-shards: codes of the 4-deep ghost links (16 Nx)
    hipStream_t own_stream = nullptr, stream = nullptr;
    hipStream_t comm_stream = nullptr;  // halo exchange overlapped with interior compute (hosted: == stream)
    bool own_comm_stream = false;       // comm_stream created by (and destroyed with) this context
    hipEvent_t ev_ready = nullptr, ev_halo = nullptr;
    // t-shard CG pass (split launches): the interior launch records ev_int at
    // its own end (hipExtLaunchKernelGGL), and the next pass's comm stream
    // waits on it instead of a marker behind it on the main stream; valid for
    // pass ev_int_pass only (-1: record the marker). kernel_events = 0 keeps
    // the markers (test option).
    hipEvent_t ev_int = nullptr;
    long ev_int_pass = -1;
    int kernel_events = 1;
    hipEvent_t ev_rccl = nullptr;   // orders an RCCL operation after the previous one on the other stream
    hipStream_t rccl_last = nullptr;  // stream of the last RCCL operation (sm_comm.cpp rccl_order)
    int rccl_ordered = 1;           // test option rccl_order=0: no ordering events (A/B)
    // t-shards: the edge block-columns run on the comm stream right after the
    // halo, concurrently with the interior launch on the main stream.
    // recompute-Ad CG on t-shards: the edge launch packs d_j's faces and the
    // exchange for pass j+1 is issued right behind it (cg_faces_for: the pass
    // whose d_{j-1} faces are already in flight); edge launch rows per block
    int cg_face_pipe = 1;
    int apply_split = 1;            // t-shard Dirac apply: interior / edge launches around the faces (0: faces first)
    int cg_edge_xchunk = -1;        // -1: by the residency rule (launch_cg_ra_pass)
    int cg_shard_blocks_per_cu[3] = {-1, -1, -1};  // occupancy of the t-shard pass by link form (-1: not asked yet)
    int n_cu = 256;                 // compute units of the device (residency of a launch)
    long cg_faces_for = -1;
    int cg_faces_packed = 0;        // face_pipe 2: cg_faces_for's faces are packed, not yet sent
    // recompute-Ad pass: ticketed tail (the pass's last block sums the partials
    // by groups of 64 and forms the scalars / the shard's sums), no scalar kernel
    int cg_tail = 1;
    int cg_red_shards = 1;          // t-shards: next pass's blocks evaluate the scalars from the all-reduced sums
    int cg_flush_sums = 0;          // the pending flush evaluates sc->sumr (t-shards), not partials
    unsigned *tick = nullptr;       // 1 + kMaxTickGroups counters, zeroed at creation
    double2 *gsum = nullptr;        // 3 per group
    ncclComm_t comm = nullptr;      // the context's one communicator; its operations in one total order
    // Device-initiated transport (sm_peer.h; sm_create_peer / sm_peer_connect,
    // sm_create_peer_loopback): every shard's region mapped here, kernels store
    // into the neighbours' regions and wait on flags in their own. One stream.
    bool peer = false;
    bool peer_connected = false;
    char *peer_region = nullptr;    // mine (uncached, IPC-exported)
    char *peer_open[sm::kPeerMaxRanks] = {};  // the others' regions as opened here (null: mine / not open)
    sm::PeerView peer_view{};       // host copy (kernel arguments)
    sm::PeerView *peer_view_dev = nullptr;  // device copy (the CG pass's tail)
    unsigned long long peer_coll_seq = 0, peer_face_seq = 0;  // the next collective / face exchange is seq + 1
    unsigned *peer_tick = nullptr;  // zeroed ticket counter of the transport kernels
    int peer_store = 0;             // CG pass face stores: 0 16-B write-through, 1 8-B atomic, 2 plain (test option)
    unsigned long long peer_wait_ticks = sm::kPeerWaitTicks;  // one wait's time limit (test option peer_wait_ms)
    // RCCL contexts: the recompute-Ad pass's scalar sums all-reduced in its own last
    // block through 4-KiB peer headers (sm_peer.h) instead of an ncclAllReduce per
    // pass; the halos stay RCCL (sm_comm.cpp rccl_peer_sums_setup). Test option
    // rccl_sums=1 keeps the ncclAllReduce.
    bool peer_sums = false;
    int peer_sums_wish = 1;
    int hosted_psums = 0;           // host-staged contexts: the same in-pass sums (test option hosted_psums=1)
    bool hosted = false;            // host-callback transport instead of RCCL
    sm_host_transport tr{};
    double *h_face = nullptr;       // pinned: send_lo, send_hi, recv_lo, recv_hi (4 x up to 8Nx doubles)
    double *h_red = nullptr;        // pinned: all-reduce staging (8 doubles)
    bool have_gauge = false;
    double2 *U = nullptr;          // 2V
    double2 *ghostU = nullptr;     // Nx: U_t at local t = -1 (lower neighbour's last column)
    double2 *fields[NFIELDS] = {};  // 2V each, one allocation per field (stream_alloc_bytes)
    double2 *faces = nullptr;      // 4 * 2Nx per spinor being exchanged (x2 for force)
    double2 *faces2 = nullptr;     // 2-deep faces: send lo/hi of 2 fields (4Nx each), recv d, r, U (8Nx each)
    double2 *faces4 = nullptr;     // 4-deep faces (sm_capi.cpp face4_*): send lo/hi, recv d x2 (by pass parity), U
    double2 *partials = nullptr;   // 2 * max(nparts)
    double2 *sums = nullptr;       // 4 complex scratch (allreduce)
    double *Fbuf = nullptr;        // 2V doubles (force)
    sm::CGScalars *sc = nullptr;       // device
    sm::CGScalars *h_sc = nullptr;     // pinned host mirror
    double2 *h_sums = nullptr;     // pinned host
    int nparts_dslash = 0, nparts_red = 0;
    // molecular dynamics (sm_md.cpp; allocated on first use)
    double2 *U_alt = nullptr;       // 2V: the other gauge buffer (leapfrog copy / kept conf)
    double *Pmd = nullptr;          // 2V: momenta
    double *Fmd = nullptr;          // 2V: MD force
    // even-odd action (sm_eo.cpp; allocated on first use)
    double2 *eo = nullptr;          // checkerboard work vectors, V complex each
    double2 *Ucb = nullptr;         // gauge field in checkerboard layout (even, odd)
    double2 *eo_faces = nullptr;    // t-sharded: checkerboard face slots (sm_eo.cpp)
    double2 *eo_faces4 = nullptr;   // t-sharded: 4-deep checkerboard face slots of the one-pass eo CG
    int eo_fused = 1;               // Dhat as one fused marching pass (0: two hop launches)
    int eo_cg_td = 1;               // even-odd CG: the one-pass two-direction kernel (sm_eotd.hip, one shard;
                                    // 0.54 vs 0.94 ms per iteration at 4096^2 for the six launches)
    int eo_cg_folded = 0;           // even-odd CG: 1 = 2 passes + scalars per iteration (opt-in:
                                    // measured slower than the 6 launches from 512^2 to 2048^2)
    // active CG
    double cg_mass = 0.0;
    const double2 *cg_phi = nullptr;
    double2 *cg_x = nullptr;        // the x the passes update: the caller's, or F_X (cg_x_user != null)
    double2 *cg_x_user = nullptr;   // the caller's x when the passes run on F_X (copied back by sm_cg_finish)
    bool x_internal = false;        // fields of >= 256 MiB: a solve runs on F_X (stream_alloc_bytes) and
                                    // copies x to the caller's buffer at sm_cg_finish
    int cg_active = 0;
    long cg_issued = 0;             // iterations enqueued since sm_cg_begin
    int cg_pending_x = 0;           // fused path: last x update deferred to sm_cg_finish

    double2 *field(int i) { return fields[i]; }
};

namespace sm_host {

using namespace sm;

// How many CG iterations to enqueue before the next status read. Kernels are
// no-ops once the device's `done` flag is set, so queueing past convergence
// costs empty launches and every status read costs a host round trip: predict
// the iterations left to the stop test from the residual's observed geometric
// rate, and stay a few percent past it.
struct CgChunker {
    int chunk = 4;
    int k_prev = -1;
    double err_prev = 0.0;
    int next(int k, double err, double target) {
        int c = chunk < 64 ? 2 * chunk : 64;
        if (k_prev >= 0 && k > k_prev && err_prev > 0.0 && err > 0.0 && err < err_prev && target > 0.0) {
            const double rate = std::pow(err / err_prev, 1.0 / (k - k_prev));
            if (rate < 1.0) {
                const double left = std::log(target / err) / std::log(rate);
                c = left <= 0.0 ? 2 : (int)std::ceil(left * 1.05) + 1;
                c = c < 2 ? 2 : (c > 256 ? 256 : c);
            }
        }
        k_prev = k;
        err_prev = err;
        chunk = c;
        return c;
    }
};

// Largest face exchanged, in doubles per x: 4 columns x 2 planes x complex.
constexpr size_t kMaxFaceDoubles = 16;

TFaces faces_for(sm_ctx *c, const double2 *in, const double2 *recv_lo, const double2 *recv_hi);
double2 *face_buf(sm_ctx *c, int set, int which);
int exchange_faces_on(sm_ctx *c, hipStream_t s, double2 *slo, double2 *shi, double2 *rlo, double2 *rhi,
                      size_t cnt);
// n independent face exchanges in ONE transport round (RCCL: one group of 4n
// point-to-point operations; the host-staged transport runs them in turn)
int exchange_faces_multi(sm_ctx *c, hipStream_t s, int n, double2 *const *slo, double2 *const *shi,
                         double2 *const *rlo, double2 *const *rhi, size_t cnt);
// RCCL contexts hold ONE communicator; every RCCL operation runs on the
// stream it is issued on, ordered on the GPU after the previous RCCL
// operation (sm_comm.cpp rccl_order), in host issue order -- the same
// sequence on every rank. n face exchanges in one group:
// send_up[i] -> up rank's recv_down[i], send_down[i] -> down rank's recv_up[i].
int rccl_p2p_group(sm_ctx *c, hipStream_t s, int n, const double2 *const *send_up, double2 *const *recv_down,
                   const double2 *const *send_down, double2 *const *recv_up, size_t cnt);
// shards 1..P-1 send cnt doubles to shard 0, which receives shard r's at recv + r*cnt
int rccl_gather_to0(sm_ctx *c, hipStream_t s, const double *send, double *recv, size_t cnt);
// waiter has waited for an event recorded on signaler after its last RCCL
// operation (a launch schedule's own join): no ordering event needed
void rccl_joined(sm_ctx *c, hipStream_t waiter, hipStream_t signaler);
int exchange_faces(sm_ctx *c, double2 *slo, double2 *shi, double2 *rlo, double2 *rhi, size_t cnt);
int allreduce_dev(sm_ctx *c, double *dev, int n);
int halo(sm_ctx *c, const double2 *field, int set, int kind, TFaces *f);  // kind: FaceKind
const double2 *loU(sm_ctx *c);
int apply(sm_ctx *c, const double2 *in, double2 *out, double mass, int dagger, const double2 *aux,
          double2 *partials, const CGScalars *skip);
int global_sum(sm_ctx *c, int nparts, const double2 *part, int slot);
// alpha (which = 0) / beta (1) from per-block partials: local sum, all-reduce, scalar
int cg_scalar(sm_ctx *c, int nparts, int which);
int check_ready(sm_ctx *c);
int upload_plane_pair(sm_ctx *c, double2 *dst, const double *p0, const double *p1);
int download_plane_pair(sm_ctx *c, const double2 *src, double *p0, double *p1);
double2 *face2_recv(sm_ctx *c, int which);  // 0: d, 1: r, 2: U, 3: Ad
double2 *face4_recv_U(sm_ctx *c);           // 4-deep ghost links (recompute-Ad CG)
bool cg_ra_ok(const sm_ctx *c);             // the recompute-Ad pass fits this shard (Wt >= 4 when sharded)
int exchange_ghost_U(sm_ctx *c);
// (sm_comm.cpp) the peer transport connected; the in-pass CG sums' headers of an
// RCCL / host-staged context (agreed over the shards; never fail on a local
// failure); the peer view and its handshake; the recompute-Ad pass's 4-deep
// faces: send buffers, receive slot of pass `pass`, pack + exchange into recv
int up_rank(const sm_ctx *c);    // t + 1 neighbour shard (periodic)
int down_rank(const sm_ctx *c);  // t - 1 neighbour shard
int peer_ready(const sm_ctx *c);
int rccl_peer_sums_setup(sm_ctx *c);
int hosted_peer_sums_setup(sm_ctx *c);
int peer_set_view(sm_ctx *c);
double2 *face4_send(sm_ctx *c, int hi);
double2 *face4_recv_d(sm_ctx *c, long pass);
int halo4(sm_ctx *c, hipStream_t s, const double2 *field, double2 *recv);
// the fused CG kernel's 2-deep faces of nf <= 3 fields in one transport round
// (receive buffers faces[f]); halo2: one field on the main stream
int halo2_multi(sm_ctx *c, hipStream_t s, const double2 *const *fields, double2 *const *faces, int nf);
int halo2(sm_ctx *c, const double2 *field, double2 *face);

// Streamed CG buffers and the placement probe (sm_place.cpp)
size_t stream_alloc_bytes(size_t bytes, size_t floor_bytes = size_t(2) << 30);
hipError_t stream_malloc(sm_ctx *c, void **p, size_t bytes);
void stream_free(sm_ctx *c, void *p);
size_t link_code_bytes(long n);           // codes of n links (sm_linkcode.h), flag words and flag bytes
int placement_probe(sm_ctx *c, size_t fb);
int placement_probe_default();            // candidates per buffer for new contexts

// even-odd preconditioned pseudofermion action (sm_eo.cpp); phi / chi in the
// full layout, only their even sites used
int eo_ready(sm_ctx *c);
int eo_md_force(sm_ctx *c, const sm_hmc_params *p, const double2 *phi_full, double *F, sm_cg_result *res);
int eo_fermion_action(sm_ctx *c, const sm_hmc_params *p, const double2 *phi_full, double *S, sm_cg_result *res);
int eo_pseudofermion(sm_ctx *c, const sm_hmc_params *p, const double2 *chi_full, double2 *phi_full);

}  // namespace sm_host
