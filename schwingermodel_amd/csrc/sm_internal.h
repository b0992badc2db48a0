// sm_internal.h -- private interface between the C-ABI host layer (sm_capi.cpp)
// and the gfx950 kernels (sm_kernels.hip). Not installed; include/sm_hip.h is
// the public boundary.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sm {

// Device field layout: the reference's SoA spinor, i.e.
// two planes of complex<double> (double2), plane stride V = Nx*Wt sites,
// site n = x*Wt + t (t fastest). U: plane 0 = U_t (mu=0), plane 1 = U_x.
// A face is one t-column for all x, stored [plane][x] (plane stride Nx).

// Neighbour sources of a t-domain. For one GPU (nshard == 1) the "faces" are
// aliases into the field itself (periodic wrap, xs = Wt); for a t-shard they
// are the received halo buffers (xs = 1).
struct TFaces {
    const double2 *lo;   // psi at local t = -1   : lo[x*lo_xs] (+ lo_ps for plane 1)
    const double2 *hi;   // psi at local t = Wt   : hi[x*hi_xs] (+ hi_ps for plane 1)
    long lo_xs, lo_ps, hi_xs, hi_ps;
    // proj = 1: spin-projected t-faces (t-shards), ONE complex per x and side:
    // hi = the forward hop's spin combination at t = Wt (D: p0 - p1, D^dag:
    // p0 + p1; force: l0 + l1 / r0 - r1), lo = the backward hop's whole product
    // conj(U_t(t = -1)) * combination (D: p0 + p1, D^dag: p0 - p1), formed by
    // the sending shard with its own link (launch_pack_faces_proj).
    int proj = 0;
};
enum FaceKind { FACE_D = 0, FACE_DDAG = 1, FACE_FORCE_L = 2, FACE_FORCE_R = 3 };

struct PeerView;  // sm_peer.h

struct Geometry {
    int Nx, Wt;          // local block (all x, Wt t-values)
    int t0, Ntg;         // global t offset of this shard, global Nt
    long V;              // Nx*Wt
};

// One-pass CG scalar state after evaluating one pass's partials (the
// redundant-scalar path of small grids keeps it per pass parity, sm_cgfused.hip).
struct CGRed {
    double2 rn, alpha, beta;
    double2 alpha2, beta2;   // alpha, beta of the pass before (two-direction CG)
    double err;
    int k, done, converged, pad;
};

// Scalars of one CG solve, resident on the device (no host round trip per
// iteration). Mirrors the locals of conjugate_gradient(),
// src/conjugate_gradient.cpp:6-14.
struct CGScalars {
    double2 rn;          // r_norm2 (complex, as the reference keeps it)
    double2 alpha, beta;
    double2 alpha2, beta2;  // two-direction CG: alpha_{j-1}, beta_{j-1} while alpha, beta are alpha_j, beta_j
    double2 sum;         // last globally reduced dot
    double phi_norm;     // sqrt(Re <phi,phi>)
    double tol;
    double err;          // sqrt(Re <r,r>) of the last iteration
    int k;               // iterations executed
    int done;            // 1 once converged: every later CG kernel is a no-op
    int converged;
    int max_iter;        // one-pass path: the device stops itself at k == max_iter
    double2 sum3[3];     // one-pass path, multi-shard: all-reduced <d,Ad>, <r,Ad>, (|r|^2,|Ad|^2)
    CGRed red[2];        // one-pass path, redundant scalars: state S_i in red[i & 1]; red[1] = S_-1
    double2 sumr[2][3];  // recompute-Ad pass on t-shards, redundant scalars: pass i's all-reduced sums in sumr[i & 1]
};

enum Epilogue { EPI_NONE = 0, EPI_DOT = 1 };

// ---- launchers (sm_kernels.hip) -------------------------------------------
struct LaunchCfg {
    int bt;              // threads per block along t (64/128/256)
    int xchunk;          // rows marched per block
    int xcd_remap;       // 1: consecutive tiles of one XCD are x-adjacent (L2 reuse of halo rows)
    int variant;         // dslash code variant (sm_kernels.hip)
};
constexpr int kMaxPartials = 1 << 16;
LaunchCfg dslash_config(const Geometry &g);

// out = D in (dagger=0) or D^dagger in (dagger=1). EPI_DOT additionally
// writes per-block partials of sum aux * conj(out) to `partials`.
void launch_dslash(hipStream_t s, const Geometry &g, const LaunchCfg &c, int dagger,
                   const double2 *in, double2 *out, const double2 *U, const double2 *loU,
                   const TFaces &f, double mass, const double2 *aux, double2 *partials,
                   const CGScalars *skip_if_done, int tb0 = 0, int tbn = -1);
int dslash_blocks(const Geometry &g, const LaunchCfg &c);

void launch_force(hipStream_t s, const Geometry &g, const double2 *U, const double2 *l,
                  const double2 *r, const TFaces &fl, const TFaces &fr, double *F);

int reduce_blocks(long n);   // grid size used by the BLAS-1 reductions of n complex
void launch_dot_partial(hipStream_t s, long n, const double2 *a, const double2 *b, double2 *partials);
void launch_sum_partials(hipStream_t s, int nparts, const double2 *partials, double2 *out);

void launch_copy(hipStream_t s, long n, const double2 *src, double2 *dst);
void launch_cg_init(hipStream_t s, long n, const double2 *phi, const double2 *Ax, double2 *r,
                    double2 *d, double2 *part_rr, double2 *part_pp);
void launch_cg_finalize_init(hipStream_t s, int nparts, const double2 *part_rr,
                             const double2 *part_pp, CGScalars *sc, double tol);
void launch_cg_alpha(hipStream_t s, int nparts, const double2 *part, CGScalars *sc);
void launch_cg_update_xr(hipStream_t s, long n, double2 *x, double2 *r, const double2 *d,
                         const double2 *Ad, CGScalars *sc, double2 *part);
void launch_cg_beta(hipStream_t s, int nparts, const double2 *part, CGScalars *sc);
void launch_cg_update_d(hipStream_t s, long n, double2 *d, const double2 *r, const CGScalars *sc);

// Multi-GPU helpers: partial -> local sum (into sc->sum) and global-sum
// consumers that take the already all-reduced value.
void launch_sum_to_scalar(hipStream_t s, int nparts, const double2 *part, CGScalars *sc);
void launch_cg_alpha_from_sum(hipStream_t s, CGScalars *sc);
void launch_cg_beta_from_sum(hipStream_t s, CGScalars *sc);
void launch_cg_init_from_sums(hipStream_t s, const double2 *rr_pp, CGScalars *sc, double tol);

// ---- fused CG iteration (sm_cgfused.hip) ----
constexpr int kFusedWaveCols = 60;  // output t-columns per wave (64 lanes - 2x2 halo)
struct CGFusedCfg {
    int NWT, TBk;        // wave tiles along t (60 columns each; 56 for sm_cgra.hip), blocks along t (4 waves)
    int xchunk, XB;      // rows per block, blocks along x
    int remap;
    int fold = 0;        // sm_cgra.hip: folded hopping-bracket arithmetic (dirac_bracket_folded)
    int wpb = 4;         // sm_cgra.hip: waves per block (1, 2, 4)
    int rev_odd = 0;     // sm_cgra.hip: odd one-shard tail passes march backwards over reversed tiles
    int strip = 0;       // sm_cgra.hip: the block's 4 waves share one t-strip (one shard; TBk = strips)
    int xbal = 0;        // sm_cgra.hip: XB balanced chunks of Nx / XB rows instead of xchunk-row chunks
};
CGFusedCfg cg_fused_config(const Geometry &g);
int cg_fused_blocks(const CGFusedCfg &c);
// The two-direction one-pass iteration with a stored Ad (mode 4): partials are
// 3 per block; d_{j-1} in dold, d_{j-2} in rold (faces fd / fr), Ad_{j-1} in aold.
void launch_cg_onepass(hipStream_t s, const Geometry &g, const CGFusedCfg &c, int nshard,
                       const double2 *dold, const double2 *rold, const double2 *aold, double2 *dnew,
                       double2 *anew, double2 *x, const double2 *U, const double2 *fd, const double2 *fr,
                       const double2 *fa, const double2 *fU, double mass, int first, CGScalars *sc,
                       double2 *partials, int tb0, int tbn,
                       const double2 *prev_partials = nullptr,  // != null: redundant scalars (see below)
                       long pass = 0);
// Two-direction pass that recomputes Ad_{j-1} = D D^dag d_{j-1} in-kernel
// instead of storing Ad (sm_cgra.hip): 160 B/site; d_i in d[i % 3] as below.
// Faces (t-shard, 4-deep [col -4..-1, Wt..Wt+3][plane][x]): f1 = d_{j-1},
// f2 = d_{j-2} (the previous pass's f1), fU = U.
constexpr int kRAWaveCols = 56;  // output t-columns per wave (64 lanes - 2x4 halo)
CGFusedCfg cg_ra_config(const Geometry &g);
// t-strip blocks on (strip = 1: 4 waves, 248 owned columns per block) or off;
// sets wpb / TBk accordingly and returns TBk
int cg_ra_set_strip(CGFusedCfg &c, const Geometry &g, int strip);
// Returns the link bytes per site the launched pass reads: 32 (complex links),
// 20 (codes, 16-bit flag words) or 17 (codes, packed flag bytes); 0 if nothing launched.
int launch_cg_ra(hipStream_t s, const Geometry &g, const CGFusedCfg &c, int nshard, const double2 *d1,
                 const double2 *d2, double2 *dn, double2 *x, const double2 *U, const double2 *f1,
                 const double2 *f2, const double2 *fU, double mass, long pass, CGScalars *sc, double2 *partials,
                 int tb0, int tbn, const double2 *prev_partials = nullptr, const double *Uang = nullptr,
                 const double *fUang = nullptr, double2 *fsend = nullptr, int pbase = 0,
                 unsigned *tick = nullptr, int ntiles = 0, double2 *gsum = nullptr, double2 *out3 = nullptr,
                 int red_sums = 0, int link_fmt = 1, double2 *fsendh = nullptr, const PeerView *peer = nullptr,
                 unsigned long long pseq = 0, int pstore = 0, int sched = 0, hipEvent_t stop = nullptr);
// Resident blocks per CU of the t-shard pass kernel at c's block size (0 if
// the runtime cannot tell); link_fmt 0 = complex links, 1 / 2 = the code forms.
int cg_ra_shard_blocks_per_cu(const CGFusedCfg &c, int link_fmt);
// (tick != null: ticketed tail over the ntiles tiles of every launch of the
// pass -- the last block forms the scalars in sc, or writes the shard's three
// sums to out3; tick holds 1 + ceil(ntiles / 64) zeroed counters, gsum 3 per group)
constexpr int kMaxTickGroups = 1024;
// (partial slot of a tile: pbase + (t-block - tb0) * XB + x-chunk; fsend (t-shards):
// the blocks owning columns 0..3 / Wt-4..Wt-1 also write d_j's 4-deep send
// faces, lo at fsend and hi at fsendh (default fsend + 8 Nx), as
// launch_pack_faces_k would; peer (device copy of the peer view): those faces
// go out as write-through system-scope stores (fsend / fsendh then point into
// the neighbours' regions) and the tail all-reduces the shard's sums itself,
// collective number pseq, into out3)
// Link codes of U for the passes above (Uang: 20 instead of 32 B/site of
// links, sm_linkcode.h): writes the codes v of n links to Ua[0, n) and their
// flag words to the n uint16 right after them, and per block the count of
// links the pass's decoder does NOT rebuild bitwise to partials; returns the
// block count.
int launch_link_codes(hipStream_t s, long n, const double2 *U, double *Ua, double2 *partials);
// Packed link flags (launch_cg_ra link_fmt 2): one byte per site holding the
// U_t and U_x flag nibbles, written after the flag words of the V-site code
// block / of the 4-deep face block (sm_linkcode.h sm_lc_nibble; only for
// fields whose every flag word fits a nibble)
void launch_link_nibbles(hipStream_t s, long V, const double *Ua);
void launch_face_nibbles(hipStream_t s, int Nx, const double *fUa);
// Diagnostic: encode + decode each of n links (the pass's functions) into
// out (may be null); per block (count not rebuilt bitwise, largest
// per-component error) to partials; returns the block count.
int launch_link_code_check(hipStream_t s, long n, const double2 *U, double2 *out, double2 *partials);
// Recompute-Ad CG: after the last pass add alpha_{k-1} d_{k-1} to the rows
// whose x update is still pending (parity != k & 1; x row = site / Wt).
void launch_cg_ra_finish_x(hipStream_t s, const Geometry &g, double2 *x, const double2 *d0, const double2 *d1,
                           const double2 *d2, const CGScalars *sc);
// prev_partials != null (one shard, fold 2): redundant scalars as in
// cg_onepass_kernel: every block evaluates pass j-1's scalars from its partials
// (cg1_redundant); the caller keeps the partials by pass parity and flushes.
// Pack the k-deep t-faces of a field: lo = columns 0..k-1, hi = columns Wt-k..Wt-1, [col][plane][x].
void launch_pack_faces_k(hipStream_t s, const Geometry &g, int k, const double2 *field, double2 *lo, double2 *hi);
// Two-direction form, after the last pass J = sc->k: if J is odd, x += alpha_{J-1} d_{J-1}
// (d_i lives in d[i % 3]).
void launch_cg_td_finish_x(hipStream_t s, long n, double2 *x, const double2 *d0, const double2 *d1,
                           const double2 *d2, const CGScalars *sc);
// Redundant scalars (small one-shard grids): pass j writes its partials (by
// pass parity) and every block of pass j + 1 evaluates them itself (fixed
// order, bitwise the same in every block) -- no ticket, no scalar launch.
// launch_cg1_flush evaluates the last issued pass's partials into sc for the
// host (idempotent: the next pass recomputes the same state).
void launch_cg1_flush(hipStream_t s, int nparts, const double2 *partials, CGScalars *sc, long pass);
// stored-Ad pass: redundant scalars up to this grid size (64^2: 64 blocks, 11.2 vs 12.0 us per
// iteration with a scalar ticket; 128^2 11.6 vs 12.9 us)
constexpr int kRedundantMaxBlocks = 128;
void launch_cg1_scalars(hipStream_t s, int nparts, const double2 *partials, CGScalars *sc, int first);
void launch_cg1_local_sum(hipStream_t s, int nparts, const double2 *partials, CGScalars *sc);
// t-shard redundant scalars (sm_cgra.hip): S_J of the last issued pass J from its all-reduced sums
void launch_cg_ra_flush_sums(hipStream_t s, CGScalars *sc, long pass);
void launch_cg1_from_sums(hipStream_t s, CGScalars *sc, int first);
void launch_pack_faces2(hipStream_t s, const Geometry &g, const double2 *field, double2 *lo,
                        double2 *hi);

void launch_stream(hipStream_t s, int two, long n, const double2 *a, const double2 *b, double2 *out,
                   int blocks);

// ---- gauge field / molecular dynamics (sm_gauge.hip) ----
// fU: the 2-deep U faces (nshard > 1; ignored for one shard, which wraps).
int gauge_reduce_blocks(const Geometry &g);
void launch_plaquette(hipStream_t s, const Geometry &g, int nshard, const double2 *U, const double2 *fU,
                      double beta, double2 *field, double2 *partials);
void launch_staple_force(hipStream_t s, const Geometry &g, int nshard, const double2 *U, const double2 *fU,
                         double beta, double *F, double2 *staples);
void launch_md_update(hipStream_t s, const Geometry &g, double2 *U, double *P, const double *F, double eps,
                      int do_p, double coef);
void launch_kinetic(hipStream_t s, const Geometry &g, const double *P, double2 *partials);
void launch_draw_momenta(hipStream_t s, const Geometry &g, uint64_t seed, double *P);
void launch_draw_source(hipStream_t s, const Geometry &g, uint64_t seed, double2 *chi);
void launch_draw_gauge(hipStream_t s, const Geometry &g, uint64_t seed, double sigma, double2 *U);

// ---- even-odd checkerboard (sm_eo.hip) ----
void launch_to_cb(hipStream_t s, const Geometry &g, const double2 *full, double2 *e, double2 *o);
void launch_from_cb(hipStream_t s, const Geometry &g, const double2 *e, const double2 *o, double2 *full);
// Received t-faces of checkerboard fields ([side][plane][col][x], 8*Nx
// complex each; sm_eo.hip); all null on one shard (periodic wrap).
struct EoFaces {
    const double2 *v = nullptr, *ue = nullptr, *uo = nullptr;
};
void launch_pack_cb_faces(hipStream_t s, const Geometry &g, const double2 *f, double2 *out);
// out_p = a*aux_p + b*H in_q (H: the hopping bracket of D / D^dag), parity p;
// inf / uqf: faces of `in` and Uq when t-sharded (else null)
void launch_eo_hop(hipStream_t s, const Geometry &g, int dagger, int p, const double2 *in, const double2 *Up,
                   const double2 *Uq, const double2 *aux, double a, double b, double2 *out,
                   const double2 *inf = nullptr, const double2 *uqf = nullptr);
// Fused Dhat / Dhat^dag (both hops in one marching pass); aux != null adds
// per-block partials of sum aux * conj(out) (eo_fused_blocks of them).
struct EoFusedCfg {
    int NWT, TBk, xchunk, XB;
};
EoFusedCfg eo_fused_config(const Geometry &g);
int eo_fused_blocks(const EoFusedCfg &c);
void launch_eo_dhat_fused(hipStream_t s, const Geometry &g, const EoFusedCfg &c, int dagger, const double2 *v,
                          const double2 *Ue, const double2 *Uo, double mass, double2 *out, const double2 *aux,
                          double2 *partials, const EoFaces &f);

// Folded even-odd CG iteration j (sm_eo.hip, eo_dhat_fused_kernel MODE 1/2):
// which = 0: pass A (r_j, d_j, x update; W = Dhat^dag d_j; partial |r_j|^2),
// which = 1: pass B (Ad_j = Dhat W; <d_j,Ad_j>, <r_j,Ad_j>, |Ad_j|^2). The 3
// partials per block feed launch_cg1_scalars (sm_cgfused.hip).
struct EoCgPass {
    const double2 *dold, *rold;
    double2 *dnew, *rnew, *x, *W, *ad;
    const double2 *rf = nullptr, *af = nullptr, *wf = nullptr;  // t-sharded faces of rold, ad, W
    int first;
};
void launch_eo_cg_pass(hipStream_t s, const Geometry &g, const EoFusedCfg &c, int which, const EoCgPass &q,
                       const double2 *Ue, const double2 *Uo, double mass, const EoFaces &f, CGScalars *sc,
                       double2 *partials);

// One-pass even-odd CG iteration on Dhat Dhat^dag (sm_eotd.hip, one shard):
// the two-direction recurrence, four checkerboard hops in registers; 3
// partials per block ((|W|^2, 0), <r,Ad>, (|r|^2, |Ad|^2)) for cg1_scalars.
constexpr int kEoTdWaveCols = 56;
struct EoTdCfg {
    int NWT, TBk, xchunk, XB;
};
EoTdCfg eo_td_config(const Geometry &g);
int eo_td_blocks(const EoTdCfg &c);
// t-shards: 4-deep checkerboard faces ([side][plane][col][x], 16*Nx complex)
// of d_{j-1}, d_{j-2}, Ad_{j-1} and both link parities; all null on one shard.
struct EoTdFaces {
    const double2 *d1 = nullptr, *d2 = nullptr, *ad = nullptr, *ue = nullptr, *uo = nullptr;
};
void launch_eo_td(hipStream_t s, const Geometry &g, const EoTdCfg &c, const double2 *d1, const double2 *d2,
                  const double2 *aold, double2 *dn, double2 *anew, double2 *x, const double2 *Ue, const double2 *Uo,
                  double mass, long pass, CGScalars *sc, double2 *partials, const EoTdFaces &f,
                  unsigned *tick = nullptr, double2 *gsum = nullptr, double2 *out3 = nullptr,  // tick: ticketed tail
                  int red = 0);  // red: t-shard scalars from sc->sumr (out3 = this pass's sumr slot)
void launch_pack_cb_faces4(hipStream_t s, const Geometry &g, const double2 *f, double2 *out);

// Pack the t = 0 and t = Wt-1 columns (both planes) into contiguous faces.
void launch_pack_faces(hipStream_t s, const Geometry &g, const double2 *field, double2 *lo_face,
                       double2 *hi_face);
// Spin-projected faces (TFaces::proj) of `field` for the operator `kind`:
// lo_face (my t = 0, sent down) = the forward combination, hi_face (my
// t = Wt-1, sent up) = conj(U_t) * the backward combination; Nx complex each.
void launch_pack_faces_proj(hipStream_t s, const Geometry &g, const double2 *field, const double2 *U, int kind,
                            double2 *lo_face, double2 *hi_face);

// ---- device-initiated shard transport (sm_peer.hip, layout in sm_peer.h) ----
// n (<= 3) face exchanges of cnt doubles per field and side, as exchange_faces_on:
// slo[f] goes down (arriving as the receiver's rhi[f]), shi[f] up (its rlo[f])
struct PeerXfer {
    const double *slo[3], *shi[3];
    double *rlo[3], *rhi[3];
    int n;
    long cnt;
};
// in-place sum of n <= 8 doubles over every shard, in rank order
void launch_peer_allreduce(hipStream_t s, double *dev, int n, const PeerView &v, unsigned long long seq);
// the exchange through the receivers' mailboxes (two kernels; tick: a zeroed counter)
void launch_peer_exchange(hipStream_t s, const PeerXfer &x, const PeerView &v, unsigned long long seq,
                          unsigned *tick);
// launch_pack_faces_proj's faces stored into the neighbours' apply slot seq % 4, then the handoff
void launch_peer_pack_proj(hipStream_t s, const Geometry &g, const double2 *field, const double2 *U, int kind,
                           const PeerView &v, unsigned long long seq, unsigned *tick);
void launch_peer_put(hipStream_t s, const double *src, long cnt, double *dst_remote);
void launch_peer_get(hipStream_t s, const double *src_local, long cnt, double *dst);

}  // namespace sm
