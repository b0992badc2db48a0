/*
 * sm_hip.h -- C-ABI of the MI355X-native Wilson-Dirac / CG hot path
 * (libsm_hip.so). Plain pointers and sizes only; no HIP, RCCL or torch types.
 *
 * This is the drop-in boundary for Fabian2598/SchwingerModel's
 *   src/dirac_operator.cpp   (D_phi, D_dagger_phi, D_D_dagger_phi,
 *                             phi_dag_partialD_phi)
 *   src/conjugate_gradient.cpp (conjugate_gradient)
 *   include/variables.h:181-192 (dot)
 * Each entry point below names the reference function it replaces. A C++
 * shim with the reference's exact signatures (schwingermodel_amd/csrc/
 * dirac_operator_hip.cpp) is built on top of it; see INTEGRATION.md.
 *
 * Host field layout = the reference's spinor (include/variables.h:54-100):
 * for every field two separate arrays (mu0, mu1) of complex<double>, each
 * complex stored as (re, im) doubles, site n = x*Wt + t over this shard's
 * block (all Nx rows, Wt = Nt/nshard t-values starting at t0 = shard*Wt).
 * U: mu0 = U_t (mu = 0, t-direction), mu1 = U_x. re_field (force) = two
 * arrays of doubles.
 *
 * Device ("_dev") variants take ONE device buffer per field: plane mu0
 * followed by plane mu1 (2*Nx*Wt complex<double>), already resident in HBM.
 *
 * Multi-GPU: the lattice is sharded along t over nshard processes (one GPU
 * each), neighbours t+-1 exchanged over RCCL (xGMI). Every rank must call
 * every operator/CG entry point in lockstep, as in the reference (SPMD).
 *
 * Return codes: 0 = OK, nonzero = error (sm_last_error() describes it).
 * No C++ exceptions cross this boundary.
 */
#ifndef SM_HIP_H
#define SM_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SM_OK 0
#define SM_ERR_ARG 1    /* bad argument / geometry                      */
#define SM_ERR_HIP 2    /* HIP runtime error (incl. no GPU)             */
#define SM_ERR_RCCL 3   /* RCCL error                                   */
#define SM_ERR_STATE 4  /* call out of order (e.g. no gauge uploaded)   */

typedef struct sm_ctx sm_ctx;

/* CG outcome (the reference returns only 1/0; it also prints err on failure,
 * src/conjugate_gradient.cpp:64-65). */
typedef struct {
    int converged;     /* 1 = ||r|| < tol*||phi||, 0 = max_iter reached   */
    int iterations;    /* loop passes (D D^dag applications in the loop)  */
    double residual;   /* ||r|| of the last iteration (reference "err")    */
    double phi_norm;   /* ||phi||                                          */
} sm_cg_result;

/* ---- library / host-only helpers (no GPU needed) ------------------------ */
int sm_abi_version(void);
const char *sm_last_error(void);

/* t-shard geometry: replaces include/mpi_setup.h:6-23 (assignWidth) for the
 * ranks_x = 1, ranks_t = nshard decomposition. */
int sm_shard_plan(int Nt, int nshard, int shard, int *t0, int *Wt);

/* Counter-based synthetic fields: gauge U = exp(i theta),
 * theta ~ N(0, sigma^2) (sigma > 0), uniform (sigma < 0, "hot"), 0 ("cold");
 * spinor as HMC::RandomCHI (src/hmc.cpp:19-28). Writes rows [x0, x0+nx),
 * t in [t0, t0+Wt) of the global Nx x Nt_global field. */
void sm_fill_gauge(uint64_t seed, double sigma, int Nt_global, int x0, int nx, int t0, int Wt,
                   double *U0, double *U1);
void sm_fill_spinor(uint64_t seed, int Nt_global, int x0, int nx, int t0, int Wt, double *p0,
                    double *p1);

/* 28-byte-record binary gauge configuration (src/gauge_conf.cpp:378-423
 * SaveConf / :495-546 readBinary): per site x-major, t-minor, mu = 0,1:
 * int32 x, int32 t, int32 mu, float64 re, float64 im. Global field. */
int sm_conf_write(const char *path, int Nx, int Nt, const double *U0, const double *U1);
int sm_conf_read(const char *path, int Nx, int Nt, double *U0, double *U1);

/* Number of visible GPUs (0 and an error code when there is none). */
int sm_device_count(int *n);

/* RCCL unique id for nshard > 1 (rank 0 creates, all ranks receive it). */
int sm_comm_unique_id(void *id_out, int id_bytes);  /* id_bytes >= 128 */

/* ---- context -------------------------------------------------------------- */
/* One context = one t-shard on one GPU. unique_id is ignored for nshard == 1. */
int sm_create(sm_ctx **out, int Nx, int Nt_global, int nshard, int shard, int device,
              const void *unique_id);

/* Host-staged transport (instead of RCCL) for nshard > 1: halos and scalar
 * all-reduces go through caller callbacks on host buffers. Used to run several
 * shards on ONE GPU (tests: torch.distributed gloo) or over a caller's own
 * MPI; slower than RCCL, same kernels and the same results.
 *   exchange: send_up -> shard+1 (arrives there as recv_lo),
 *             send_down -> shard-1 (arrives there as recv_hi); n doubles each.
 *   allreduce_sum: in-place global sum of n doubles, identical on all shards. */
typedef struct {
    void *user;
    int (*exchange)(void *user, const double *send_down, const double *send_up, double *recv_lo,
                    double *recv_hi, long n);
    int (*allreduce_sum)(void *user, double *buf, long n);
} sm_host_transport;
int sm_create_hosted(sm_ctx **out, int Nx, int Nt_global, int nshard, int shard, int device,
                     const sm_host_transport *transport);
/* RCCL loopback: ONE shard (the whole lattice) driven through the t-shard code
 * path -- faces packed and exchanged with ncclSend/ncclRecv to itself, scalar
 * sums through ncclAllReduce -- over a one-rank communicator built from
 * unique_id (sm_comm_unique_id). The results equal sm_create's one-shard
 * context; it exists so the RCCL data path can be verified on a single GPU. */
int sm_create_loopback(sm_ctx **out, int Nx, int Nt_global, int device, const void *unique_id);
/* Device-initiated shard transport ("peer", round 6; replaces the halo
 * MPI_Send/MPI_Recv of src/dirac_operator.cpp:66-88 and the dot's
 * MPI_Allreduce of include/variables.h:190 like the RCCL path does, without
 * RCCL). Each shard owns one region of uncached device memory; kernels store
 * faces and scalar sums straight into the neighbours' / every shard's region
 * over xGMI and publish sequence flags there; the receiving kernel waits on
 * the flags in its own region (one waiting thread, a time limit on every
 * wait). The recompute-Ad CG pass writes d_j's faces into the neighbours'
 * rings and all-reduces its sums in its own last block, so a pass is ONE
 * launch on ONE stream. Works between processes on one GPU as well (the
 * one-GPU tests) and needs no RCCL communicator.
 * Two steps, with any host-side all-gather in between:
 *   sm_create_peer writes this shard's region handle (sm_peer_handle_bytes()
 *   bytes) to handle_out; sm_peer_connect takes the nshard handles in rank
 *   order (handle_bytes_each apart), maps the others' regions, and checks the
 *   world with one all-reduce. The context is unusable for sharded work until
 *   then. */
int sm_peer_handle_bytes(void);
int sm_create_peer(sm_ctx **out, int Nx, int Nt_global, int nshard, int shard, int device, void *handle_out,
                   int handle_bytes);
int sm_peer_connect(sm_ctx *ctx, const void *handles, int handle_bytes_each);
/* One shard through the peer transport's t-shard path, its own neighbour on
 * both sides (the peer counterpart of sm_create_loopback). */
int sm_create_peer_loopback(sm_ctx **out, int Nx, int Nt_global, int device);
/* Synchronises the context's stream; SM_ERR_RCCL if a peer-transport wait
 * timed out (*timed_out_seq = its sequence number, 0 if none; may be NULL).
 * sm_cg_finish checks it too. SM_OK on other transports. */
int sm_peer_status(sm_ctx *ctx, unsigned long long *timed_out_seq);
int sm_destroy(sm_ctx *ctx);
/* Launch on a caller stream (a hipStream_t, e.g. torch's current stream);
 * NULL restores the context's own stream. Synchronises the previous stream
 * first. A sharded context has ONE RCCL communicator and orders every RCCL
 * operation on the GPU after the previous one (events between this stream and
 * the context's private comm stream, which carries the faces that travel under
 * an interior launch), in issue order: no two of its RCCL kernels are ever in
 * flight at once. */
int sm_set_stream(sm_ctx *ctx, void *hip_stream);
/* The context's communication world, read from the transport itself:
 * transport 0 = none (one shard), 1 = host-staged (sm_create_hosted),
 * 2 = RCCL (sm_create with nshard > 1, or sm_create_loopback), 3 = peer
 * (sm_create_peer: *nranks / *rank = the shards its connected view holds and
 * this one's place in it; the peer loopback: 1 / 0); for RCCL *nranks /
 * *rank = ncclCommCount / ncclCommUserRank of the RCCL communicator, and
 * 1 / 0 without one (the RCCL world of a host-staged or one-shard context is
 * this process alone). Any output pointer may be NULL. */
int sm_comm_info(const sm_ctx *ctx, int *transport, int *nranks, int *rank);
/* 1 if the recompute-Ad CG pass of a sharded context all-reduces its scalar
 * sums in its own last block (the peer transport; RCCL contexts whose shards
 * agreed on the peer headers at creation), 0 if it calls the transport's
 * all-reduce after each pass. */
int sm_cg_sums_in_pass(const sm_ctx *ctx, int *in_pass);
int sm_synchronize(sm_ctx *ctx);
/* Launch-geometry knobs of the stencil kernels (tuning / A-B benchmarks):
 * bt = t-columns per block (64, 128, 256), xchunk = rows marched per block,
 * xcd_remap = 1 maps the tiles one XCD receives to x-adjacent tiles,
 * variant selects the stencil code variant. Values <= 0 (< 0 for xcd_remap
 * and variant) keep the current setting. */
int sm_tune(sm_ctx *ctx, int bt, int xchunk, int xcd_remap, int variant);
/* CG path: fused = 5 (the default from 256^2 sites per shard up) is the
 * two-direction iteration that recomputes
 * Ad_{j-1} = D D^dag d_{j-1} in-kernel instead of storing it (sm_cgra.hip):
 * 160 B/site. fused = 4 (the default on smaller shards) is the
 * two-direction one-pass iteration that stores Ad:
 * no r vector (r_{j-1} = d_{j-1} - beta_{j-2} d_{j-2} is rebuilt from the two
 * stored directions) and x updated on even passes only, 224 B/site.
 * fused = 0 is the reference's six-launch sequence (576 B/site). Other
 * values return SM_ERR_ARG (the two-pass and r-vector iterations of round 1
 * were dominated at every size and removed). xchunk = rows per block of the
 * active one-pass kernel. < 0 / <= 0 keep. */
int sm_tune_cg(sm_ctx *ctx, int fused, int xchunk);
/* Launch geometry of the recompute-Ad CG pass (fused = 5): waves per block
 * (1, 2 or 4; each wave owns 56 t-columns) and rows marched per block.
 * Values <= 0 keep the current setting. */
int sm_tune_cg_geometry(sm_ctx *ctx, int waves_per_block, int xchunk);
/* t-strip blocks of the recompute-Ad pass (one-shard contexts): strip = 1
 * makes each block's waves (4, or 2 after sm_tune_cg_geometry(ctx, 2, .))
 * march ONE strip of 64 * waves t-columns (8 of them halo; the stencil stages'
 * t-hops between its waves go through LDS) instead of one window of 56 owned
 * columns per wave; balanced = 1 splits x into XB equal chunks of
 * ~Nx/XB rows instead of xchunk-row chunks. < 0 keeps. SM_ERR_ARG on a
 * t-shard context. */
int sm_tune_cg_strip(sm_ctx *ctx, int strip, int balanced);
/* Compact links in the recompute-Ad CG pass (fused = 5, on by default from
 * 4M sites per shard): the pass reads each link as its smaller component v
 * (one double, exact) plus a 16-bit flag word -- which component v is, the
 * sign of the other, and the other's offset in ulps from sqrt(1 - v^2) -- and
 * rebuilds the link BITWISE in registers (schwingermodel_amd/csrc/
 * sm_linkcode.h): 20 instead of 32 B/site of links, 148 instead of 160 B/site
 * per iteration, and the same iterates as the complex-link pass. The codes are
 * rebuilt at the first solve after U changes, by a kernel that also decodes
 * every code with the pass's own decoder; they are used only if EVERY link
 * comes back bitwise (it does unless a link is off the unit circle by more
 * than ~1e-12 in |U|^2, far beyond the drift of the reference's leapfrog,
 * src/hmc.cpp:70-100), else the pass reads the complex links. D, D^dag and
 * the force always read the stored links. sm_cg_link_angles is the round-2
 * name of the same call (the code was then the link's angle). */
int sm_cg_link_codes(sm_ctx *ctx, int on, int *in_use);
/* Round-2 name of sm_cg_link_codes; same behaviour, kept for old callers.
 * on: 1 / 0 enable / disable, < 0 keep; *in_use (may be NULL): 1 if the last
 * sm_cg_begin / sm_cg set the codes up for the active path. The choice is
 * each context's own, also on t-shards: the codes are exact, so shards that
 * choose differently still compute bitwise the same iterates with the same
 * collectives (each shard checks its own links and the ghost links it
 * receives). */
int sm_cg_link_angles(sm_ctx *ctx, int on, int *in_use);
/* Bytes of link data per site the last CG pass launched on this context read,
 * recorded at its launch: 32 (complex links; every path but the recompute-Ad
 * pass), 20 (codes with 16-bit flag words) or 17 (codes with the flag
 * nibbles of both links packed into one byte, the form every field takes
 * whose ulp offsets all lie in [-2, 1], e.g. fresh exp(i theta) fields); 0
 * before the first pass. A later gauge upload or Metropolis reject does not
 * change it. The recompute-Ad pass streams 128 B/site besides. */
int sm_cg_link_bytes(const sm_ctx *ctx, int *bytes_per_site);
/* Diagnostic (tests): encode every link of the context's current U and decode
 * it again ON THE DEVICE with the CG pass's own functions. Writes the rebuilt
 * links to U_out_dev (device, the layout of sm_upload_gauge_dev; may be NULL),
 * the largest per-component |rebuilt - stored| to *max_err (0 when every link
 * comes back bitwise) and the count of links NOT rebuilt bitwise to *n_bad
 * (this shard only). Synchronous. */
int sm_link_code_check(sm_ctx *ctx, double *U_out_dev, double *max_err, long *n_bad);
/* Streaming-bandwidth ceiling on the ctx stream (measured roofline reference):
 * out = a + b (two_reads = 1: the stencil's 2-read/1-write byte mix) or
 * out = a, over n complex<double> device elements. */
int sm_bench_stream(sm_ctx *ctx, int two_reads, long n, const double *a, const double *b, double *out,
                    int blocks);
int sm_local_sites(const sm_ctx *ctx, long *V, int *Nx, int *Wt, int *t0);
/* Build id of this library: 16 hex digits of the SHA-256 of its sources,
 * headers and compile flags (schwingermodel_amd/build.py source_id). Profile
 * summaries under profiles/ record it, and bench.py cites only a summary of
 * the build that runs. */
const char *sm_build_id(void);
/* Placement probe of the context's creation (fields >= 256 MiB): the CG pass
 * runs at one of two speeds depending on where the driver physically places
 * its streamed buffers relative to each other, so creation searches one buffer
 * at a time (x, then the three direction buffers), trying up to
 * `candidates` fresh allocations of that buffer and keeping the fastest
 * (schwingermodel_amd/csrc/sm_place.cpp placement_probe; not on host-staged
 * contexts, where shard processes share one GPU); a sweep over the four
 * buffers that improved the pass by > 1 % is followed by another (at most 3).
 * *n = timings (0: no probe, else 1 + 4 per sweep), us_per_pass[0] (may be
 * NULL; room for 16) = median microseconds per pass of the initial placement,
 * us_per_pass[i] = after the search of the i-th buffer searched; *chosen = bit
 * mask of the buffers that moved, bit i = buffer i of the search order, whose
 * names sm_placement_buffer_name gives. */
int sm_placement_report(const sm_ctx *ctx, double *us_per_pass, int *n, int *chosen);
/* Name of bit i of sm_placement_report's mask ("x", "d1", "d0", "d2"; the
 * order the probe searches the buffers in), NULL past the last. */
const char *sm_placement_buffer_name(int i);
/* Candidates per buffer of the placement probe for contexts created after
 * this call (process-wide; default 3, 0 disables the probe, at most 8).
 * Transient memory while probing: that many allocations of one buffer.
 * SM_ERR_ARG for a value out of range, which leaves the setting as it was. */
int sm_set_placement_probe(int candidates);
/* The current process-wide setting of sm_set_placement_probe (callers that
 * change it temporarily restore this value). */
int sm_get_placement_probe(void);

/* Gauge field (host / device). Must precede every operator call; re-upload
 * whenever the caller changes U (the reference mutates U between calls,
 * src/hmc.cpp:69-99). */
int sm_upload_gauge(sm_ctx *ctx, const double *U0, const double *U1);
int sm_upload_gauge_dev(sm_ctx *ctx, const double *U_dev);

/* ---- operators, host pointers (drop-in; synchronous) ---------------------- */
/* D_phi (dagger = 0), src/dirac_operator.cpp:24; D_dagger_phi (dagger = 1), :247 */
int sm_dirac(sm_ctx *ctx, const double *in0, const double *in1, double *out0, double *out1,
             double m0, int dagger);
/* D_D_dagger_phi, src/dirac_operator.cpp:477 */
int sm_ddag(sm_ctx *ctx, const double *in0, const double *in1, double *out0, double *out1,
            double m0);
/* phi_dag_partialD_phi(U, left, right) -> re_field, src/dirac_operator.cpp:486 */
int sm_force(sm_ctx *ctx, const double *l0, const double *l1, const double *r0, const double *r1,
             double *F0, double *F1);
/* dot(a, b) = sum a conj(b) over all shards, include/variables.h:181. out = (re, im) */
int sm_dot(sm_ctx *ctx, const double *a0, const double *a1, const double *b0, const double *b1,
           double *out);
/* conjugate_gradient(U, phi, x, m0), src/conjugate_gradient.cpp:4: solves
 * D D^dag x = phi with x0 = phi and the stop test ||r|| < tol ||phi||. */
int sm_cg(sm_ctx *ctx, const double *phi0, const double *phi1, double *x0, double *x1, double m0,
          double tol, int max_iter, sm_cg_result *res);

/* ---- operators, device-resident fields (asynchronous on the ctx stream) --- */
int sm_dirac_dev(sm_ctx *ctx, const double *in, double *out, double m0, int dagger);
int sm_ddag_dev(sm_ctx *ctx, const double *in, double *out, double m0);
int sm_force_dev(sm_ctx *ctx, const double *l, const double *r, double *F);
int sm_dot_dev(sm_ctx *ctx, const double *a, const double *b, double *out_host); /* syncs */
int sm_cg_dev(sm_ctx *ctx, const double *phi, double *x, double m0, double tol, int max_iter,
              sm_cg_result *res);
/* Stepwise CG for benchmarking: begin (x = phi, r, d, norms), enqueue n
 * iterations without host synchronisation, then read the status (syncs). */
int sm_cg_begin(sm_ctx *ctx, const double *phi, double *x, double m0, double tol);
int sm_cg_iterate(sm_ctx *ctx, int n);
int sm_cg_status(sm_ctx *ctx, sm_cg_result *res);
/* End a stepwise solve: apply the x update the fused iteration defers to the
 * next pass (x += alpha_{k-1} d_{k-1}), then report like sm_cg_status. Until
 * then x lags one update behind the reference's x; on fields of 256 MiB and
 * more (4096^2 / 2 planes and up) the passes work on an internal x, and the
 * caller's x holds the solution only after this call. */
int sm_cg_finish(sm_ctx *ctx, sm_cg_result *res);

/* ==== gauge field, molecular dynamics and HMC =====
 * The next layer out from the Dirac/CG path: the whole MD force step of
 * src/hmc.cpp with U, momenta and forces resident on the device (the drop-in
 * shim above re-uploads U per call; these never do). Every sum is global over
 * shards (all ranks call in lockstep). Momenta: two planes of V doubles. */

/* Copy this shard's gauge field to the host (reference layout). */
int sm_download_gauge(sm_ctx *ctx, double *U0, double *U1);
/* Draw the gauge field on the device with the sm_fill_gauge generator
 * (sigma > 0 Gaussian angle, < 0 hot start as GaugeConf::initialization
 * src/gauge_conf.cpp:32-37, 0 cold). Same distribution as the host draw;
 * the device's log/sincos may differ from glibc in the last bit. */
int sm_fill_gauge_dev(sm_ctx *ctx, uint64_t seed, double sigma);

/* Compute_Plaquette01 + MeasureSp_HMC + Compute_gaugeAction
 * (src/gauge_conf.cpp:41-85, 430-453): *sp = sum_n Re U_01(n),
 * *gauge_action = sum_n beta Re(1 - U_01(n)). plaq (host, nullable) receives
 * this shard's U_01(n) field (V complex). */
int sm_plaquette(sm_ctx *ctx, double beta, double *sp, double *gauge_action, double *plaq);
/* GaugeConf::Compute_Staple (src/gauge_conf.cpp:89-373): both directions,
 * host output (reference spinor layout). */
int sm_staples(sm_ctx *ctx, double *S0, double *S1);
/* HMC::Force_G (src/hmc.cpp:31-40): F += -beta Im(U conj(staple)), host F. */
int sm_gauge_force(sm_ctx *ctx, double beta, double *F0, double *F1);

/* HMC parameters (src/main.cpp:19-27 inputs + the CG settings). */
typedef struct {
    double m0;          /* bare mass                                       */
    double beta;        /* gauge coupling                                  */
    double tau;         /* trajectory length                               */
    int md_steps;       /* leapfrog steps (the reference evaluates the force
                           md_steps - 1 times, src/hmc.cpp:76)             */
    double cg_tol;      /* CG::tol (1e-10 in src/main.cpp:27)              */
    int cg_max_iter;    /* CG::max_iter (10000)                            */
    uint64_t seed;      /* counter-based draws: momenta, sources, Metropolis */
    int even_odd;       /* 0: the reference's action phi^dag (DD^dag)^-1 phi;
                           1: the even-odd preconditioned action
                           phi_e^dag (Dhat Dhat^dag)^-1 phi_e, same gauge
                           distribution, one half-lattice CG per force
                           (even Nx and shard width, shards >= 4 wide;
                           see sm_eo_* below)                               */
} sm_hmc_params;

/* HMC::Force (src/hmc.cpp:44-60) at the current U: psi = (DD^dag)^-1 phi,
 * F = phi_dag_partialD_phi(U, psi, D^dag psi) + gauge force. res: the CG. */
int sm_md_force(sm_ctx *ctx, const sm_hmc_params *p, const double *phi0, const double *phi1, double *F0,
                double *F1, sm_cg_result *res);
int sm_md_force_dev(sm_ctx *ctx, const sm_hmc_params *p, const double *phi, double *F, sm_cg_result *res);
/* HMC::Leapfrog (src/hmc.cpp:63-101): evolves the context's U and the
 * momenta P (in/out) along one trajectory; *cg_iters = CG loop passes summed
 * over the force evaluations; *cg_failures = non-converged solves. */
int sm_leapfrog(sm_ctx *ctx, const sm_hmc_params *p, const double *phi0, const double *phi1, double *P0,
                double *P1, long *cg_iters, int *cg_failures);
int sm_leapfrog_dev(sm_ctx *ctx, const sm_hmc_params *p, const double *phi, double *P, long *cg_iters,
                    int *cg_failures);
/* HMC::Hamiltonian (src/hmc.cpp:104-148) at the current U:
 * H = sum 0.5 P^2 + (beta sum Re(1 - U_01) + Re dot((DD^dag)^-1 phi, phi)). */
typedef struct {
    double H;             /* the Hamiltonian                                */
    double kinetic;       /* sum 0.5 P^2                                    */
    double gauge_action;  /* beta sum Re(1 - U_01)                          */
    double fermion;       /* Re dot((DD^dag)^-1 phi, phi)                   */
    double sp;            /* sum Re U_01                                    */
    int cg_iterations;
    int cg_converged;
} sm_hamiltonian_terms;
int sm_hamiltonian(sm_ctx *ctx, const sm_hmc_params *p, const double *phi0, const double *phi1, const double *P0,
                   const double *P1, sm_hamiltonian_terms *out);
int sm_hamiltonian_dev(sm_ctx *ctx, const sm_hmc_params *p, const double *phi, const double *P,
                       sm_hamiltonian_terms *out);

/* One HMC update, HMC::HMC_Update (src/hmc.cpp:151-178), entirely on the
 * device: momenta and chi drawn for trajectory `traj` (counter-based, the
 * same on every rank), phi = D chi, leapfrog on a copy of U, Metropolis with
 * r = uniform(seed, traj) (identical on all ranks, no broadcast). On reject
 * the previous U is restored by a buffer swap. */
typedef struct {
    double H_old, H_new, dH;
    double r;              /* the Metropolis uniform                          */
    int accepted;
    double sp;             /* sum Re U_01 of the configuration kept           */
    double gauge_action;   /* beta sum Re(1 - U_01) of the configuration kept */
    long cg_iterations;    /* all solves: H_old, the forces, H_new            */
    int cg_failures;
} sm_hmc_result;
int sm_hmc_trajectory(sm_ctx *ctx, const sm_hmc_params *p, uint64_t traj, sm_hmc_result *out);

/* One pure-gauge (quenched) molecular-dynamics trajectory on the device:
 * HMC::Leapfrog (src/hmc.cpp:63-101, with its loop bound) driven by
 * HMC::Force_G alone (:31-40, p->beta), momenta drawn for `traj` as in
 * sm_hmc_trajectory; the evolved U is kept (no Metropolis step). No CG runs,
 * so it evolves large fields cheaply through the leapfrog's own link update
 * U <- U exp(i eps P), whose rounding moves |U| off 1 the way an HMC does
 * (bench.py times the CG on such a field). p->m0, cg_* and even_odd unused. */
int sm_quenched_trajectory(sm_ctx *ctx, const sm_hmc_params *p, uint64_t traj);

/* HMC::HMC_algorithm (src/hmc.cpp:181-213): optional hot start
 * (GaugeConf::initialization, drawn on the device), Ntherm thermalisation
 * updates, then Nmeas measurements of Sp and the gauge action separated by
 * Nsteps decorrelation updates. Ep = mean(Sp)/V, dEp = Jackknife_error(Sp,
 * 20)/V, gS and dgS likewise (src/statistics.cpp:4-34, restated with its
 * integer binning), V = Nx*Nt. Trajectories are numbered 0, 1, ... from
 * first_traj (the counter-based draws' key). acceptance = accepted /
 * (Nmeas + Nsteps*(Nmeas-1)): the updates of the measurement phase (the
 * reference's SimData value, src/main.cpp:169). sp_series / gs_series
 * (nullable, Nmeas doubles) receive the measured Sp / gauge action.
 * save_prefix (nullable): after measurement i, shard 0 writes
 * <save_prefix>_<i>.ctxt in the 28-byte record format (SaveConf). */
typedef struct {
    double Ep, dEp, gS, dgS;
    double acceptance;
    long accepted;          /* measurement-phase accepts                  */
    long trajectories;      /* all updates run                            */
    long cg_iterations;
    int cg_failures;
    int cg_link_bytes;      /* link bytes per site the CG pass read in the last
                               solve (sm_cg_link_bytes: 32 complex links, 20
                               codes + flag words, 17 codes + packed flags) */
} sm_hmc_summary;
int sm_hmc_run(sm_ctx *ctx, const sm_hmc_params *p, int hot_start, uint64_t first_traj, int Ntherm, int Nmeas,
               int Nsteps, const char *save_prefix, sm_hmc_summary *out, double *sp_series, double *gs_series);

/* Jackknife_error (src/statistics.cpp:25-34) with its binning as written:
 * bin blocks of n/bin samples; leftover samples only enter the mean. */
double sm_jackknife_error(const double *dat, int n, int bin);

/* Even-odd pieces, for tests and callers of the preconditioned action:
 * Dhat = m - (1/m) D_eo D_oe on the even sites (m = m0 + 2): out = Dhat in
 * (dagger = 0) or Dhat^dag in, on the even sites of full-layout fields (odd
 * sites of out are 0); sm_eo_cg solves Dhat Dhat^dag x = phi_e the same way.
 * t-sharded contexts exchange 2-column checkerboard faces per hop (SM_ERR_ARG
 * for odd Nx, odd shard width or shards narrower than 4). */
int sm_eo_dhat(sm_ctx *ctx, int dagger, const double *in0, const double *in1, double *out0, double *out1,
               double m0);
int sm_eo_cg(sm_ctx *ctx, const double *phi0, const double *phi1, double *x0, double *x1, double m0, double tol,
             int max_iter, sm_cg_result *res);

/* Gather the sharded gauge field to shard 0 (SaveConf's MPI_Gatherv,
 * src/gauge_conf.cpp:378-396): U0/U1 on shard 0 receive the global
 * Nx x Nt field (n = x*Nt + t); other shards may pass NULL. RCCL transport
 * or one shard only. */
int sm_gather_gauge(sm_ctx *ctx, double *U0, double *U1);

#ifdef __cplusplus
}
#endif
#endif
