// dirac_operator_hip.cpp -- drop-in replacement for the reference's
//   src/dirac_operator.cpp      (D_phi, D_dagger_phi, D_D_dagger_phi,
//                                phi_dag_partialD_phi, I_number)
//   src/conjugate_gradient.cpp  (conjugate_gradient)
// of Fabian2598/SchwingerModel, with the reference's exact signatures
// (include/dirac_operator.h:8,71,80,87,93; include/conjugate_gradient.h:16),
// implemented on the MI355X C-ABI (include/sm_hip.h, libsm_hip.so).
//
// Build inside the reference tree instead of those two files, e.g.
//   g++ -std=c++20 -O3 -I<ref>/include -I<this repo>/include -c dirac_operator_hip.cpp
//   ... link with -L<this repo>/schwingermodel_amd -lsm_hip
// (INTEGRATION.md). It reads the same globals the reference reads: LV::Nx/Nt,
// mpi::{rank, rank2d, ranks_x, ranks_t, coords, width_x, width_t, maxSize,
// cart_comm}, CG::{tol, max_iter}.
//
// Decomposition. The GPU path shards along t only; any ranks_x x ranks_t grid
// of the reference works. The ranks_x ranks of one t-column (same coords[1])
// form a column communicator: their local blocks (x-major, n = x*width_t + t,
// include/variables.h Coords) concatenated in coords[0] order are exactly the
// column's full-x t-shard in the GPU layout, so the column leader
// (coords[0] == 0) gathers inputs with one MPI_Gather per plane, drives t-shard
// coords[1] of ranks_t on its GPU, and scatters the results back. GPUs used =
// ranks_t; ranks_x > 1 also keeps the reference's own gauge code away from its
// blocking self-send/recv along x (src/gauge_conf.cpp:57-61 with
// include/mpi_setup.h:50-52 when ranks_x = 1).
//
// Transport between the leaders (SM_DROPIN_TRANSPORT): "rccl" (RCCL over
// xGMI, one GPU per leader), "peer" (the device-initiated transport, the
// region handles all-gathered over MPI), "mpi" (host-staged: faces and the 6-double scalar
// sums through MPI_Sendrecv / MPI_Reduce + MPI_Bcast on the leaders'
// communicator, so several leaders may share one GPU), or "auto" (default):
// rccl when every node has at least as many GPUs as leaders, else mpi.
// Setup errors abort, like the reference's exit(1) (include/mpi_setup.h:7-19).
#include "conjugate_gradient.h"
#include "dirac_operator.h"
#include "sm_hip.h"

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <string>
#include <vector>

c_double I_number(0, 1);  // src/dirac_operator.cpp:3

namespace {

[[noreturn]] void die(const char *what) {
    std::cerr << "[sm_hip] " << what << ": " << sm_last_error() << std::endl;
    MPI_Abort(MPI_COMM_WORLD, 1);
    std::exit(1);
}

void call(int rc, const char *what) {
    if (rc != SM_OK) die(what);
}

struct Shim {
    sm_ctx *ctx = nullptr;
    MPI_Comm col = MPI_COMM_NULL;   // the ranks_x ranks of my t-column, rank = coords[0]
    MPI_Comm lead = MPI_COMM_NULL;  // the ranks_t column leaders, rank = coords[1] (leaders only)
    bool leader = false;
    int ncol = 1;                   // ranks_x
    int nshard = 1, shard = 0;
    long Vloc = 0, Vcol = 0;        // sites of my block / of my column's t-shard
    std::vector<double> U, a, b, c; // leader: column-gathered planes (2 per field)
    std::vector<double> lastU;      // every rank: the U block last uploaded (exact change test)
    bool have_gauge = false;
    sm_host_transport tr{};
};
Shim g;

// ---- host-staged transport over MPI (sm_create_hosted) ----------------------
// Face protocol of include/sm_hip.h: send_up -> shard+1 (its recv_lo),
// send_down -> shard-1 (its recv_hi).
int mpi_exchange(void *, const double *send_down, const double *send_up, double *recv_lo, double *recv_hi, long n) {
    const int up = (g.shard + 1) % g.nshard, down = (g.shard - 1 + g.nshard) % g.nshard;
    int rc = MPI_Sendrecv(send_up, (int)n, MPI_DOUBLE, up, 11, recv_lo, (int)n, MPI_DOUBLE, down, 11, g.lead,
                          MPI_STATUS_IGNORE);
    if (rc == MPI_SUCCESS)
        rc = MPI_Sendrecv(send_down, (int)n, MPI_DOUBLE, down, 12, recv_hi, (int)n, MPI_DOUBLE, up, 12, g.lead,
                          MPI_STATUS_IGNORE);
    return rc == MPI_SUCCESS ? 0 : 1;
}

// Global sum with identical bits on every shard (all shards must take the same
// CG stop decision): reduced on shard 0, then broadcast.
int mpi_allreduce(void *, double *buf, long n) {
    std::vector<double> sum(n);
    int rc = MPI_Reduce(buf, sum.data(), (int)n, MPI_DOUBLE, MPI_SUM, 0, g.lead);
    if (rc == MPI_SUCCESS && g.shard == 0) std::memcpy(buf, sum.data(), sizeof(double) * n);
    if (rc == MPI_SUCCESS) rc = MPI_Bcast(buf, (int)n, MPI_DOUBLE, 0, g.lead);
    return rc == MPI_SUCCESS ? 0 : 1;
}

std::string transport_choice(int local_leaders, int ndev) {
    const char *e = std::getenv("SM_DROPIN_TRANSPORT");
    std::string t = e ? e : "auto";
    if (t == "auto") t = local_leaders > ndev ? "mpi" : "rccl";
    if (t != "mpi" && t != "rccl" && t != "peer") {
        std::cerr << "[sm_hip] SM_DROPIN_TRANSPORT must be auto, peer, rccl or mpi" << std::endl;
        MPI_Abort(MPI_COMM_WORLD, 1);
    }
    return t;
}

Shim &shim() {
    if (g.col != MPI_COMM_NULL) return g;
    g.ncol = mpi::ranks_x;
    g.nshard = mpi::ranks_t;
    g.shard = mpi::coords[1];
    g.leader = mpi::coords[0] == 0;
    g.Vloc = mpi::maxSize;
    g.Vcol = (long)LV::Nx * mpi::width_t;
    MPI_Comm_split(mpi::cart_comm, mpi::coords[1], mpi::coords[0], &g.col);
    MPI_Comm_split(mpi::cart_comm, g.leader ? 0 : MPI_UNDEFINED, mpi::coords[1], &g.lead);
    g.lastU.assign((size_t)4 * g.Vloc, 0.0);
    if (!g.leader) return g;
    if (g.ncol > 1) {
        for (auto *v : {&g.U, &g.a, &g.b, &g.c}) v->assign((size_t)4 * g.Vcol, 0.0);
    }
    // one GPU per leader on a node: node-local leader index modulo the device count
    MPI_Comm node;
    int local = 0, nlocal = 1, ndev = 1;
    MPI_Comm_split_type(g.lead, MPI_COMM_TYPE_SHARED, g.shard, MPI_INFO_NULL, &node);
    MPI_Comm_rank(node, &local);
    MPI_Comm_size(node, &nlocal);
    MPI_Comm_free(&node);
    call(sm_device_count(&ndev), "sm_device_count");
    if (ndev < 1) ndev = 1;
    const int device = local % ndev;
    if (g.nshard == 1) {
        call(sm_create(&g.ctx, LV::Nx, LV::Nt, 1, 0, device, nullptr), "sm_create");
    } else if (const std::string t = transport_choice(nlocal, ndev); t == "mpi") {
        g.tr.user = nullptr;
        g.tr.exchange = mpi_exchange;
        g.tr.allreduce_sum = mpi_allreduce;
        call(sm_create_hosted(&g.ctx, LV::Nx, LV::Nt, g.nshard, g.shard, device, &g.tr), "sm_create_hosted");
    } else if (t == "peer") {
        // the device-initiated transport: the leaders all-gather their regions'
        // IPC handles over MPI (in shard order: g.lead ranks are coords[1])
        const int nb = sm_peer_handle_bytes();
        std::vector<char> mine((size_t)nb), all((size_t)nb * g.nshard);
        call(sm_create_peer(&g.ctx, LV::Nx, LV::Nt, g.nshard, g.shard, device, mine.data(), nb), "sm_create_peer");
        MPI_Allgather(mine.data(), nb, MPI_BYTE, all.data(), nb, MPI_BYTE, g.lead);
        call(sm_peer_connect(g.ctx, all.data(), nb), "sm_peer_connect");
    } else {
        unsigned char uid[128] = {0};
        if (g.shard == 0) call(sm_comm_unique_id(uid, sizeof uid), "sm_comm_unique_id");
        MPI_Bcast(uid, sizeof uid, MPI_BYTE, 0, g.lead);
        call(sm_create(&g.ctx, LV::Nx, LV::Nt, g.nshard, g.shard, device, uid), "sm_create");
    }
    return g;
}

const double *re(const c_double *p) { return reinterpret_cast<const double *>(p); }
double *re(c_double *p) { return reinterpret_cast<double *>(p); }

// Column gather / scatter of one plane (dpp doubles per site: 2 complex, 1 real).
// With ranks_x == 1 the leader works on the caller's arrays directly.
const double *gather(const double *mine, std::vector<double> &buf, size_t off, int dpp) {
    if (g.ncol == 1) return mine;
    const int cnt = (int)(g.Vloc * dpp);
    MPI_Gather(mine, cnt, MPI_DOUBLE, g.leader ? buf.data() + off : nullptr, cnt, MPI_DOUBLE, 0, g.col);
    return g.leader ? buf.data() + off : nullptr;
}
double *out_plane(double *mine, std::vector<double> &buf, size_t off) {
    return g.ncol == 1 ? mine : (g.leader ? buf.data() + off : nullptr);
}
void scatter(double *mine, std::vector<double> &buf, size_t off, int dpp) {
    if (g.ncol == 1) return;
    const int cnt = (int)(g.Vloc * dpp);
    MPI_Scatter(g.leader ? buf.data() + off : nullptr, cnt, MPI_DOUBLE, mine, cnt, MPI_DOUBLE, 0, g.col);
}

struct Planes {
    const double *p0, *p1;
};
Planes gather_spinor(const spinor &s, std::vector<double> &buf) {
    const size_t half = (size_t)2 * g.Vcol;
    return {gather(re(s.mu0), buf, 0, 2), gather(re(s.mu1), buf, half, 2)};
}
void scatter_spinor(spinor &s, std::vector<double> &buf) {
    const size_t half = (size_t)2 * g.Vcol;
    scatter(re(s.mu0), buf, 0, 2);
    scatter(re(s.mu1), buf, half, 2);
}

// The caller mutates U between calls (src/hmc.cpp:69-99), but also calls the
// operators many times on one U (a CG, then D^dag, then the force): U goes to
// the device only when some rank's block changed since the last upload
// (exact comparison against the kept copy, agreed over the column).
void upload(const spinor &U) {
    Shim &s = shim();
    const size_t n = (size_t)2 * s.Vloc;
    int same = s.have_gauge && !std::memcmp(s.lastU.data(), re(U.mu0), sizeof(double) * n) &&
               !std::memcmp(s.lastU.data() + n, re(U.mu1), sizeof(double) * n);
    int all_same = same;
    MPI_Allreduce(&same, &all_same, 1, MPI_INT, MPI_LAND, mpi::cart_comm);
    if (all_same) return;
    std::memcpy(s.lastU.data(), re(U.mu0), sizeof(double) * n);
    std::memcpy(s.lastU.data() + n, re(U.mu1), sizeof(double) * n);
    const Planes u = gather_spinor(U, s.U);
    if (s.leader) call(sm_upload_gauge(s.ctx, u.p0, u.p1), "sm_upload_gauge");
    s.have_gauge = true;
}

// out = op(in) for the Dirac operators (dagger 0/1, or 2 = D D^dag)
void apply(const spinor &U, const spinor &phi, spinor &Dphi, double m0, int which, const char *what) {
    upload(U);
    Shim &s = shim();
    const Planes in = gather_spinor(phi, s.a);
    if (s.leader) {
        const size_t half = (size_t)2 * s.Vcol;
        double *o0 = out_plane(re(Dphi.mu0), s.b, 0), *o1 = out_plane(re(Dphi.mu1), s.b, half);
        if (which == 2) call(sm_ddag(s.ctx, in.p0, in.p1, o0, o1, m0), what);
        else call(sm_dirac(s.ctx, in.p0, in.p1, o0, o1, m0, which), what);
    }
    scatter_spinor(Dphi, s.b);
}

}  // namespace

void D_phi(const spinor &U, const spinor &phi, spinor &Dphi, const double &m0) {
    apply(U, phi, Dphi, m0, 0, "D_phi");
}

void D_dagger_phi(const spinor &U, const spinor &phi, spinor &Dphi, const double &m0) {
    apply(U, phi, Dphi, m0, 1, "D_dagger_phi");
}

void D_D_dagger_phi(const spinor &U, const spinor &phi, spinor &Dphi, const double &m0) {
    apply(U, phi, Dphi, m0, 2, "D_D_dagger_phi");
}

re_field phi_dag_partialD_phi(const spinor &U, const spinor &left, const spinor &right) {
    re_field F(mpi::maxSize);
    upload(U);
    Shim &s = shim();
    const Planes l = gather_spinor(left, s.a), r = gather_spinor(right, s.b);
    if (s.leader) {
        call(sm_force(s.ctx, l.p0, l.p1, r.p0, r.p1, out_plane(F.mu0, s.c, 0), out_plane(F.mu1, s.c, s.Vcol)),
             "phi_dag_partialD_phi");
    }
    scatter(F.mu0, s.c, 0, 1);
    scatter(F.mu1, s.c, s.Vcol, 1);
    return F;
}

int conjugate_gradient(const spinor &U, const spinor &phi, spinor &x, const double &m0) {
    if (x.size != phi.size) x = phi;  // spinor::operator= reallocation semantics
    upload(U);
    Shim &s = shim();
    const Planes in = gather_spinor(phi, s.a);
    double st[2] = {0.0, 0.0};  // converged, residual
    if (s.leader) {
        const size_t half = (size_t)2 * s.Vcol;
        sm_cg_result r;
        call(sm_cg(s.ctx, in.p0, in.p1, out_plane(re(x.mu0), s.b, 0), out_plane(re(x.mu1), s.b, half), m0, CG::tol,
                   CG::max_iter, &r),
             "conjugate_gradient");
        st[0] = r.converged;
        st[1] = r.residual;
    }
    scatter_spinor(x, s.b);
    if (s.ncol > 1) MPI_Bcast(st, 2, MPI_DOUBLE, 0, s.col);
    if (st[0] == 0.0) {
        if (mpi::rank2d == 0)  // src/conjugate_gradient.cpp:64-65
            std::cout << "CG for DD^+ did not converge in " << CG::max_iter << " iterations"
                      << " Error " << st[1] << std::endl;
        return 0;
    }
    return 1;
}
