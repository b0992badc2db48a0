// dirac_operator_hip.cpp -- drop-in replacement for the reference's
//   src/dirac_operator.cpp      (D_phi, D_dagger_phi, D_D_dagger_phi,
//                                phi_dag_partialD_phi, I_number)
//   src/conjugate_gradient.cpp  (conjugate_gradient)
// of Fabian2598/SchwingerModel, with the reference's exact signatures
// (include/dirac_operator.h:8,71,80,87,93; include/conjugate_gradient.h:16),
// implemented on the MI355X C-ABI (include/sm_hip.h, libsm_hip.so).
//
// Build inside the reference tree instead of those two files, e.g.
//   hipcc -std=c++20 -O3 -I<ref>/include -I<this repo>/include -c dirac_operator_hip.cpp
//   ... link with -L<this repo>/schwingermodel_amd -lsm_hip
// (INTEGRATION.md). It reads the same globals the reference reads: LV::Nx/Nt,
// mpi::{size, rank2d, ranks_x, ranks_t, coords, maxSize, cart_comm}, CG::{tol, max_iter}.
//
// Decomposition: the GPU path shards along t only, so it needs ranks_x == 1
// (ranks_t = number of MPI ranks = number of GPUs); each rank drives the GPU
// (node-local rank mod device count). Setup errors abort, like the reference's exit(1)
// (include/mpi_setup.h:7-19); there is no other error channel.
#include "conjugate_gradient.h"
#include "dirac_operator.h"
#include "sm_hip.h"

#include <cstdio>
#include <cstdlib>
#include <iostream>

c_double I_number(0, 1);  // src/dirac_operator.cpp:3

namespace {

sm_ctx *g_ctx = nullptr;

[[noreturn]] void die(const char *what) {
    std::cerr << "[sm_hip] " << what << ": " << sm_last_error() << std::endl;
    MPI_Abort(MPI_COMM_WORLD, 1);
    std::exit(1);
}

void call(int rc, const char *what) {
    if (rc != SM_OK) die(what);
}

sm_ctx *ctx() {
    if (g_ctx) return g_ctx;
    if (mpi::ranks_x != 1) {
        std::cerr << "[sm_hip] the GPU path shards along t only: run with ranks_x = 1" << std::endl;
        MPI_Abort(MPI_COMM_WORLD, 1);
    }
    const int nshard = mpi::ranks_t, shard = mpi::coords[1];
    unsigned char uid[128] = {0};
    if (nshard > 1) {
        if (mpi::rank2d == 0) call(sm_comm_unique_id(uid, sizeof uid), "sm_comm_unique_id");
        MPI_Bcast(uid, sizeof uid, MPI_BYTE, 0, mpi::cart_comm);
    }
    // one GPU per rank: node-local rank modulo the visible device count
    MPI_Comm node;
    int local = 0, ndev = 1;
    MPI_Comm_split_type(MPI_COMM_WORLD, MPI_COMM_TYPE_SHARED, mpi::rank, MPI_INFO_NULL, &node);
    MPI_Comm_rank(node, &local);
    MPI_Comm_free(&node);
    call(sm_device_count(&ndev), "sm_device_count");
    const int device = local % (ndev > 0 ? ndev : 1);
    call(sm_create(&g_ctx, LV::Nx, LV::Nt, nshard, shard, device, nshard > 1 ? uid : nullptr), "sm_create");
    return g_ctx;
}

const double *re(const c_double *p) { return reinterpret_cast<const double *>(p); }
double *re(c_double *p) { return reinterpret_cast<double *>(p); }

// The caller mutates U between calls (src/hmc.cpp:69-99): upload every time.
void upload(const spinor &U) { call(sm_upload_gauge(ctx(), re(U.mu0), re(U.mu1)), "sm_upload_gauge"); }

}  // namespace

void D_phi(const spinor &U, const spinor &phi, spinor &Dphi, const double &m0) {
    upload(U);
    call(sm_dirac(ctx(), re(phi.mu0), re(phi.mu1), re(Dphi.mu0), re(Dphi.mu1), m0, 0), "D_phi");
}

void D_dagger_phi(const spinor &U, const spinor &phi, spinor &Dphi, const double &m0) {
    upload(U);
    call(sm_dirac(ctx(), re(phi.mu0), re(phi.mu1), re(Dphi.mu0), re(Dphi.mu1), m0, 1), "D_dagger_phi");
}

void D_D_dagger_phi(const spinor &U, const spinor &phi, spinor &Dphi, const double &m0) {
    upload(U);
    call(sm_ddag(ctx(), re(phi.mu0), re(phi.mu1), re(Dphi.mu0), re(Dphi.mu1), m0), "D_D_dagger_phi");
}

re_field phi_dag_partialD_phi(const spinor &U, const spinor &left, const spinor &right) {
    re_field F(mpi::maxSize);
    upload(U);
    call(sm_force(ctx(), re(left.mu0), re(left.mu1), re(right.mu0), re(right.mu1), F.mu0, F.mu1),
         "phi_dag_partialD_phi");
    return F;
}

int conjugate_gradient(const spinor &U, const spinor &phi, spinor &x, const double &m0) {
    if (x.size != phi.size) x = phi;  // spinor::operator= reallocation semantics
    upload(U);
    sm_cg_result r;
    call(sm_cg(ctx(), re(phi.mu0), re(phi.mu1), re(x.mu0), re(x.mu1), m0, CG::tol, CG::max_iter, &r),
         "conjugate_gradient");
    if (!r.converged) {
        if (mpi::rank2d == 0)  // src/conjugate_gradient.cpp:64-65
            std::cout << "CG for DD^+ did not converge in " << CG::max_iter << " iterations"
                      << " Error " << r.residual << std::endl;
        return 0;
    }
    return 1;
}
