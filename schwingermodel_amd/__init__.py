"""schwingermodel_amd -- MI355X-native hot path of Fabian2598/SchwingerModel.

The Wilson-Dirac apply D, D^dagger, D D^dagger, the fermion-force bilinear
and the CG solve of (D D^dagger)^{-1} run as hand-written HIP kernels for
gfx950 inside libsm_hip.so (C-ABI: include/sm_hip.h). This package is the
thin host-side mirror of the reference's function interface, so that code
written against src/dirac_operator.cpp / src/conjugate_gradient.cpp reads the
same:

    reference (C++)                                   here (Python)
    D_phi(U, phi, Dphi, m0)          :24             D_phi(U, phi, Dphi, m0)
    D_dagger_phi(U, phi, Dphi, m0)   :247            D_dagger_phi(U, phi, Dphi, m0)
    D_D_dagger_phi(U, phi, Dphi, m0) :477            D_D_dagger_phi(U, phi, Dphi, m0)
    phi_dag_partialD_phi(U, l, r)    :486            phi_dag_partialD_phi(U, l, r)
    conjugate_gradient(U, phi, x, m0)  cg.cpp:4      conjugate_gradient(U, phi, x, m0)
    dot(x, y)              include/variables.h:181   dot(x, y)
    CG::tol, CG::max_iter  src/variables.cpp:35-38   CG.tol, CG.max_iter
    spinor / re_field      include/variables.h:54    spinor / re_field

The lattice geometry (the reference's compile-time NS/NT plus mpi::) is set
once with init(Nx, Nt, nshard, shard, device, unique_id). There is no CPU
fallback: without the HIP library or a GPU every call raises.
"""
import ctypes

import numpy as np

from ._lib import CGResult, HamiltonianTerms, HMCParams, HMCResult, HMCSummary, SMError, check, lib

__all__ = ["spinor", "re_field", "c_double", "I_number", "CG", "init", "lattice", "Lattice",
           "D_phi", "D_dagger_phi", "D_D_dagger_phi", "phi_dag_partialD_phi",
           "conjugate_gradient", "dot", "SMError", "CGResult", "lib", "check"]

c_double = complex
I_number = complex(0.0, 1.0)


class CG:
    """Mirror of namespace CG (src/variables.cpp:35-38; set in src/main.cpp:26-27)."""
    max_iter = 10000
    tol = 1e-10


def _vp(a):
    return ctypes.c_void_p(a.ctypes.data)


class spinor:
    """Reference spinor (include/variables.h:54): two complex<double> arrays."""

    def __init__(self, N=None):
        if N is None:
            N = lattice().V
        self.size = int(N)
        self.mu0 = np.zeros(self.size, dtype=np.complex128)
        self.mu1 = np.zeros(self.size, dtype=np.complex128)

    @classmethod
    def from_arrays(cls, mu0, mu1):
        s = cls.__new__(cls)
        s.mu0 = np.ascontiguousarray(mu0, dtype=np.complex128)
        s.mu1 = np.ascontiguousarray(mu1, dtype=np.complex128)
        s.size = s.mu0.size
        return s

    def copy(self):
        return spinor.from_arrays(self.mu0.copy(), self.mu1.copy())


class re_field:
    """Reference re_field (include/variables.h:102): two double arrays."""

    def __init__(self, N=None):
        if N is None:
            N = lattice().V
        self.size = int(N)
        self.mu0 = np.zeros(self.size, dtype=np.float64)
        self.mu1 = np.zeros(self.size, dtype=np.float64)


class Lattice:
    """One t-shard of an Nx x Nt lattice on one GPU (owns an sm_ctx)."""

    def __init__(self, Nx, Nt, nshard=1, shard=0, device=0, unique_id=None, loopback=False):
        self.Nx, self.Nt, self.nshard, self.shard, self.device = Nx, Nt, nshard, shard, device
        t0, Wt = ctypes.c_int(), ctypes.c_int()
        check(lib.sm_shard_plan(Nt, nshard, shard, ctypes.byref(t0), ctypes.byref(Wt)))
        self.t0, self.Wt = t0.value, Wt.value
        self.V = Nx * self.Wt
        h = ctypes.c_void_p()
        uid = None
        if unique_id is not None:
            uid = ctypes.create_string_buffer(bytes(unique_id), len(unique_id))
        if loopback == "peer":  # one shard through the t-shard path over the peer transport, to itself
            if nshard != 1:
                raise ValueError("loopback is one shard")
            check(lib.sm_create_peer_loopback(ctypes.byref(h), Nx, Nt, device))
        elif loopback:  # one shard through the t-shard path over a one-rank RCCL communicator
            if nshard != 1:
                raise ValueError("loopback is one shard")
            if uid is None:
                uid = ctypes.create_string_buffer(128)
                check(lib.sm_comm_unique_id(uid, 128))
            check(lib.sm_create_loopback(ctypes.byref(h), Nx, Nt, device, uid))
        else:
            check(lib.sm_create(ctypes.byref(h), Nx, Nt, nshard, shard, device, uid))
        self.ctx = h
        self.last_cg = CGResult()

    TRANSPORTS = {0: "none", 1: "hosted", 2: "rccl", 3: "peer"}

    def comm_info(self):
        """(transport, nranks, rank) as the context's transport reports them
        (sm_comm_info: ncclCommCount / ncclCommUserRank for RCCL)."""
        t, n, r = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        check(lib.sm_comm_info(self.ctx, ctypes.byref(t), ctypes.byref(n), ctypes.byref(r)))
        return self.TRANSPORTS[t.value], n.value, r.value

    def close(self):
        if self.ctx:
            lib.sm_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check_field(self, s, name):
        if s.mu0.size < self.V or s.mu1.size < self.V:
            raise ValueError(f"{name}: size {s.mu0.size} < local volume {self.V}")
        for a in (s.mu0, s.mu1):
            if not a.flags.c_contiguous:
                raise ValueError(f"{name}: arrays must be C-contiguous")

    def upload_gauge(self, U):
        self._check_field(U, "U")
        check(lib.sm_upload_gauge(self.ctx, _vp(U.mu0), _vp(U.mu1)))


_LATTICE = None


def init(Nx, Nt, nshard=1, shard=0, device=0, unique_id=None, loopback=False):
    """Set the lattice geometry (the reference's NS/NT + mpi:: setup).
    loopback=True: one shard driven through the multi-GPU (RCCL) code path."""
    global _LATTICE
    if _LATTICE is not None:
        _LATTICE.close()
    _LATTICE = Lattice(Nx, Nt, nshard, shard, device, unique_id, loopback)
    return _LATTICE


def lattice():
    if _LATTICE is None:
        raise SMError("call schwingermodel_amd.init(Nx, Nt, ...) first")
    return _LATTICE


def _apply(U, phi, Dphi, m0, dagger):
    L = lattice()
    L._check_field(phi, "phi")
    L._check_field(Dphi, "Dphi")
    L.upload_gauge(U)  # the caller may have changed U since the last call (src/hmc.cpp:69-99)
    check(lib.sm_dirac(L.ctx, _vp(phi.mu0), _vp(phi.mu1), _vp(Dphi.mu0), _vp(Dphi.mu1),
                       float(m0), dagger))


def D_phi(U, phi, Dphi, m0):
    """Dphi = D phi, eq. (34); src/dirac_operator.cpp:24."""
    _apply(U, phi, Dphi, m0, 0)


def D_dagger_phi(U, phi, Dphi, m0):
    """Dphi = D^dagger phi, eqs. (35)-(36); src/dirac_operator.cpp:247."""
    _apply(U, phi, Dphi, m0, 1)


def D_D_dagger_phi(U, phi, Dphi, m0):
    """Dphi = D D^dagger phi; src/dirac_operator.cpp:477."""
    L = lattice()
    L._check_field(phi, "phi")
    L._check_field(Dphi, "Dphi")
    L.upload_gauge(U)
    check(lib.sm_ddag(L.ctx, _vp(phi.mu0), _vp(phi.mu1), _vp(Dphi.mu0), _vp(Dphi.mu1), float(m0)))


def phi_dag_partialD_phi(U, left, right):
    """Fermion-force bilinear, eqs. (37)-(38); src/dirac_operator.cpp:486. Returns a re_field."""
    L = lattice()
    L._check_field(left, "left")
    L._check_field(right, "right")
    L.upload_gauge(U)
    F = re_field(L.V)
    check(lib.sm_force(L.ctx, _vp(left.mu0), _vp(left.mu1), _vp(right.mu0), _vp(right.mu1),
                       _vp(F.mu0), _vp(F.mu1)))
    return F


def dot(x, y):
    """sum_n x conj(y) over all shards; include/variables.h:181."""
    L = lattice()
    out = np.zeros(2)
    check(lib.sm_dot(L.ctx, _vp(x.mu0), _vp(x.mu1), _vp(y.mu0), _vp(y.mu1), _vp(out)))
    return complex(out[0], out[1])


def conjugate_gradient(U, phi, x, m0):
    """Solve D D^dagger x = phi (x0 = phi); src/conjugate_gradient.cpp:4.

    Returns 1 if converged, 0 otherwise (and prints the reference's message on
    shard 0). Details of the last solve are in lattice().last_cg.
    """
    L = lattice()
    L._check_field(phi, "phi")
    if x.mu0.size != phi.mu0.size:  # spinor::operator= reallocates, include/variables.h:73-86
        x.mu0 = np.zeros_like(phi.mu0)
        x.mu1 = np.zeros_like(phi.mu1)
        x.size = phi.size
    L.upload_gauge(U)
    res = CGResult()
    check(lib.sm_cg(L.ctx, _vp(phi.mu0), _vp(phi.mu1), _vp(x.mu0), _vp(x.mu1), float(m0),
                    float(CG.tol), int(CG.max_iter), ctypes.byref(res)))
    L.last_cg = res
    if not res.converged and L.shard == 0:
        print(f"CG for DD^+ did not converge in {CG.max_iter} iterations Error {res.residual}")
    return 1 if res.converged else 0
