"""Process-group glue for the t-sharded path (one process per GPU).

The data path between shards is RCCL inside libsm_hip.so (halos to t+-1,
scalar all-reduces). torch.distributed is control plane only:

* broadcast_unique_id(): rank 0 creates the RCCL unique id, everyone gets it;
* max_over_ranks():      bench timing (the slowest rank defines the step);
* GlooTransport:         the host-staged transport of sm_create_hosted(), so
                         several shards can share ONE GPU (tests) or run
                         without RCCL. Same kernels, same face protocol.

Face protocol (include/sm_hip.h, sm_host_transport): shard s sends its
t = Wt-1 column to s+1 (arriving there as recv_lo = its t = -1) and its t = 0
column to s-1 (arriving as recv_hi = its t = Wt); the lattice is periodic in
t over shards (the antiperiodic sign is applied by the owners of global t = 0
and t = Nt-1 inside the kernels).
"""
import ctypes

import numpy as np

from ._lib import SMError, check, lib

EXCHANGE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                               ctypes.c_void_p, ctypes.c_void_p, ctypes.c_long)
ALLREDUCE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_long)


class HostTransport(ctypes.Structure):
    _fields_ = [("user", ctypes.c_void_p), ("exchange", EXCHANGE_FN), ("allreduce_sum", ALLREDUCE_FN)]


def _arr(ptr, n):
    return np.ctypeslib.as_array(ctypes.cast(ptr, ctypes.POINTER(ctypes.c_double)), shape=(n,))


def neighbours(rank, world):
    """(down, up) shard ranks along t (periodic), include/mpi_setup.h:49-51 for ranks_x = 1."""
    return (rank - 1) % world, (rank + 1) % world


def exchange_faces(send_down, send_up, recv_lo, recv_hi):
    """Exchange two numpy face buffers with the t-1 / t+1 shards over torch.distributed."""
    import torch
    import torch.distributed as dist
    rank, world = dist.get_rank(), dist.get_world_size()
    down, up = neighbours(rank, world)
    tl, th = torch.from_numpy(recv_lo), torch.from_numpy(recv_hi)
    reqs = [dist.isend(torch.from_numpy(np.ascontiguousarray(send_up)), up, tag=11),
            dist.isend(torch.from_numpy(np.ascontiguousarray(send_down)), down, tag=12),
            dist.irecv(tl, down, tag=11),
            dist.irecv(th, up, tag=12)]
    for r in reqs:
        r.wait()


def allreduce_sum(buf):
    """In-place sum over ranks, reduced in rank order so every rank gets identical bits
    (all shards must take the same CG stop decision)."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size()
    t = torch.from_numpy(np.ascontiguousarray(buf))
    parts = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(parts, t)
    acc = parts[0].numpy().copy()
    for p in parts[1:]:
        acc = acc + p.numpy()
    buf[:] = acc


class GlooTransport:
    """sm_host_transport backed by torch.distributed (gloo). Keep the object alive
    as long as the context that uses it."""

    def __init__(self):
        self._ex = EXCHANGE_FN(self._exchange)
        self._ar = ALLREDUCE_FN(self._allreduce)
        self.struct = HostTransport(None, self._ex, self._ar)
        self.error = None

    def _exchange(self, user, sd, su, rl, rh, n):
        try:
            exchange_faces(_arr(sd, n), _arr(su, n), _arr(rl, n), _arr(rh, n))
            return 0
        except Exception as e:  # noqa: BLE001 -- no exceptions across the C boundary
            self._report(e)
            return 1

    def _allreduce(self, user, buf, n):
        try:
            allreduce_sum(_arr(buf, n))
            return 0
        except Exception as e:  # noqa: BLE001
            self._report(e)
            return 1

    def _report(self, e):
        import sys
        import traceback
        self.error = e
        traceback.print_exception(type(e), e, e.__traceback__, file=sys.stderr)


def create_hosted_context(Nx, Nt, device=0):
    """sm_create_hosted over the current torch.distributed group. Returns (ctx, transport)."""
    import torch.distributed as dist
    tr = GlooTransport()
    h = ctypes.c_void_p()
    check(lib.sm_create_hosted(ctypes.byref(h), Nx, Nt, dist.get_world_size(), dist.get_rank(), device,
                               ctypes.c_void_p(ctypes.addressof(tr.struct))))
    return h, tr


def create_peer_context(Nx, Nt, device=0):
    """sm_create_peer + sm_peer_connect over the current torch.distributed group:
    the region handles are all-gathered in rank order (control plane only; the
    data path is the device-initiated transport). Returns the context."""
    import torch.distributed as dist
    nb = lib.sm_peer_handle_bytes()
    buf = ctypes.create_string_buffer(nb)
    h = ctypes.c_void_p()
    err = None
    try:
        check(lib.sm_create_peer(ctypes.byref(h), Nx, Nt, dist.get_world_size(), dist.get_rank(), device, buf, nb))
    except Exception as e:  # noqa: BLE001 -- the all-gather below must still run on every rank
        err = e
    handles = [None] * dist.get_world_size()
    dist.all_gather_object(handles, bytes(buf.raw) if err is None else b"")
    if err is not None:
        raise err
    if any(len(x) != nb for x in handles):
        lib.sm_destroy(h)
        raise RuntimeError("peer transport: sm_create_peer failed on another rank")
    allh = ctypes.create_string_buffer(b"".join(handles), nb * len(handles))
    rc = lib.sm_peer_connect(h, allh, nb)
    if rc != 0:
        msg = lib.sm_last_error().decode(errors="replace")
        lib.sm_destroy(h)
        raise SMError(f"sm_hip error {rc}: {msg}")
    return h


def create_shard_context(Nx, Nt, device=0, transport="hosted"):
    """One t-shard of the current torch.distributed group on `device`, over the
    host-staged transport ("hosted": returns (ctx, transport object to keep
    alive)) or the peer transport ("peer": returns (ctx, None))."""
    if transport == "peer":
        return create_peer_context(Nx, Nt, device), None
    return create_hosted_context(Nx, Nt, device)


def broadcast_unique_id():
    """RCCL unique id created on rank 0 (needs a GPU there) and broadcast to all."""
    import torch.distributed as dist
    buf = ctypes.create_string_buffer(128)
    if dist.get_rank() == 0:
        check(lib.sm_comm_unique_id(buf, 128))
    obj = [bytes(buf.raw)]
    dist.broadcast_object_list(obj, src=0)
    return obj[0]


def max_over_ranks(values):
    """Elementwise max of a list of floats over all ranks (bench: slowest rank wins)."""
    import torch
    import torch.distributed as dist
    t = torch.tensor(list(values), dtype=torch.float64)
    if dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return [float(v) for v in t]
