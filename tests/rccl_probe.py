"""Probe: can two RCCL ranks share one GPU on this box? (diagnostic, not a test)"""
import ctypes, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch.distributed as dist
dist.init_process_group("gloo")
import schwingermodel_amd as sm
from schwingermodel_amd import dist as smd
uid = smd.broadcast_unique_id()
h = ctypes.c_void_p()
rc = sm.lib.sm_create(ctypes.byref(h), 64, 64, dist.get_world_size(), dist.get_rank(), 0, uid)
print("rank", dist.get_rank(), "sm_create rc", rc, sm.lib.sm_last_error().decode(), flush=True)
if rc == 0:
    sm.lib.sm_destroy(h)
dist.barrier()
