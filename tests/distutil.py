"""Launch tests/dist_worker.py as WORLD_SIZE local processes (gloo, 127.0.0.1)."""
import json
import os
import socket
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def run_world(mode, fixture, world, tmp_path, timeout=300, extra_env=None):
    port = free_port()
    result = os.path.join(str(tmp_path), f"{mode}_{fixture}_{world}.json")
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK=str(r),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), OMP_NUM_THREADS="1", **(extra_env or {}))
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "dist_worker.py"), mode, fixture, result],
                                      env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    outs = []
    try:
        for p in procs:
            out, _ = p.communicate(timeout=timeout)
            outs.append((p.returncode, out))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    for rc, out in outs:
        assert rc == 0, out[-3000:]
    with open(result) as f:
        return json.load(f)
