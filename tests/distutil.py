"""Launch tests/dist_worker.py as WORLD_SIZE local processes (gloo, 127.0.0.1)."""
import json
import os
import signal
import socket
import subprocess
import sys
import time

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
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), OMP_NUM_THREADS="1",
                   SM_WORKER_WATCHDOG=str(max(10, timeout - 20)), **(extra_env or {}))
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "dist_worker.py"), mode, fixture, result],
                                      env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    outs = []
    try:
        for p in procs:
            try:
                out, _ = p.communicate(timeout=timeout)
            except subprocess.TimeoutExpired:
                # a rank is stuck: every worker dumps its Python stack (faulthandler,
                # SIGUSR1) before it is killed, so the report names the call
                for q in procs:
                    if q.poll() is None:
                        q.send_signal(signal.SIGUSR1)
                time.sleep(2)
                for q in procs:
                    if q.poll() is None:
                        q.kill()
                tails = []
                for r, q in enumerate(procs):
                    out, _ = q.communicate()
                    tails.append(f"--- rank {r} (rc {q.returncode}) ---\n{(out or '')[-2500:]}")
                raise AssertionError(f"world {world} timed out after {timeout} s\n" + "\n".join(tails))
            outs.append((p.returncode, out))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    for rc, out in outs:
        assert rc == 0, out[-3000:]
    with open(result) as f:
        return json.load(f)
