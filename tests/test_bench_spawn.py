"""bench.py's rank spawner fails loudly (CPU, no GPU): a hung rank is ended at
the deadline with exit 124, a failing rank ends its siblings at once, and
healthy ranks return 0 (a rank stuck in ncclCommInitRank
or a mismatched collective must not hang the driver's multi-GPU run)."""
import os
import sys
import time

import pytest

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

CHILD = """
import os, sys, time
mode = sys.argv[1]
rank = int(os.environ["RANK"])
if mode == "ok":
    sys.exit(0)
if mode == "hang":
    time.sleep(3600)
if mode == "fail1":
    if rank == 1:
        sys.exit(3)
    time.sleep(3600)
"""


@pytest.fixture()
def child(tmp_path):
    p = tmp_path / "child.py"
    p.write_text(CHILD)
    return str(p)


def test_spawn_all_ok(child):
    assert bench.spawn_ranks(3, ["ok"], timeout=60, script=child) == 0


def test_spawn_hung_rank_hits_deadline(child):
    t = time.monotonic()
    assert bench.spawn_ranks(2, ["hang"], timeout=2, script=child) == 124
    assert time.monotonic() - t < 40


def test_spawn_failing_rank_ends_siblings(child):
    t = time.monotonic()
    assert bench.spawn_ranks(3, ["fail1"], timeout=600, script=child) == 3
    assert time.monotonic() - t < 40


def test_rank_watchdog_exits_124(tmp_path):
    import subprocess
    code = ("import sys; sys.path.insert(0, %r); import bench, time; bench.start_rank_watchdog(1.0); "
            "time.sleep(60)" % os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60)
    assert r.returncode == 124
    assert "no result after" in r.stderr
