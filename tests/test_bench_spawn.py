"""bench.py --gpus N without a launcher: the parent spawns N rank
processes before anything touches the GPU, rank 0's JSON line is the only stdout line, a
failing rank stops the run with its status, and --gpus that disagrees with WORLD_SIZE
exits non-zero.  CPU only: the ranks here are tests/helpers/dist_probe.py over gloo,
started by the same bench.spawn_ranks that starts bench.py's ranks."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROBE = os.path.join(ROOT, "tests", "helpers", "dist_probe.py")


def _env(**kw):
    e = {k: v for k, v in os.environ.items()
         if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    e.update(kw)
    return e


def _spawn(n, env):
    code = ("import sys; sys.path.insert(0, %r); import bench; "
            "sys.exit(bench.spawn_ranks(%d, [%r], script=%r))" % (ROOT, n, str(n), PROBE))
    return subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                          timeout=180)


@pytest.mark.parametrize("n", [2, 3])
def test_spawn_ranks_gloo(n):
    r = _spawn(n, _env())
    assert r.returncode == 0, r.stderr
    lines = [x for x in r.stdout.splitlines() if x.strip()]
    # rank 0's JSON line only: every other stdout line of any rank went to stderr
    assert len(lines) == 1 and lines[0].startswith("{")
    assert "rank 0 stdout chatter" in r.stderr
    got = json.loads(lines[-1])
    assert got["ranks_seen"] == n and got["spawned"] == "1"
    assert sorted(map(tuple, got["ranks"])) == [(r_, r_) for r_ in range(n)]
    assert "rank 1 stdout chatter" in r.stderr


def test_spawn_ranks_failure_stops_all():
    r = _spawn(2, _env(PROBE_FAIL_RANK="1"))
    assert r.returncode == 3, (r.returncode, r.stderr)
    assert "stopping the others" in r.stderr
    assert not r.stdout.strip()


def test_gpus_world_mismatch_exits():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"],
                       env=_env(WORLD_SIZE="3", RANK="0", LOCAL_RANK="0"), capture_output=True,
                       text=True, timeout=120)
    assert r.returncode != 0 and "WORLD_SIZE=3" in r.stderr
    assert not r.stdout.strip()


def test_gpus_over_rccl_needs_gpus():
    # no GPU here: --gpus 2 over RCCL is refused before any rank starts
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"],
                       env=_env(), capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "needs 2 GPUs" in r.stderr
