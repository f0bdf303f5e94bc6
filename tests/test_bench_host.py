"""bench.py's host logic on the CPU (no GPU calls): the rank launcher's
argument checks and failure propagation, the config labels and the CPU
baseline's core accounting."""
from __future__ import annotations

import importlib.util
import os
import subprocess
import sys
import time

from conftest import REPO

BENCH = os.path.join(REPO, "bench.py")


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", BENCH)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(kw)
    return env


def test_world_size_mismatch_fails():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "4", "--batch", "1", "--steps", "1"],
                       capture_output=True, text=True, timeout=120, cwd=REPO,
                       env=_env(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0"))
    assert r.returncode == 2 and "disagrees" in r.stderr


def test_spawned_rank_failure_ends_the_job():
    """Without a GPU every spawned rank refuses the RCCL exchange (one GPU per
    rank); the launcher must return that failure, not hang or print a line."""
    t0 = time.time()
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--batch", "1", "--steps", "1", "--no-cpu"],
                       capture_output=True, text=True, timeout=240, cwd=REPO, env=_env())
    assert r.returncode == 2, (r.returncode, r.stderr[-2000:])
    assert "one GPU per rank" in r.stderr
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert time.time() - t0 < 200


def test_config_labels():
    b = _bench()

    class A:
        width, height, octaves, upright, extend, batch = 1920, 1080, 4, 1, 0, 256
    assert b.config_name(A, 1) == "config#3"
    assert b.config_name(A, 8) == "config#4"
    A.batch = 1
    assert b.config_name(A, 1) == "config#2"
    A.width, A.height, A.octaves, A.upright, A.extend, A.batch = 3840, 2160, 5, 0, 1, 64
    assert b.config_name(A, 8) == "config#5"
    assert b.config_name(A, 1).startswith("config#5 per-rank")
    A.octaves = 4
    assert b.config_name(A, 1) == "custom"


def test_cpu_share_reports_host():
    b = _bench()
    share, host = b.cpu_share()
    assert 1 <= share <= host["host_cpus"]
    assert share <= host["affinity_cpus"]
    assert host["cpu_model"]
