"""Config #2 latency guard, in the module pytest
runs first among the GPU tests.

bench.py --batch 1 (one 1080p frame per step, BASELINE config #2) measured
0.19-0.21 ms per frame standalone in round 4 (profiles/r04i_config2_bench.json,
r04u_config2_*, r04ze_config2_*), but 0.33-0.35 ms when launched from the
test suite: conftest.py sets SURFHIP_HESS_GATHER=0 for the parity tests, the
bench subprocess inherited it, and its one-frame detector ran the streaming
Hessian kernels (15 waves for a frame) instead of the gather plan a 1-frame
detector picks.  The child now gets the environment a standalone caller has.
Round 5 brought the standalone figure to 0.122-0.131 ms (small-batch plan,
rank sort, no per-batch memsets: profiles/r05f/ab_ms2_*).  Boxes differ
(round 5 saw 0.122-0.131 ms on different boxes, and throughput spreads by a
few percent between boxes, README): the guard is 2x 0.13 ms, wide enough for
box-to-box spread, tight enough for the regressions it exists for (round 4's
leak cost 1.7x), and the test prints the box (device, clocks) with the
figure."""
from __future__ import annotations

import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CONFIG2_MS_REF = 0.13
CONFIG2_MS_GUARD = 2.0 * CONFIG2_MS_REF


def test_bench_config2_latency_guard():
    """bench.py --batch 1 (config #2): single-frame detect+describe latency
    stays under CONFIG2_MS_GUARD ms per frame."""
    env = {k: v for k, v in os.environ.items() if not k.startswith("SURFHIP_")}
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--batch", "1", "--steps", "1000",
                        "--warmup", "1000", "--no-cpu", "--no-exchange-probe", "--no-stream-peak"],
                       capture_output=True, text=True, timeout=240, cwd=REPO, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.strip()][0])
    assert line["config"]["workload"].startswith("config#2"), line["config"]
    box = line.get("device", {})
    print(f"config #2: {line['ms_per_step']} ms per frame on {box}")
    assert line["ms_per_step"] < CONFIG2_MS_GUARD, line["ms_per_step"]
