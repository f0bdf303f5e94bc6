#!/bin/bash
# GPU tests only (optionally a -k filter / a file), one process, time-limited
set -u
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
T=${1:-tests}; K=${2:-}
if [ -n "$K" ]; then
  timeout -k 10 900 python -u -m pytest $T -m gpu -x -v --timeout 300 --timeout-method thread -k "$K" > gpurun_out/gt_pytest.log 2>&1 || { tail -40 gpurun_out/gt_pytest.log; exit 1; }
else
  timeout -k 10 900 python -u -m pytest $T -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gt_pytest.log 2>&1 || { tail -40 gpurun_out/gt_pytest.log; exit 1; }
fi
grep -E "PASSED|FAILED|ERROR" gpurun_out/gt_pytest.log | tail -40; tail -2 gpurun_out/gt_pytest.log
