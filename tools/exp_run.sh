#!/bin/bash
# experiment pass: selected GPU tests (-k expr), then kernel traces of the Hessian stage per SURFHIP_V0_SPLIT value
#   bash tools/exp_run.sh "<pytest -k expr or ->" v1 v2 ...
set -u
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
K=$1; shift
if [ "$K" != "-" ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$K" > gpurun_out/exp_pytest.log 2>&1 || { tail -30 gpurun_out/exp_pytest.log; exit 1; }
  tail -2 gpurun_out/exp_pytest.log
fi
bash tools/exp_v0.sh "$@"
