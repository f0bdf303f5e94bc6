#!/bin/bash
# Full GPU check of the current tree: GPU tests, a default bench line, then
# the profile passes (kernel trace + Hessian FETCH/WRITE) under a tag.
#   bash tools/round_check.sh <tag>
set -u
TAG=${1:-rXX}
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/rc_${TAG}_pytest.log 2>&1 || { tail -40 gpurun_out/rc_${TAG}_pytest.log; exit 1; }
tail -2 gpurun_out/rc_${TAG}_pytest.log
timeout -k 10 300 python -u bench.py > gpurun_out/rc_${TAG}_bench.json 2> gpurun_out/rc_${TAG}_bench.err || { tail -20 gpurun_out/rc_${TAG}_bench.err; exit 1; }
cat gpurun_out/rc_${TAG}_bench.json
bash tools/profile_round.sh ${TAG}
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > gpurun_out/rc_${TAG}_smoke.log 2>&1 || { tail -20 gpurun_out/rc_${TAG}_smoke.log; exit 1; }
tail -1 gpurun_out/rc_${TAG}_smoke.log
