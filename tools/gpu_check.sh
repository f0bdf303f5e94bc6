#!/bin/bash
# One GPU-box pass: parity tests, the default bench line, a kernel trace and
# an SQ counter pass over the Hessian stage.  Run from the repo root under
# gpurun; every GPU step has its own time limit and the script stops at the
# first failure.
#   bash tools/gpu_check.sh <tag> [skip-tests]
set -u
TAG=${1:-chk}
SKIP_TESTS=${2:-0}
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
O=gpurun_out
if [ "$SKIP_TESTS" = "0" ]; then
    timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
        > $O/${TAG}_pytest.log 2>&1 || { tail -30 $O/${TAG}_pytest.log; exit 1; }
    tail -3 $O/${TAG}_pytest.log
fi
timeout -k 10 300 python3 bench.py > $O/${TAG}_bench.json 2> $O/${TAG}_bench.err || { tail -20 $O/${TAG}_bench.err; exit 1; }
cat $O/${TAG}_bench.json
bash tools/ktrace.sh ${TAG} || exit 1
bash tools/pmc.sh ${TAG}_sq "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT" --hessian-only || exit 1
echo GPU_CHECK_DONE
