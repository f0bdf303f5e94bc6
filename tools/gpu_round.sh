#!/bin/bash
# Round check on the GPU box: every -m gpu test, the default bench line, the
# profiles of the three single-GPU configs, smoke.  Each GPU step has its own
# time limit; the script stops at the first failure.
#   bash tools/gpu_round.sh <tag> [skip-tests]
set -u
TAG=$1; SKIP=${2:-}
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
O=gpurun_out
if [ -z "$SKIP" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
      > $O/${TAG}_pytest.log 2>&1 || { tail -60 $O/${TAG}_pytest.log; exit 1; }
  tail -3 $O/${TAG}_pytest.log
fi
timeout -k 10 300 python3 bench.py > $O/${TAG}_bench.json 2> $O/${TAG}_bench.err || { tail -20 $O/${TAG}_bench.err; exit 1; }
cat $O/${TAG}_bench.json
bash tools/profile_configs.sh ${TAG} || exit $?
if [ -z "$SKIP" ]; then
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > $O/${TAG}_smoke.log 2>&1 || { tail -20 $O/${TAG}_smoke.log; exit 1; }
  tail -1 $O/${TAG}_smoke.log
fi
echo ROUND_DONE
