#!/bin/bash
# Round-end check on one box: every -m gpu test, smoke(), the default bench
# line, then tools/profile_round.sh (kernel trace + FETCH/WRITE passes).
set -u
TAG=${1:-r04k}
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
O=gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
    > $O/${TAG}_pytest.log 2>&1 || { tail -60 $O/${TAG}_pytest.log; exit 1; }
tail -3 $O/${TAG}_pytest.log
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > $O/${TAG}_smoke.log 2>&1 || { tail -20 $O/${TAG}_smoke.log; exit 1; }
tail -1 $O/${TAG}_smoke.log
timeout -k 10 300 python3 bench.py > $O/${TAG}_bench_full.json 2> $O/${TAG}_bench_full.err || { tail -20 $O/${TAG}_bench_full.err; exit 1; }
head -c 1500 $O/${TAG}_bench_full.json; echo
bash tools/profile_round.sh $TAG || exit 1
echo FINAL_DONE
