#!/bin/bash
# Quick GPU iteration: selected pytest expression, then the default bench
# line and a kernel trace.  Every GPU step has its own time limit; the
# script stops at the first failure.
#   bash tools/gpu_quick.sh <tag> "<pytest -k expr or ''>" [bench args...]
set -u
TAG=$1; KEXPR=$2; shift 2
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
O=gpurun_out
if [ -n "$KEXPR" ]; then
    timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$KEXPR" \
        > $O/${TAG}_pytest.log 2>&1 || { tail -40 $O/${TAG}_pytest.log; exit 1; }
    tail -3 $O/${TAG}_pytest.log
fi
timeout -k 10 300 python3 bench.py --steps 20 --no-cpu "$@" > $O/${TAG}_bench.json 2> $O/${TAG}_bench.err || { tail -20 $O/${TAG}_bench.err; exit 1; }
cat $O/${TAG}_bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d $O/prof_${TAG}_kt -o run -- \
    python3 bench.py --steps 5 --warmup 1 --no-cpu "$@" > $O/prof_${TAG}_kt.json 2> $O/prof_${TAG}_kt.err || exit 1
f=$(ls $O/prof_${TAG}_kt/*/run_kernel_trace.csv $O/prof_${TAG}_kt/run_kernel_trace.csv 2>/dev/null | head -1); python3 tools/kstats.py $f | head -30
echo QUICK_DONE
