#!/bin/bash
# L2 / L1 hit counters of one bench run per pass (describe's bound, DESIGN 6
# item 32): TCC hits and misses; TCP requests to L2 and total accesses.
#   bash tools/l2_pass.sh <tag>
set -u
TAG=$1
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out
mkdir -p $OUT
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -T -f csv -d $OUT/prof_${TAG}_tcc -o run -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu --no-profile --no-stream-peak > $OUT/prof_${TAG}_tcc.json 2> $OUT/prof_${TAG}_tcc.err || exit $?
timeout -s KILL 120 rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum -T -f csv -d $OUT/prof_${TAG}_tcp -o run -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu --no-profile --no-stream-peak > $OUT/prof_${TAG}_tcp.json 2> $OUT/prof_${TAG}_tcp.err || exit $?
echo L2_PASS_DONE
