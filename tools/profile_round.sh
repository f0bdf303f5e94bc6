#!/bin/bash
# Profile the bench workload on the GPU box (run from the repo root under gpurun).
#   1. rocprofv3 --kernel-trace --stats over a short bench run (all kernels)
#   2. rocprofv3 --pmc FETCH_SIZE  over the Hessian-only bench (own pass)
#   3. rocprofv3 --pmc WRITE_SIZE  over the Hessian-only bench (own pass)
# Outputs under gpurun_out/prof_<tag>_*/; tools/summarize_profiles.py turns
# them into the committed profiles/ summaries.
set -u
TAG=${1:-r01}
STEPS=${STEPS:-5}
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
OUT=gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d $OUT/prof_${TAG}_kt -o run -- \
    python3 bench.py --steps $STEPS --warmup 1 --no-cpu > $OUT/prof_${TAG}_kt.json 2> $OUT/prof_${TAG}_kt.err || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -T -f csv -d $OUT/prof_${TAG}_fetch -o run -- \
    python3 bench.py --hessian-only --steps $STEPS --warmup 1 --no-cpu > $OUT/prof_${TAG}_fetch.json 2> $OUT/prof_${TAG}_fetch.err || exit $?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -T -f csv -d $OUT/prof_${TAG}_write -o run -- \
    python3 bench.py --hessian-only --steps $STEPS --warmup 1 --no-cpu > $OUT/prof_${TAG}_write.json 2> $OUT/prof_${TAG}_write.err || exit $?
echo PROFILE_DONE
