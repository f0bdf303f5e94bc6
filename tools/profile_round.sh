#!/bin/bash
# Profile one bench configuration on the GPU box (run from the repo root under gpurun).
#   1. rocprofv3 --kernel-trace --stats over a short bench run (all kernels)
#   2. rocprofv3 --pmc SQ counters (8, one pass) over the same bench run
#   3. rocprofv3 --pmc FETCH_SIZE over the Hessian-only bench (own pass)
#   4. rocprofv3 --pmc WRITE_SIZE over the Hessian-only bench (own pass)
#   5-6. FETCH_SIZE / WRITE_SIZE over the full pipeline (every kernel's bytes:
#      profiles/<tag>_stage_bytes.csv; skipped with STAGE_BYTES=0)
# Outputs under gpurun_out/prof_<tag>_*/; tools/summarize_profiles.py (config
# #3) and tools/hessian_profile.py (any config) turn them into the committed
# profiles/ summaries.
#   bash tools/profile_round.sh <tag> [bench args for the config, e.g. --batch 1]
set -u
TAG=${1:-r01}
shift || true
STEPS=${STEPS:-5}
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
OUT=gpurun_out
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d $OUT/prof_${TAG}_kt -o run -- \
    python3 bench.py --steps $STEPS --warmup 1 --no-cpu --no-stream-peak "$@" > $OUT/prof_${TAG}_kt.json 2> $OUT/prof_${TAG}_kt.err || exit $?
timeout -s KILL 120 rocprofv3 --pmc $SQ -T -f csv -d $OUT/prof_${TAG}_sq -o run -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu --no-profile --no-stream-peak "$@" > $OUT/prof_${TAG}_sq.json 2> $OUT/prof_${TAG}_sq.err || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -T -f csv -d $OUT/prof_${TAG}_fetch -o run -- \
    python3 bench.py --hessian-only --steps $STEPS --warmup 1 --no-cpu --no-stream-peak "$@" > $OUT/prof_${TAG}_fetch.json 2> $OUT/prof_${TAG}_fetch.err || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -T -f csv -d $OUT/prof_${TAG}_write -o run -- \
    python3 bench.py --hessian-only --steps $STEPS --warmup 1 --no-cpu --no-stream-peak "$@" > $OUT/prof_${TAG}_write.json 2> $OUT/prof_${TAG}_write.err || exit $?
if [ "${STAGE_BYTES:-1}" != 0 ]; then
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -T -f csv -d $OUT/prof_${TAG}_fetchall -o run -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu --no-profile --no-stream-peak "$@" > $OUT/prof_${TAG}_fetchall.json 2> $OUT/prof_${TAG}_fetchall.err || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -T -f csv -d $OUT/prof_${TAG}_writeall -o run -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu --no-profile --no-stream-peak "$@" > $OUT/prof_${TAG}_writeall.json 2> $OUT/prof_${TAG}_writeall.err || exit $?
fi
echo PROFILE_DONE
