#!/bin/bash
# HBM bytes of the NMS scan and the integral fill (FETCH / WRITE passes)
set -u
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
bash tools/pmc_kern.sh nmsb k_ "FETCH_SIZE" "WRITE_SIZE" -- --no-pipeline || exit 1
echo EXP18_DONE
