#!/bin/bash
set -u
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
DETAIL=1 timeout -k 10 200 python3 -u tools/desc_determinism.py 4 0 > gpurun_out/e8_ring6.log 2>&1; rc=$?; tail -60 gpurun_out/e8_ring6.log; exit $rc
