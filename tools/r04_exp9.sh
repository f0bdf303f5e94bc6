#!/bin/bash
set -u
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
O=gpurun_out
for v in if0 narrowonly forcewide dualonly; do
  echo "== $v"; SURFHIP_LIB_DIR=cuda-surf_amd/diag/$v timeout -k 10 150 python3 -u tools/desc_determinism.py 3 0 > $O/e9_$v.log 2>&1; rc=$?; grep -E "^run|^single" $O/e9_$v.log; [ $rc -eq 0 ] || exit 1
done
echo EXP9_DONE
