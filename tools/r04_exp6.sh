#!/bin/bash
# describe ring race: determinism per variant
set -u
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
O=gpurun_out
for v in ring6if3 ring6if2 ring8; do
  echo "== $v"; SURFHIP_LIB_DIR=cuda-surf_amd/diag/$v timeout -k 10 150 python3 -u tools/desc_determinism.py 3 0 > $O/e6_$v.log 2>&1; rc=$?; tail -4 $O/e6_$v.log; [ $rc -eq 0 ] || exit 1
done
echo EXP6_DONE
