#!/bin/bash
# describe determinism: batch repeated + single-frame, default (ring 6) and ring 4
set -u
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
O=gpurun_out
echo "== ring6"; timeout -k 10 150 python3 -u tools/desc_determinism.py 3 48 > $O/e5_ring6.log 2>&1; rc=$?; cat $O/e5_ring6.log | tail -12; [ $rc -eq 0 ] || exit 1
echo "== ring4"; SURFHIP_LIB_DIR=cuda-surf_amd/diag/ring4 timeout -k 10 150 python3 -u tools/desc_determinism.py 3 48 > $O/e5_ring4.log 2>&1; rc=$?; cat $O/e5_ring4.log | tail -12; [ $rc -eq 0 ] || exit 1
echo "== ur"; SURFHIP_DESC_UR=1 timeout -k 10 150 python3 -u tools/desc_determinism.py 3 48 > $O/e5_ur.log 2>&1; rc=$?; cat $O/e5_ur.log | tail -12; [ $rc -eq 0 ] || exit 1
echo EXP5_DONE
