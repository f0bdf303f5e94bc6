#!/bin/bash
# describe ring race vs LDS footprint: ring 4 padded to 3 workgroups/CU, ring 6 padded to 2
set -u
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
O=gpurun_out
run() { local tag=$1; shift; echo "== $tag"; env "$@" timeout -k 10 150 python3 -u tools/desc_determinism.py 3 0 > $O/e7_$tag.log 2>&1; rc=$?; tail -3 $O/e7_$tag.log; [ $rc -eq 0 ]; }
run ring4pad SURFHIP_LIB_DIR=cuda-surf_amd/diag/ring4 SURFHIP_U2_LDSPAD=17408 || exit 1
run ring6pad SURFHIP_U2_LDSPAD=16384 || exit 1
run ring4 SURFHIP_LIB_DIR=cuda-surf_amd/diag/ring4 || exit 1
echo EXP7_DONE
