#!/bin/bash
# describe ring WAR fix: determinism (ring 6 default, ring 4 padded to 2 WG/CU, ring 8), then timing
set -u
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
O=gpurun_out
export SURFHIP_DESC_U2=1
run() { local tag=$1; shift; echo "== $tag"; env "$@" timeout -k 10 150 python3 -u tools/desc_determinism.py 4 0 > $O/e10_$tag.log 2>&1; rc=$?; grep -E "^run|^single" $O/e10_$tag.log; [ $rc -eq 0 ]; }
run ring6 SURFHIP_X=1 || exit 1
run ring4pad SURFHIP_LIB_DIR=cuda-surf_amd/diag/ring4 SURFHIP_U2_LDSPAD=17408 || exit 1
run ring8 SURFHIP_LIB_DIR=cuda-surf_amd/diag/ring8 || exit 1
bash tools/diag_run.sh k_describe default ring4 ring8 || exit 1
bash tools/diag_run.sh k_hess_w default hw1nt default hw1nt || exit 1
echo EXP10_DONE
