#!/bin/bash
# config #5 rotated describe occupancy: 2 / 3 (default) / 4 waves per SIMD; parity of the default
set -u
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
   -k "config5 or rotated or describe_u2 or batch256" > $O/e12_pytest.log 2>&1 || { tail -40 $O/e12_pytest.log; exit 1; }
tail -2 $O/e12_pytest.log
C5="--batch 64 --width 3840 --height 2160 --octaves 5 --upright 0 --extend 1"
bash tools/diag_run.sh k_describe default rotw2 rotw4 default -- $C5 || exit 1
echo EXP12_DONE
