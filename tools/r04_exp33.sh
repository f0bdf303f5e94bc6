#!/bin/bash
# config #5: orientation with two samples per pass, both gathers in flight (diag/ori2) vs HEAD
set -u
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
O=gpurun_out
SURFHIP_LIB_DIR=cuda-surf_amd/diag/ori2 timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/e33_pytest.log 2>&1 || { tail -40 $O/e33_pytest.log; exit 1; }
tail -2 $O/e33_pytest.log
C5="--batch 64 --width 3840 --height 2160 --octaves 5 --upright 0 --extend 1"
b5() {  # tag env
  local tag=$1 ev=$2
  if [ "$ev" = "-" ]; then EV=(); else EV=($ev); fi
  env "${EV[@]}" timeout -k 10 300 python3 bench.py --steps 10 --warmup 2 --no-cpu $C5 > $O/z_$tag.json 2> $O/z_$tag.err || { tail -5 $O/z_$tag.err; return 1; }
  python3 -c "import json,sys;d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][0]);print(sys.argv[2], d['value'], d['ms_per_step'], d.get('stage_ms_per_step_serial'))" $O/z_$tag.json "$tag"
}
b5 o_new_a SURFHIP_LIB_DIR=cuda-surf_amd/diag/ori2 || exit 1
b5 o_old_a - || exit 1
b5 o_new_b SURFHIP_LIB_DIR=cuda-surf_amd/diag/ori2 || exit 1
b5 o_old_b - || exit 1
echo EXP33_DONE
