#!/bin/bash
# integral fill: 2 rows loaded ahead (87 VGPRs, 5 waves per SIMD; diag/fa2) vs 4 (118 VGPRs, 4 waves)
set -u
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
O=gpurun_out
SURFHIP_LIB_DIR=cuda-surf_amd/diag/fa2 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
   -k "integral or config3 or golden or batch_next or wide" > $O/e35_pytest.log 2>&1 || { tail -40 $O/e35_pytest.log; exit 1; }
tail -2 $O/e35_pytest.log
bench() {  # tag env args...
  local tag=$1 ev=$2; shift 2
  if [ "$ev" = "-" ]; then EV=(); else EV=($ev); fi
  env "${EV[@]}" timeout -k 10 120 python3 bench.py --steps 30 --warmup 3 --no-cpu "$@" > $O/x_$tag.json 2> $O/x_$tag.err || { tail -5 $O/x_$tag.err; return 1; }
  python3 -c "import json,sys;d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][0]);s=d['stage_ms_per_step_serial'];r=d['roofline'];print(sys.argv[2], d['value'], d['ms_per_step'], 'integral', s.get('integral'), 'desc', s.get('describe'), 'hess_in', r['launch_ms'])" $O/x_$tag.json "$tag"
}
bench f_new_a SURFHIP_LIB_DIR=cuda-surf_amd/diag/fa2 || exit 1
bench f_old_a - || exit 1
bench f_new_b SURFHIP_LIB_DIR=cuda-surf_amd/diag/fa2 || exit 1
bench f_old_b - || exit 1
echo EXP35_DONE
