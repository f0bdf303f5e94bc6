#!/bin/bash
# next batch's band sums beside this batch's Hessian, only the fill beside NMS
# (diag/split with SURFHIP_PREFETCH=split) vs HEAD
set -u
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
O=gpurun_out
SURFHIP_LIB_DIR=cuda-surf_amd/diag/split SURFHIP_PREFETCH=split timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
   -k "batch_next or config3 or golden or batch_equals" > $O/e29_pytest.log 2>&1 || { tail -40 $O/e29_pytest.log; exit 1; }
tail -2 $O/e29_pytest.log
bench() {  # tag env args...
  local tag=$1 ev=$2; shift 2
  if [ "$ev" = "-" ]; then EV=(); else EV=($ev); fi
  env "${EV[@]}" timeout -k 10 120 python3 bench.py --steps 30 --warmup 3 --no-cpu "$@" > $O/x_$tag.json 2> $O/x_$tag.err || { tail -5 $O/x_$tag.err; return 1; }
  python3 -c "import json,sys;d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][0]);s=d['stage_ms_per_step_serial'];r=d['roofline'];print(sys.argv[2], d['value'], d['ms_per_step'], 'desc', s.get('describe'), 'hess_in', r['launch_ms'], 'hess_ser', r['launch_ms_serial'])" $O/x_$tag.json "$tag"
}
SP="SURFHIP_LIB_DIR=cuda-surf_amd/diag/split SURFHIP_PREFETCH=split"
bench p_new_a "$SP" || exit 1
bench p_old_a - || exit 1
bench p_new_b "$SP" || exit 1
bench p_old_b - || exit 1
echo EXP29_DONE
