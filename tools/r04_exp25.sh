#!/bin/bash
# batch counters reset in one kernel on the side stream, queue zeroed by k_worklist, two-kernel item scan (diag/new) vs HEAD
set -u
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
O=gpurun_out
export SURFHIP_LIB_DIR=cuda-surf_amd/diag/new
timeout -k 10 300 python3 -u tools/desc_determinism.py 3 16 > $O/e25_det.log 2>&1 || { tail -20 $O/e25_det.log; exit 1; }
tail -4 $O/e25_det.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/e25_pytest.log 2>&1 || { tail -40 $O/e25_pytest.log; exit 1; }
tail -2 $O/e25_pytest.log
unset SURFHIP_LIB_DIR
bench() {  # tag env args...
  local tag=$1 ev=$2; shift 2
  if [ "$ev" = "-" ]; then EV=(); else EV=($ev); fi
  env "${EV[@]}" timeout -k 10 120 python3 bench.py --steps 30 --warmup 3 --no-cpu "$@" > $O/x_$tag.json 2> $O/x_$tag.err || { tail -5 $O/x_$tag.err; return 1; }
  python3 -c "import json,sys;d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][0]);s=d['stage_ms_per_step_serial'];r=d['roofline'];print(sys.argv[2], d['value'], d['ms_per_step'], 'desc', s.get('describe'), 'hess_in', r['launch_ms'], 'hess_ser', r['launch_ms_serial'])" $O/x_$tag.json "$tag"
}
bench r_new_a SURFHIP_LIB_DIR=cuda-surf_amd/diag/new || exit 1
bench r_old_a - || exit 1
bench r_new_b SURFHIP_LIB_DIR=cuda-surf_amd/diag/new || exit 1
bench r_old_b - || exit 1
echo EXP25_DONE
