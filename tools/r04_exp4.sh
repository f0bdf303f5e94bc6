#!/bin/bash
# describe ring depth: parity subset, bench, then kernel time per ring size
set -u
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
   -k "config3 or detect_batch_next or golden or batch_equals or descriptor or describe or upright or doubled or max_pts or flat or 1080p" > $O/e4_pytest.log 2>&1 || { tail -40 $O/e4_pytest.log; exit 1; }
tail -2 $O/e4_pytest.log
bench() {  # tag env args...
  local tag=$1 ev=$2; shift 2
  if [ "$ev" = "-" ]; then EV=(); else EV=($ev); fi
  env "${EV[@]}" timeout -k 10 120 python3 bench.py --steps 30 --warmup 3 --no-cpu "$@" > $O/x_$tag.json 2> $O/x_$tag.err || { tail -5 $O/x_$tag.err; return 1; }
  python3 -c "import json,sys;d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][0]);s=d['stage_ms_per_step_serial'];r=d['roofline'];print(sys.argv[2], d['value'], d['ms_per_step'], 'desc', s.get('describe'), 'hess_in', r['launch_ms'], 'hess_ser', r['launch_ms_serial'])" $O/x_$tag.json "$tag"
}
bench e4_pipe - || exit 1
bench e4_ring4 SURFHIP_LIB_DIR=cuda-surf_amd/diag/ring4 || exit 1
bash tools/diag_run.sh k_describe default ring4 ring8 norows || exit 1
echo EXP4_DONE
