#!/bin/bash
# describe u2: DMA lanes past the span and sparse-path loads masked off instead of out of bounds (diag/mask) vs default
set -u
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
O=gpurun_out
export SURFHIP_LIB_DIR=cuda-surf_amd/diag/mask
timeout -k 10 300 python3 -u tools/desc_determinism.py 3 16 > $O/e32_det.log 2>&1 || { tail -20 $O/e32_det.log; exit 1; }
tail -4 $O/e32_det.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
   -k "config3 or golden or batch_equals or descriptor or describe or upright or doubled or max_pts or flat or 1080p or surfor or match" > $O/e32_pytest.log 2>&1 || { tail -40 $O/e32_pytest.log; exit 1; }
tail -2 $O/e32_pytest.log
unset SURFHIP_LIB_DIR
bench() {  # tag env args...
  local tag=$1 ev=$2; shift 2
  if [ "$ev" = "-" ]; then EV=(); else EV=($ev); fi
  env "${EV[@]}" timeout -k 10 120 python3 bench.py --steps 30 --warmup 3 --no-cpu "$@" > $O/x_$tag.json 2> $O/x_$tag.err || { tail -5 $O/x_$tag.err; return 1; }
  python3 -c "import json,sys;d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][0]);s=d['stage_ms_per_step_serial'];r=d['roofline'];print(sys.argv[2], d['value'], d['ms_per_step'], 'desc', s.get('describe'), 'hess_in', r['launch_ms'], 'hess_ser', r['launch_ms_serial'])" $O/x_$tag.json "$tag"
}
bench n_new_a SURFHIP_LIB_DIR=cuda-surf_amd/diag/mask || exit 1
bench n_old_a - || exit 1
bench n_new_b SURFHIP_LIB_DIR=cuda-surf_amd/diag/mask || exit 1
bench n_old_b - || exit 1
echo EXP32_DONE
