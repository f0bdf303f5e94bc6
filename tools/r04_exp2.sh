#!/bin/bash
# describe v2 check: parity subset, then step A/B and per-kernel diag timings
set -u
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
   -k "descriptor or upright or config3 or detect_batch_next or dropin or golden or describe" > $O/e2_pytest.log 2>&1 || { tail -40 $O/e2_pytest.log; exit 1; }
tail -2 $O/e2_pytest.log
bench() {  # tag env args...
  local tag=$1 ev=$2; shift 2
  if [ "$ev" = "-" ]; then EV=(); else EV=($ev); fi
  env "${EV[@]}" timeout -k 10 120 python3 bench.py --steps 30 --warmup 3 --no-cpu "$@" > $O/x_$tag.json 2> $O/x_$tag.err || { tail -5 $O/x_$tag.err; return 1; }
  python3 -c "import json,sys;d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][0]);s=d['stage_ms_per_step_serial'];r=d['roofline'];print(sys.argv[2], d['value'], d['ms_per_step'], 'desc', s.get('describe'), 'hess_in', r['launch_ms'], 'hess_ser', r['launch_ms_serial'])" $O/x_$tag.json "$tag"
}
bench e2_pipe - || exit 1
bench e2_p0g4 SURFHIP_P0=94 --no-pipeline || exit 1
bench e2_nopipe - --no-pipeline || exit 1
bash tools/diag_run.sh k_describe default norows nosmp onlyseg -- --no-pipeline || exit 1
echo EXP2_DONE
