#!/bin/bash
# u2 (ring 4, WAR fix) vs ur: determinism, whole-step A/B, then the VERDICT measurements
set -u
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
O=gpurun_out
SURFHIP_DESC_U2=1 timeout -k 10 150 python3 -u tools/desc_determinism.py 3 16 > $O/e11_det.log 2>&1 || { tail -20 $O/e11_det.log; exit 1; }
grep -E "^run|^single" $O/e11_det.log
bench() {  # tag env args...
  local tag=$1 ev=$2; shift 2
  if [ "$ev" = "-" ]; then EV=(); else EV=($ev); fi
  env "${EV[@]}" timeout -k 10 120 python3 bench.py --steps 30 --warmup 3 --no-cpu "$@" > $O/x_$tag.json 2> $O/x_$tag.err || { tail -5 $O/x_$tag.err; return 1; }
  python3 -c "import json,sys;d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][0]);s=d['stage_ms_per_step_serial'];r=d['roofline'];print(sys.argv[2], d['value'], d['ms_per_step'], 'desc', s.get('describe'), 'hess_in', r['launch_ms'], 'hess_ser', r['launch_ms_serial'])" $O/x_$tag.json "$tag"
}
bench ab_ur1 - || exit 1
bench ab_u21 SURFHIP_DESC_U2=1 || exit 1
bench ab_ur2 - || exit 1
bench ab_u22 SURFHIP_DESC_U2=1 || exit 1
bash tools/r04_measure.sh || exit 1
echo EXP11_DONE
