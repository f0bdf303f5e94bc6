#!/bin/bash
# describe u2: row spans 33-64 chunks on the LDS ring (default) vs the sparse path (segw32)
set -u
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
O=gpurun_out
bench() {  # tag env args...
  local tag=$1 ev=$2; shift 2
  if [ "$ev" = "-" ]; then EV=(); else EV=($ev); fi
  env "${EV[@]}" timeout -k 10 120 python3 bench.py --steps 30 --warmup 3 --no-cpu "$@" > $O/x_$tag.json 2> $O/x_$tag.err || { tail -5 $O/x_$tag.err; return 1; }
  python3 -c "import json,sys;d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][0]);s=d['stage_ms_per_step_serial'];r=d['roofline'];print(sys.argv[2], d['value'], d['ms_per_step'], 'desc', s.get('describe'), 'hess_in', r['launch_ms'], 'hess_ser', r['launch_ms_serial'])" $O/x_$tag.json "$tag"
}
bench w64a - || exit 1
bench w32a SURFHIP_LIB_DIR=cuda-surf_amd/diag/segw32 || exit 1
bench w64b - || exit 1
bench w32b SURFHIP_LIB_DIR=cuda-surf_amd/diag/segw32 || exit 1
bash tools/diag_run.sh k_describe default segw32 default segw32 || exit 1
echo EXP14_DONE
