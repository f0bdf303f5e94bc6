#!/bin/bash
# describe u2 time split on the current build: without rows / reduction reads / sample arithmetic (diag builds, wrong values)
set -u
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
O=gpurun_out
bench() {  # tag env
  local tag=$1 ev=$2; shift 2
  if [ "$ev" = "-" ]; then EV=(); else EV=($ev); fi
  env "${EV[@]}" timeout -k 10 120 python3 bench.py --steps 20 --warmup 3 --no-cpu "$@" > $O/x_$tag.json 2> $O/x_$tag.err || { tail -5 $O/x_$tag.err; return 1; }
  python3 -c "import json,sys;d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][0]);s=d['stage_ms_per_step_serial'];print(sys.argv[2], d['ms_per_step'], 'desc', s.get('describe'))" $O/x_$tag.json "$tag"
}
bench d_default - || exit 1
bench d_norows SURFHIP_LIB_DIR=cuda-surf_amd/diag/norows || exit 1
bench d_nored SURFHIP_LIB_DIR=cuda-surf_amd/diag/nored || exit 1
bench d_nosmp SURFHIP_LIB_DIR=cuda-surf_amd/diag/nosmp || exit 1
echo EXP30_DONE
