#!/bin/bash
# config #2 (batch 1) latency: diag/new (fewer launches) vs HEAD, two pairs
set -u
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
O=gpurun_out
b1() {  # tag env
  local tag=$1 ev=$2
  if [ "$ev" = "-" ]; then EV=(); else EV=($ev); fi
  env "${EV[@]}" timeout -k 10 120 python3 bench.py --batch 1 --steps 400 --warmup 20 --no-cpu > $O/y_$tag.json 2> $O/y_$tag.err || { tail -5 $O/y_$tag.err; return 1; }
  python3 -c "import json,sys;d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][0]);print(sys.argv[2], d['value'], d['ms_per_step'], d.get('stage_ms_per_step_serial'))" $O/y_$tag.json "$tag"
}
b1 n_a SURFHIP_LIB_DIR=cuda-surf_amd/diag/new || exit 1
b1 o_a - || exit 1
b1 n_b SURFHIP_LIB_DIR=cuda-surf_amd/diag/new || exit 1
b1 o_b - || exit 1
echo EXP26_DONE
