#!/bin/bash
# describe u2: how much do the row reads' LDS bank conflicts cost?  diag/noconf
# reads lane-contiguous words (conflict-free, wrong values) -- timing only
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
bench c_diag_a SURFHIP_LIB_DIR=cuda-surf_amd/diag/noconf || exit 1
bench c_def_a - || exit 1
bench c_diag_b SURFHIP_LIB_DIR=cuda-surf_amd/diag/noconf || exit 1
bench c_def_b - || exit 1
SURFHIP_LIB_DIR=cuda-surf_amd/diag/noconf bash tools/pmc_kern.sh u2nc k_describe_u2 "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_WAIT_ANY SQ_BUSY_CYCLES" || exit 1
echo EXP24_DONE
