#!/bin/bash
# Round-4 describe / pipelining experiments (each step time-limited).
set -u
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
O=gpurun_out
timeout -s KILL 60 rocprofv3 -L > $O/r04_counters.txt 2>&1 || true
bench() {  # tag env args...
  local tag=$1 ev=$2; shift 2
  if [ "$ev" = "-" ]; then EV=(); else EV=($ev); fi
  env "${EV[@]}" timeout -k 10 120 python3 bench.py --steps 30 --warmup 3 --no-cpu "$@" > $O/x_$tag.json 2> $O/x_$tag.err || { tail -5 $O/x_$tag.err; return 1; }
  python3 -c "import json,sys;d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][0]);s=d['stage_ms_per_step_serial'];r=d['roofline'];print(sys.argv[2], d['value'], d['ms_per_step'], 'desc', s.get('describe'), 'hess_in', r['launch_ms'], 'hess_ser', r['launch_ms_serial'])" $O/x_$tag.json "$tag"
}
bench pipe3 - || exit 1
bench pipe4 SURFHIP_DESC_BESIDE=4 || exit 1
bench pipe2 SURFHIP_DESC_BESIDE=2 || exit 1
bench nopipe - --no-pipeline || exit 1
bench old_pipe3 SURFHIP_DESC_UR=1 || exit 1
bench old_nopipe SURFHIP_DESC_UR=1 --no-pipeline || exit 1
bash tools/diag_run.sh k_describe default norows nosmp nored -- --no-pipeline || exit 1
bash tools/pmc_kern.sh u2 k_describe "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" "SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM" -- --no-pipeline || exit 1
echo EXP1_DONE
