#!/bin/bash
# describe u2 breakdown: SQ counters of the default build, and diag builds without rows / reduction / non-seg keypoints
set -u
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
bash tools/pmc_kern.sh u2sq k_describe_u2 "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU" "SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VALU_CVT SQ_BUSY_CYCLES" || exit 1
bash tools/diag_run.sh k_describe default norows nored onlyseg || exit 1
echo EXP15_DONE
