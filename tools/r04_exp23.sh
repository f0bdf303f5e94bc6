#!/bin/bash
# describe u2: LDS counters of the default build (bank conflicts vs LDS-active cycles)
set -u
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
bash tools/pmc_kern.sh u2lds k_describe_u2 "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES" "SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_WAVES" > gpurun_out/e23_pmc.txt 2>&1 || { tail -20 gpurun_out/e23_pmc.txt; exit 1; }
cat gpurun_out/e23_pmc.txt
echo EXP23_DONE
