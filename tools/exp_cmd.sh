set -u
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
bash tools/diag_run.sh k_hess_far default r8 noacc noload -- --hessian-only
for v in default r8 noacc noload; do echo $v; python3 tools/kstats.py gpurun_out/dg_$v/run_kernel_trace.csv k_hess_far; done
bash tools/pmc_kern.sh sqf k_hess_far "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU" -- --hessian-only
