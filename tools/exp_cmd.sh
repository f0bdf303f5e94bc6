set -u
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q --timeout 120 --timeout-method thread -k "hessian or config" > gpurun_out/e25_pytest.log 2>&1 || { tail -30 gpurun_out/e25_pytest.log; exit 1; }
tail -1 gpurun_out/e25_pytest.log
bash tools/diag_run.sh k_hess_far default prev default prev -- --hessian-only > /dev/null
for v in default prev; do echo $v; python3 tools/kstats.py gpurun_out/dg_$v/run_kernel_trace.csv k_hess_far; done
