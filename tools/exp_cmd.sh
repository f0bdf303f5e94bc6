set -u
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "hessian_alternate or hessian_planes" > gpurun_out/e0_pytest.log 2>&1 || { tail -30 gpurun_out/e0_pytest.log; exit 1; }
tail -1 gpurun_out/e0_pytest.log
SURFHIP_LIB_DIR=cuda-surf_amd/diag/strip512 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "hessian_alternate and O0_RING" > gpurun_out/e1_pytest.log 2>&1 || { tail -30 gpurun_out/e1_pytest.log; exit 1; }
tail -1 gpurun_out/e1_pytest.log
bash tools/diag_run.sh k_hess default strip512 -- --hessian-only
SURFHIP_Q1=0 bash tools/diag_run.sh k_hess default -- --hessian-only
