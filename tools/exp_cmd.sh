set -u
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
SURFHIP_Q1=1 timeout -k 10 120 python -u tools/dbg_planes.py 1920 1080 4 7 || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "hessian" > gpurun_out/e3_pytest.log 2>&1 || { tail -30 gpurun_out/e3_pytest.log; exit 1; }
tail -1 gpurun_out/e3_pytest.log
