set -u
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/g23_pytest.log 2>&1 || { tail -30 gpurun_out/g23_pytest.log; exit 1; }
tail -1 gpurun_out/g23_pytest.log
