set -u
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/g13_pytest.log 2>&1 || { tail -30 gpurun_out/g13_pytest.log; exit 1; }
tail -1 gpurun_out/g13_pytest.log
timeout -k 10 300 python3 bench.py --no-cpu > gpurun_out/g13_bench.json 2> gpurun_out/g13_bench.err || { tail gpurun_out/g13_bench.err; exit 1; }
cat gpurun_out/g13_bench.json
