set -u
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/e17_pytest.log 2>&1 || { tail -30 gpurun_out/e17_pytest.log; exit 1; }
tail -1 gpurun_out/e17_pytest.log
timeout -k 10 120 rocprofv3 --kernel-trace -T -f csv -d gpurun_out/kt_sort2 -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu --no-profile > gpurun_out/kt_sort2.json 2>&1 || exit 1
python3 tools/kstats.py gpurun_out/kt_sort2/run_kernel_trace.csv k_sort
