set -u
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/e15_pytest.log 2>&1 || { tail -30 gpurun_out/e15_pytest.log; exit 1; }
tail -1 gpurun_out/e15_pytest.log
for c in 1 0 1 0; do
SURFHIP_FIT_CUBE=$c timeout -k 10 120 rocprofv3 --kernel-trace -T -f csv -d gpurun_out/kt_cube$c -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu --no-profile > gpurun_out/kt_cube$c.json 2>&1 || exit 1
echo cube $c; python3 tools/kstats.py gpurun_out/kt_cube$c/run_kernel_trace.csv k_nms
done
