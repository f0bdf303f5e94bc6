set -u
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
SURFHIP_LIB_DIR=cuda-surf_amd/diag/nt timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "integral" > gpurun_out/e24_pytest.log 2>&1 || { tail -30 gpurun_out/e24_pytest.log; exit 1; }
tail -1 gpurun_out/e24_pytest.log
for v in default nt default nt; do
LD=cuda-surf_amd/diag/$v; [ "$v" = default ] && LD=cuda-surf_amd
SURFHIP_LIB_DIR=$LD timeout -k 10 120 rocprofv3 --kernel-trace -T -f csv -d gpurun_out/nt_$v -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu > gpurun_out/nt_$v.json 2>&1 || exit 1
echo $v; python3 tools/kstats.py gpurun_out/nt_$v/run_kernel_trace.csv k_ii k_hess_far k_describe
python3 -c "import json;d=json.loads(open('gpurun_out/nt_$v.json').read().strip().split(chr(10))[-1]);print('value', d['value'], d['stage_ms_per_step_serial'])"
done
