set -u
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/e16_pytest.log 2>&1 || { tail -30 gpurun_out/e16_pytest.log; exit 1; }
tail -1 gpurun_out/e16_pytest.log
timeout -k 10 120 rocprofv3 --kernel-trace -T -f csv -d gpurun_out/kt_sort -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu --no-profile > gpurun_out/kt_sort.json 2>&1 || exit 1
python3 tools/kstats.py gpurun_out/kt_sort/run_kernel_trace.csv k_sort k_describe k_nms
timeout -k 10 120 python3 bench.py --steps 20 --warmup 3 --no-cpu --width 3840 --height 2160 --octaves 5 --upright 0 --extend 1 --batch 64 > gpurun_out/c5.json 2> gpurun_out/c5.err || { tail -5 gpurun_out/c5.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/c5.json'));print('config5', d['value'], d['ms_per_step'], d['stage_ms_per_step_serial'], d['roofline']['kernel'])"
