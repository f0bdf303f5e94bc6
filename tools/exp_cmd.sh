set -u
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/e22_pytest.log 2>&1 || { tail -30 gpurun_out/e22_pytest.log; exit 1; }
tail -1 gpurun_out/e22_pytest.log
timeout -k 10 200 python3 bench.py --batch 1 --steps 200 --warmup 10 --no-cpu > gpurun_out/c2.json 2> gpurun_out/c2.err || { tail -5 gpurun_out/c2.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/c2.json'));print('config2', d['value'], d['ms_per_step'], d['stage_ms_per_step_serial'])"
timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-cpu > gpurun_out/c3.json 2> gpurun_out/c3.err || { tail -5 gpurun_out/c3.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/c3.json'));print('config3', d['value'], d['ms_per_step'], d['stage_ms_per_step_serial'])"
