set -u
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "hessian" > gpurun_out/e9_pytest.log 2>&1 || { tail -30 gpurun_out/e9_pytest.log; exit 1; }
tail -1 gpurun_out/e9_pytest.log
for c in 1 0 1 0; do
SURFHIP_Q01=$c timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-cpu --hessian-only > gpurun_out/hq_$c.json 2> gpurun_out/hq_$c.err || { tail -5 gpurun_out/hq_$c.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/hq_$c.json'));print('q01 $c', d['roofline']['launch_ms'], d['roofline']['frac'], d['roofline']['kernel'])"
done
