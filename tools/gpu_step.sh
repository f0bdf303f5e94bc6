set -u
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "hessian or 1080p" > gpurun_out/g19_pytest.log 2>&1 || { tail -30 gpurun_out/g19_pytest.log; exit 1; }
tail -1 gpurun_out/g19_pytest.log
for dg in 0 1; do
SURFHIP_FAR_DIAG=$dg bash tools/ktrace.sh fd$dg --hessian-only | grep hess_far || exit 1
echo "-- far diag $dg"
done
